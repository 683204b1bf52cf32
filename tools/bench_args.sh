#!/bin/bash
# Development: bench.py lines for several argument sets (each quoted), e.g.
#   bash tools/bench_args.sh "--pipes 1" "--pipes 2" "--pipes 1 --batch 48"
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/args
mkdir -p $O
cd $R
: > $O/summary.txt
i=0
for args in "$@"; do
  i=$((i + 1))
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps ${STEPS:-16} $args > $O/run_$i.log 2>&1
  echo "[$args] $(tail -1 $O/run_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["stage_ms_per_step"])')" >> $O/summary.txt
done
echo done
