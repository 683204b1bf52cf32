#!/bin/bash
# Development A/B of the whole bench line: the in-tree libcpx vs tools/_var variants named on the
# command line, alternating runs (bench.py --no-cpu-baseline).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab
mkdir -p $O
cd $R
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps ${STEPS:-16} > $O/default_$rep.log 2>&1
  for v in "$@"; do
    CPX_LIB=$R/tools/_var/libcpx_$v.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps ${STEPS:-16} > $O/${v}_$rep.log 2>&1
  done
done
for f in $O/*.log; do
  echo "$(basename $f) $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["stage_ms_per_step"])')"
done > $O/summary.txt
echo done
