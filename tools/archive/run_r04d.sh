# Batch-size / pipelines sweep of the headline bench (same workload: FOV/s of the whole pipe).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04d
mkdir -p $O
cd $R
for cfg in "48 2" "96 2" "64 2" "32 3"; do
  set -- $cfg
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --batch $1 --pipes $2 --steps 16 --pool 4 > $O/bench_b$1_p$2.log 2>&1
  python -c "import json,sys; d=json.loads(open('$O/bench_b$1_p$2.log').read().strip().splitlines()[-1]); print('batch $1 pipes $2', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
done
echo done
