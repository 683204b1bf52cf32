# Hardware queues per process vs pipelines per GPU (GPU_MAX_HW_QUEUES, the box default 4).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04ac
mkdir -p $O
cd $R
for cfg in "4 2" "8 2" "8 3" "4 2"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 16 --pipes $2 > $O/b_q$1_p$2.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('$O/b_q$1_p$2.log').read().strip().splitlines()[-1]); print('queues $1 pipes $2', d['value'])"
done
