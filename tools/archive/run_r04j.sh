# Convolution residency vs the other pipeline (CPX_X3_LDS_PAD: unused LDS per conv block).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04j
mkdir -p $O
cd $R
for pad in 0 16384 0 16384; do
  CPX_X3_LDS_PAD=$pad timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 16 > $O/b_$pad.log 2>&1
  python -c "import json; d=json.loads(open('$O/b_$pad.log').read().strip().splitlines()[-1]); print('pad $pad', d['value'], d['stage_ms_per_step']['cpnet'])"
done
echo done
