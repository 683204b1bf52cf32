# Flow-following round schedule A/B (CPX_FOLLOW_K0 / _SWITCH / _K1): seg_post stage time of the
# instrumented bench steps and the headline value; the dynamics' output does not depend on it.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04h
mkdir -p $O
cd $R
for cfg in "16 384 128" "32 384 128" "8 256 128" "16 192 64" "16 768 128" "32 512 256"; do
  set -- $cfg
  CPX_FOLLOW_K0=$1 CPX_FOLLOW_SWITCH=$2 CPX_FOLLOW_K1=$3 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 12 --stage-steps 3 > $O/b_$1_$2_$3.log 2>&1
  python -c "import json; d=json.loads(open('$O/b_$1_$2_$3.log').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['stage_ms_per_step']['seg_post'])"
done
echo done
