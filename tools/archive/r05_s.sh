# Round 5: cross-pipeline stage exclusivity (CPX_STAGE_EXCLUSIVE) A/B on the default bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05s
mkdir -p $O
cd $R
for v in none cpnet cpnet,features features cpnet,seg_post,features none2; do
  e=$v; [ "$v" = none ] || [ "$v" = none2 ] && e=""
  timeout -k 10 300 env CPX_STAGE_EXCLUSIVE=$e python -u bench.py --no-cpu-baseline > $O/bench_$v.log 2>&1
  tail -1 $O/bench_$v.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$v',d['value'],d['ms_per_step'])"
done
echo done
