# Round 5: stage-exclusivity sets with the CU-split pipelines (default cpnet,features).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05av
mkdir -p $O
cd $R
for i in 1 2; do
for ex in "cpnet,features" "cpnet" "cpnet,features,seg_post" "cpnet,features,cells"; do
  timeout -k 10 300 env CPX_STAGE_EXCLUSIVE=$ex python -u bench.py --no-cpu-baseline --steps 40 --stage-steps 1 > $O/b.log 2>&1
  tail -1 $O/b.log | tee -a $O/bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$ex', d['value'], d['ms_per_step'])"
done
done
echo done
