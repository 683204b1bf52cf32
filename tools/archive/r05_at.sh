# Round 5: (development) CU-split pipelines (contiguous halves) without the stage exclusivity
# (each pipeline has its own CUs, so two CPnets / feature stages no longer compete), and three
# pipelines in thirds, against the default.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05at
mkdir -p $O
cd $R
run() {
  timeout -k 10 300 env $1 python -u bench.py --no-cpu-baseline --steps 40 --stage-steps 1 $2 > $O/b.log 2>&1
  tail -1 $O/b.log | tee -a $O/bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$1 $2', d['value'], d['ms_per_step'])"
}
for i in 1 2; do
  run "CPX_NOP=1" ""
  run "CPX_STAGE_EXCLUSIVE=" "--cu-split halves"
  run "CPX_NOP=1" "--cu-split halves"
  run "CPX_STAGE_EXCLUSIVE=" "--cu-split halves --pipes 3"
done
echo done
