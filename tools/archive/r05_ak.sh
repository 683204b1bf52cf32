# Round 5: the bench with 8 hardware queues per process (GPU_MAX_HW_QUEUES=8: r05aj showed the
# plate CLI's five streams sharing the default 4 queues, its pipelines serialised), and three
# pipelines with 8 queues (three pipelines measured slower on 4 queues in round 4).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ak
mkdir -p $O
cd $R
run() {
  timeout -k 10 300 env $1 python -u bench.py --no-cpu-baseline --steps 60 --stage-steps 1 $2 > $O/b.log 2>&1
  tail -1 $O/b.log | tee -a $O/bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$1 $2', d['value'], d['ms_per_step'])"
}
run "GPU_MAX_HW_QUEUES=4" ""
run "GPU_MAX_HW_QUEUES=8" ""
run "GPU_MAX_HW_QUEUES=8" "--pipes 3"
run "GPU_MAX_HW_QUEUES=4" ""
run "GPU_MAX_HW_QUEUES=8" ""
run "GPU_MAX_HW_QUEUES=8" "--pipes 3"
echo done
