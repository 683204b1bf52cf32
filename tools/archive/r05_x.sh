# Round 5: batches in flight / batch size with the stage exclusivity (CPnet, features): 2 x 48
# (default) vs 3 x 32, 3 x 48, 2 x 64, 4 x 32 on the two-pipeline bench (60 steps' worth).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05x
mkdir -p $O
cd $R
run() {  # name, args
  name=$1; shift
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --stage-steps 1 "$@" > $O/bench_$name.log 2>&1
  tail -1 $O/bench_$name.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$name',d['value'],d['ms_per_step'])"
}
run p2b48 --pipes 2 --batch 48 --steps 60
run p3b32 --pipes 3 --batch 32 --steps 90
run p3b48 --pipes 3 --batch 48 --steps 60
run p2b64 --pipes 2 --batch 64 --steps 45
run p4b32 --pipes 4 --batch 32 --steps 90
run p2b48b --pipes 2 --batch 48 --steps 60
echo done
