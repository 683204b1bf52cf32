# Round 5: cpx.plate / plate_bench now raise GPU_MAX_HW_QUEUES from the box's exported 4 to 8
# (r05an: a setdefault kept the box's 4): plate tests and the plate bench at 768 / 1536 FOVs.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ao
mkdir -p $O
cd $R
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_plate.py tests/test_gpu_config3_jobs.py > $O/t_plate.log 2>&1
tail -1 $O/t_plate.log
for args in "--fovs 192 --repeat 4" "--fovs 192 --repeat 8" "--fovs 192 --repeat 8"; do
  timeout -k 10 400 python -u tools/plate_bench.py $args --dir /tmp > $O/pb.log 2>&1
  tail -1 $O/pb.log | tee -a $O/plate_bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$args', d['value'], d['value_excluding_csv'])"
done
timeout -k 10 400 env CPX_PLATE_HW_QUEUES=4 python -u tools/plate_bench.py --fovs 192 --repeat 8 --dir /tmp > $O/pb.log 2>&1
tail -1 $O/pb.log | tee -a $O/plate_bench_q4.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('q4 1536', d['value'], d['value_excluding_csv'])"
echo done
