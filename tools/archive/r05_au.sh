# Round 5: the CU-split pipeline streams as the default (cpx.device.pipeline_streams): plate and
# stream tests, smoke, the bench (default and --cu-split none) and the plate bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05au
mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_plate.py tests/test_gpu_config3_jobs.py tests/test_gpu_streams.py > $O/t.log 2>&1
tail -1 $O/t.log
for cs in auto none auto none; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 --stage-steps 1 --cu-split $cs > $O/b.log 2>&1
  tail -1 $O/b.log | tee -a $O/bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cs', d['value'], d['ms_per_step'])"
done
timeout -k 10 400 python -u tools/plate_bench.py --fovs 192 --repeat 8 --dir /tmp > $O/pb.log 2>&1
tail -1 $O/pb.log | tee -a $O/plate_bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('plate', d['value'], d['value_excluding_csv'])"
timeout -k 10 400 env CPX_CU_SPLIT=none python -u tools/plate_bench.py --fovs 192 --repeat 8 --dir /tmp > $O/pb.log 2>&1
tail -1 $O/pb.log | tee -a $O/plate_bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('plate none', d['value'], d['value_excluding_csv'])"
echo done
