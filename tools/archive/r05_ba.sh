# Round 5: plate tests after the plate's stream default went back to unrestricted CUs.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ba
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_plate.py tests/test_gpu_config3_jobs.py tests/test_gpu_config2_full.py > $O/t.log 2>&1
tail -1 $O/t.log
timeout -k 10 400 python -u tools/plate_bench.py --fovs 192 --repeat 8 --dir /tmp > $O/pb.log 2>&1
tail -1 $O/pb.log | tee -a $O/plate_bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('plate', d['value'], d['value_excluding_csv'])"
echo done
