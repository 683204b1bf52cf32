# Round 5: r05am again with GPU_MAX_HW_QUEUES set before torch loads HIP (plate_bench):
# its GPU tests, the I/O-inclusive plate bench at 768 and 1536 FOVs, and its kernel overlap.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05am
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_plate.py tests/test_gpu_config3_jobs.py > $O/t_plate.log 2>&1
tail -2 $O/t_plate.log
for args in "--fovs 192 --repeat 4" "--fovs 192 --repeat 8"; do
  timeout -k 10 400 python -u tools/plate_bench.py $args --dir /tmp > $O/pb.log 2>&1
  tail -1 $O/pb.log | tee -a $O/plate_bench.jsonl
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/pt -o run -- \
  python -u tools/plate_bench.py --fovs 96 --repeat 4 --dir /tmp > $O/pt.log 2>&1
S=$(grep '^{"metric"' $O/pt.log | python -c "import json,sys;print(json.loads(sys.stdin.read())['seconds'])")
python tools/plate_overlap.py /tmp/pt/run_kernel_trace.csv --seconds $S | tee $O/overlap.txt
rm -rf /tmp/pt
echo done
