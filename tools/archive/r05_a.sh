# Round 5, first GPU pass: the capacity / recovery / fill-holes changes and the tests around
# them, the default bench, the steady-state plate CLI run and the host decode budget.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05a
mkdir -p $O
cd $R
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_capacity.py tests/test_gpu_seg.py tests/test_gpu_flowerr_reg.py > $O/t1.log 2>&1
timeout -k 10 600 $T tests/test_gpu_recovery.py tests/test_gpu_watershed.py tests/test_gpu_e2e.py > $O/t2.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
timeout -k 10 400 python -u tools/plate_bench.py --fovs 192 --repeat 4 --dir /tmp > $O/plate.log 2>&1
timeout -k 10 200 python -u tools/decode_budget.py --pools 1 8 --threads 16 --seconds 8 --dir /tmp > $O/decode.log 2>&1
echo done
