# Round 5, first GPU pass: the capacity / recovery / fill-holes changes and the tests around
# them, the conv variant A/B, the default bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05a
mkdir -p $O
cd $R
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
timeout -k 10 300 python -u tools/conv_bench_x3.py --tiles 144 --variants 0 2 > $O/conv.log 2>&1
timeout -k 10 600 $T tests/test_gpu_capacity.py tests/test_gpu_seg.py tests/test_gpu_flowerr_reg.py > $O/t1.log 2>&1
timeout -k 10 600 $T tests/test_gpu_recovery.py tests/test_gpu_watershed.py tests/test_gpu_e2e.py > $O/t2.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
echo done
