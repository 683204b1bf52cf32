# Development GPU pass: certified fp32 screening of the flow-error filter — parity, counts, bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/screen
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_e2e.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
CPX_FE_DEBUG=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 4 --warmup 1 --pipes 1 > $O/bench_debug.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 12 > $O/bench.log 2>&1
echo done
