# Development GPU pass: watershed parity (tests + heap-oracle check) and timing A/B against the
# previous library (tools/_var/libcpx_old.so).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ws2
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_watershed.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
CPX_LIB=$R/tools/_var/libcpx_old.so timeout -k 10 200 python -u tools/ws_bench.py > $O/ws_old.log 2>&1
timeout -k 10 200 python -u tools/ws_bench.py --check > $O/ws_new.log 2>&1
CPX_LIB=$R/tools/_var/libcpx_old.so timeout -k 10 200 python -u tools/ws_bench.py > $O/ws_old2.log 2>&1
timeout -k 10 200 python -u tools/ws_bench.py > $O/ws_new2.log 2>&1
echo done
