# Residual-prefetch epilogue: parity (x3 kernels, whole forward, e2e IDs) + conv A/B vs the
# previous epilogue (tools/_var/libcpx_prevepi.so) + bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04i
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_cpnet_x3.py tests/test_gpu_e2e.py -x -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
timeout -k 10 200 python -u tools/conv_bench_x3.py --tiles 432 --reps 5 --variants 0 > $O/conv_new$i.log 2>&1
CPX_LIB=$R/tools/_var/libcpx_prevepi.so timeout -k 10 200 python -u tools/conv_bench_x3.py --tiles 432 --reps 5 --variants 0 > $O/conv_old$i.log 2>&1
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
echo done
