# p32 without spills vs with (tools/_var/libcpx_p32spill.so = the previous k_conv_x3), parity.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04g
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_cpnet_x3.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
timeout -k 10 200 python -u tools/conv_bench_x3.py --tiles 432 --reps 5 --variants 0 > $O/conv_new$i.log 2>&1
CPX_LIB=$R/tools/_var/libcpx_p32spill.so timeout -k 10 200 python -u tools/conv_bench_x3.py --tiles 432 --reps 5 --variants 0 > $O/conv_old$i.log 2>&1
done
echo done
