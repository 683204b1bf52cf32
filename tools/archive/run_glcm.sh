# Development GPU pass (via gpurun): parity tests of the touched kernels, GLCM A/B (returning-atomic
# count vs table scan), watershed timing + heap-oracle check, CPnet pair A/B, bench lines.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/glcm
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_cpnet_x3.py tests/test_gpu_parity.py tests/test_gpu_fov.py tests/test_gpu_seg.py tests/test_gpu_watershed.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for v in glcm_v1prof glcm_v2prof; do
  CPX_LIB=$R/tools/_var/libcpx_$v.so timeout -k 10 200 python -u tools/tex_bench.py --batch 16 > $O/tex_$v.log 2>&1
done
timeout -k 10 200 python -u tools/tex_bench.py --batch 16 > $O/tex_default.log 2>&1
CPX_LIB=$R/tools/_var/libcpx_glcm_v1.so timeout -k 10 200 python -u tools/tex_bench.py --batch 16 > $O/tex_v1.log 2>&1
timeout -k 10 200 python -u tools/ws_bench.py --check > $O/ws.log 2>&1
timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 12 > $O/bench.log 2>&1
CPX_X3_PAIR=0 timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 12 > $O/bench_nopair.log 2>&1
echo done
