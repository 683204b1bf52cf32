# Development GPU pass: parity of the touched kernels (expand_labels / watershed / features),
# then feature-stage and watershed timing A/B of old vs new vs the bank-swizzle variant.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/glcm3
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_watershed.py tests/test_gpu_fov.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
CPX_LIB=$R/tools/_var/libcpx_gswzp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "feature or texture or glcm" > $O/tests_swz.log 2>&1
for v in old gswzp gscanprof gprof; do
  CPX_LIB=$R/tools/_var/libcpx_$v.so timeout -k 10 200 python -u tools/tex_bench.py --batch 16 > $O/tex_$v.log 2>&1
done
timeout -k 10 200 python -u tools/tex_bench.py --batch 16 > $O/tex_new.log 2>&1
CPX_LIB=$R/tools/_var/libcpx_old.so timeout -k 10 200 python -u tools/ws_bench.py > $O/ws_old.log 2>&1
timeout -k 10 200 python -u tools/ws_bench.py --check > $O/ws_new.log 2>&1
echo done
