# The register flow-error class test on the GPU.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04w
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_flowerr_reg.py -x -v -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -4 $O/tests.log
