# Final state of the register flow-error classes (1-3; the four-wave class dropped): class test
# and seg parity.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04ab
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_flowerr_reg.py tests/test_gpu_seg.py tests/test_gpu_e2e.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
