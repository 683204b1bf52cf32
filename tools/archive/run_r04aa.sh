# Class 4 of the register flow-error screening (column pairs over 4 waves, rows <= 160): class
# test + seg / e2e parity, bench, kernel trace.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04aa
mkdir -p $O
cd $R
timeout -k 10 200 python -u -m pytest tests/test_gpu_flowerr_reg.py -x -v -s --timeout 150 --timeout-method thread > $O/class.log 2>&1
grep -E "masks per class|passed|failed" $O/class.log
RUN_TAG=r04aa bash tools/run_r04l.sh
