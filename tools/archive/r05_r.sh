# Round 5: the bench line with the new GLCM LDS roofline entry (roofline_all.glcm) and libcpx's
# GLCM launch timing; the feature tests.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05r
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_features_pair.py tests/test_gpu_parity.py > $O/t.log 2>&1
echo done
