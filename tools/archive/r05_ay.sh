# Round 5: the two-stream equality test with plain and CU-masked pipeline streams.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ay
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_streams.py > $O/t.log 2>&1
grep -E "PASS|FAIL|passed|failed" $O/t.log | tail -4
echo done
