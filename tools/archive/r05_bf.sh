# Round 5: smoke + a few GPU tests on the rebuilt final library (after reverting r05be).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05bf
mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cpnet_x3.py tests/test_gpu_streams.py tests/test_gpu_e2e.py > $O/t.log 2>&1
tail -1 $O/t.log
echo done
