# Round 5: Cells + Cytoplasm features in one pass (cpx_features_pair): bit-identity tests, the
# feature parity suite, and the bench with the pair path off / on (same box).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05d
mkdir -p $O
cd $R
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_features_pair.py tests/test_gpu_parity.py tests/test_gpu_streams.py > $O/t.log 2>&1
CPX_PAIR_FEATURES=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_off.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_on.log 2>&1
echo done
