# reg1 alone on the first mask test (hang check), then the full seg/e2e parity + A/B bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04o
mkdir -p $O
cd $R
T="tests/test_gpu_seg.py::test_masks_full_resolution_bit_exact_vs_oracle"
CPX_FE_REG=1 timeout -k 10 100 python -u -m pytest "$T" -x -v --timeout 90 --timeout-method thread > $O/reg1.log 2>&1
rc=$?
echo "reg1 rc=$rc"; tail -2 $O/reg1.log
[ $rc -eq 0 ] || exit 1
RUN_TAG=r04o bash tools/run_r04l.sh
