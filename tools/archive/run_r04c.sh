# Conflict-free halo reads + epilogue stem residual: parity (x3 kernels, whole forward, e2e IDs)
# and an A/B kernel trace against the previous tile layout (CPX_X3_STEM=0 CPX_X3_FOLD=0 does not
# restore the old layout: the old numbers are gpurun_out/r04b/kernels_old.md).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04c
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cpnet_x3.py tests/test_gpu_e2e.py -x -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/bench_kt.log 2>&1
python tools/prof_summary.py $O/kt/run_kernel_trace.csv --steps 4 --md > $O/kernels.md
rm -rf $O/kt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
echo done
