# Development GPU pass: segmentation parity (small cases + 2080^2 e2e vs the oracle), a bench line
# and a one-pipeline kernel trace.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/seg
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_e2e.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 12 > $O/bench.log 2>&1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/bench_kt.log 2>&1
python tools/prof_summary.py $O/kt/run_kernel_trace.csv --steps 4 --md > $O/kernels_steady.md
rm -rf $O/kt
echo done
