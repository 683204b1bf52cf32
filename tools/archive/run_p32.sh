# Development GPU pass: persistent weights-resident 224^2 convolution (CPX_X3_P32) — parity, A/B.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/p32
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_cpnet_x3.py tests/test_gpu_e2e.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
export TMPDIR=/tmp
for v in 1 0; do
  export CPX_X3_P32=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$v -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/bench_kt$v.log 2>&1
  python tools/prof_summary.py $O/kt$v/run_kernel_trace.csv --steps 4 --md > $O/kernels_$v.md
  rm -rf $O/kt$v
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 12 > $O/bench_$v.log 2>&1
done
echo done
