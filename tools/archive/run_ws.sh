# Development GPU pass: watershed parity + timing (with the debug counters), a bench line, trace.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ws
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_watershed.py tests/test_gpu_parity.py tests/test_gpu_fov.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -u tools/ws_bench.py --check > $O/ws.log 2>&1
CPX_WS_DEBUG=1 timeout -k 10 200 python -u tools/ws_bench.py --reps 1 > $O/ws_dbg.log 2>&1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/bench_kt.log 2>&1
python tools/prof_summary.py $O/kt/run_kernel_trace.csv --steps 4 --md > $O/kernels.md
rm -rf $O/kt
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 12 > $O/bench.log 2>&1
echo done
