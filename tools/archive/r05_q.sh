# Round 5: is the GPU ever idle with two pipelines?  A default (two-pipeline) kernel trace of the
# bench, its busy-time union (tools/busy_union.py) and per-kernel durations under overlap, plus
# the default bench line.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05q
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt2 -o run -- \
  python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/bench_kt2.log 2>&1
python tools/busy_union.py /tmp/kt2/run_kernel_trace.csv > $O/busy.txt
python tools/prof_summary.py /tmp/kt2/run_kernel_trace.csv --steps 8 --md > $O/kernels_concurrent.md
rm -rf /tmp/kt2
echo done
