# Round 5: where the one 1.7 ms __amd_rocclr_copyBuffer per bench step comes from (stream and
# neighbouring kernels in a one-pipeline kernel trace).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ar
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt -o run -- \
  python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt.log 2>&1
python tools/trace_neighbors.py /tmp/kt/run_kernel_trace.csv --match copyBuffer --min-us 300 --last 4 | tee $O/neighbors.txt
head -1 /tmp/kt/run_kernel_trace.csv > $O/columns.txt
rm -rf /tmp/kt
echo done
