# GPU busy fraction of the default two-pipeline bench (union of kernel intervals, tools/busy_union.py).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04x
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- \
  python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/bench_kt.log 2>&1
python tools/busy_union.py $O/kt/run_kernel_trace.csv > $O/busy.txt
cat $O/busy.txt
rm -rf $O/kt
