#!/bin/bash
# Development GPU pass (run via gpurun from the repo root): the given pytest files, a short bench
# line without the CPU baseline, and a one-pipeline kernel trace summarised per step.
# usage: bash tools/quick_check.sh "tests/test_a.py tests/test_b.py"
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/quick
mkdir -p $O
cd $R
if [ -n "$1" ]; then
  timeout -k 10 500 python -u -m pytest $1 -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
fi
timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 12 > $O/bench.log 2>&1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/bench_kt.log 2>&1
python tools/prof_summary.py $O/kt/run_kernel_trace.csv --steps 4 --md --series "${SERIES:-k_dyn_follow}" > $O/kernels_steady.md
rm -rf $O/kt
echo done
