# 32-bit pixel index arithmetic in k_dyn_prep / k_hist_init: seg parity, bench, kernel trace.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04z
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_flowerr_reg.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 16 > $O/bench.log 2>&1
python -c "import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['stage_ms_per_step'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/bench_kt.log 2>&1
python tools/prof_summary.py $O/kt/run_kernel_trace.csv --steps 4 --md > $O/kernels_steady.md
rm -rf $O/kt
grep -E "k_dyn_prep|k_hist_init|total" $O/kernels_steady.md
