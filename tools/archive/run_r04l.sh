# Register-resident fp32 flow-error screening (k_flow_error_reg): segmentation parity + e2e,
# undecided-mask counts, bench A/B against CPX_FE_NOREG=1, one-pipeline kernel trace.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN_TAG:-r04l}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py tests/test_gpu_e2e.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
CPX_FE_DEBUG=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 --stage-steps 1 > $O/fe_debug.log 2>&1
CPX_FE_DEBUG=1 CPX_FE_NOREG=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 --stage-steps 1 > $O/fe_debug_noreg.log 2>&1
grep "undecided" $O/fe_debug.log | head -3
grep "undecided" $O/fe_debug_noreg.log | head -3
for v in reg noreg reg; do
  if [ $v = noreg ]; then export CPX_FE_NOREG=1; else unset CPX_FE_NOREG; fi
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 16 > $O/bench_$v.log 2>&1
  python -c "import json; d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['stage_ms_per_step'])"
done
unset CPX_FE_NOREG
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/bench_kt.log 2>&1
python tools/prof_summary.py $O/kt/run_kernel_trace.csv --steps 4 --md > $O/kernels_steady.md
rm -rf $O/kt
grep "flow_error" $O/kernels_steady.md
echo done
