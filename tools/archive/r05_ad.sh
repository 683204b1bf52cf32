# Round 5: k_dyn_follow with 3 trajectories per thread (68 VGPRs, 7 waves per SIMD) against 2:
# segmentation parity at 3, one-pipeline kernel traces, benches.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ad
mkdir -p $O
cd $R
timeout -k 10 600 env CPX_FOLLOW_NI=3 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_seg.py > $O/t3.log 2>&1
tail -1 $O/t3.log
cd /tmp && export TMPDIR=/tmp && cd $R
for n in 2 3; do
  timeout -k 10 300 env CPX_FOLLOW_NI=$n rocprofv3 --kernel-trace --output-format csv -d /tmp/kt_$n -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt_$n.log 2>&1
  python tools/prof_summary.py /tmp/kt_$n/run_kernel_trace.csv --steps 4 --md > $O/k_$n.md
  rm -rf /tmp/kt_$n
  grep -h "k_dyn_follow" $O/k_$n.md
done
for n in 3 2; do
  timeout -k 10 300 env CPX_FOLLOW_NI=$n python -u bench.py --no-cpu-baseline --steps 60 --stage-steps 1 > $O/bench_$n.log 2>&1
  tail -1 $O/bench_$n.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('ni',$n,d['value'],d['ms_per_step'],d['stage_ms_per_step']['seg_post'])"
done
echo done
