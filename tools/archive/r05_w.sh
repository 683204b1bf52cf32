# Round 5: flow following in FOV groups (CPX_FOLLOW_GROUP = G FOVs per launch sequence, every
# round of a group before the next, so the gathered fields can stay in the MALL): segmentation
# parity at G = 6, one-pipeline kernel traces at G = 0 (all), 6, 12, 24, and benches; the p32
# prefetch modes on the bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05w
mkdir -p $O
cd $R
timeout -k 10 600 env CPX_FOLLOW_GROUP=6 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_seg.py > $O/t6.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R
for g in 0 6 12 24; do
  timeout -k 10 300 env CPX_FOLLOW_GROUP=$g rocprofv3 --kernel-trace --output-format csv -d /tmp/kt_$g -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt_$g.log 2>&1
  python tools/prof_summary.py /tmp/kt_$g/run_kernel_trace.csv --steps 4 --md > $O/k_$g.md
  rm -rf /tmp/kt_$g
  grep -h "k_dyn_follow\|total kernel" $O/k_$g.md
done
for g in 0 6 12; do
  timeout -k 10 300 env CPX_FOLLOW_GROUP=$g python -u bench.py --no-cpu-baseline --steps 60 --stage-steps 1 > $O/bench_$g.log 2>&1
  tail -1 $O/bench_$g.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('group',$g,d['value'],d['ms_per_step'],d['stage_ms_per_step']['seg_post'])"
done
# p32 L2 prefetch mode (1: residual + next halo, 2: residual only, 0: none) on the full bench
for m in 1 2 0; do
  timeout -k 10 300 env CPX_X3_P32_TOUCH=$m python -u bench.py --no-cpu-baseline --steps 60 --stage-steps 1 > $O/bench_touch$m.log 2>&1
  tail -1 $O/bench_touch$m.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('touch',$m,d['value'],d['ms_per_step'],d['stage_ms_per_step']['cpnet'])"
done
echo done
