# Round 5: k_dyn_follow with 1 / 2 / 4 trajectories per thread (CPX_FOLLOW_NI): segmentation
# parity tests at each setting, then one-pipeline kernel traces; non-temporal conv stores now
# default (CPnet tests).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05l
mkdir -p $O
cd $R
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_seg.py tests/test_gpu_cpnet_x3.py > $O/t1.log 2>&1
timeout -k 10 600 env CPX_FOLLOW_NI=2 $T tests/test_gpu_seg.py > $O/t2.log 2>&1
timeout -k 10 600 env CPX_FOLLOW_NI=4 $T tests/test_gpu_seg.py > $O/t4.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R
kt() {  # name, then env assignments
  name=$1; shift
  timeout -k 10 300 env "$@" rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$name -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt_$name.log 2>&1
  python tools/prof_summary.py $O/kt_$name/run_kernel_trace.csv --steps 4 --md > $O/k_$name.md
  rm -rf $O/kt_$name
}
kt ni1 CPX_FOLLOW_NI=1
kt ni2 CPX_FOLLOW_NI=2
kt ni4 CPX_FOLLOW_NI=4
echo done
