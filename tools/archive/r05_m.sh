# Round 5: k_dyn_follow with paired 16-byte buffer gathers (CPX_FOLLOW_V4=1; 1 / 2 trajectories
# per thread) — segmentation parity tests, then one-pipeline kernel traces; the conv epilogue's
# per-channel tables loaded before the y stores (tools/_var/libcpx_epre.so).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05m
mkdir -p $O
cd $R
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 env CPX_FOLLOW_V4=1 $T tests/test_gpu_seg.py > $O/t_v4.log 2>&1
timeout -k 10 600 env CPX_FOLLOW_V4=1 CPX_FOLLOW_NI=2 $T tests/test_gpu_seg.py > $O/t_v4n2.log 2>&1
timeout -k 10 600 env CPX_LIB=$R/tools/_var/libcpx_epre.so $T tests/test_gpu_cpnet_x3.py > $O/t_epre.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R
kt() {  # name, then env assignments
  name=$1; shift
  timeout -k 10 300 env "$@" rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$name -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt_$name.log 2>&1
  python tools/prof_summary.py $O/kt_$name/run_kernel_trace.csv --steps 4 --md > $O/k_$name.md
  rm -rf $O/kt_$name
}
kt base CPX_FOLLOW_V4=0
kt v4 CPX_FOLLOW_V4=1
kt v4n2 CPX_FOLLOW_V4=1 CPX_FOLLOW_NI=2
kt epre CPX_LIB=$R/tools/_var/libcpx_epre.so
echo done
