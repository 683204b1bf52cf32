# Round 5: k_obj_stage phase breakdown (-DCPX_STAGE_PROF build through tools/tex_bench.py), the
# f16x3 CPnet tests with the p32 L2 prefetch, and non-temporal epilogue stores
# (tools/_var/libcpx_nt.so) against the default library in a one-pipeline kernel trace.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05j
mkdir -p $O
cd $R
timeout -k 10 300 env CPX_LIB=$R/tools/_var/libcpx_sprof.so python -u tools/tex_bench.py --batch 16 --reps 3 > $O/stage_prof.log 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cpnet_x3.py > $O/t.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R
kt() {  # name, then env assignments
  name=$1; shift
  timeout -k 10 300 env "$@" rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$name -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt_$name.log 2>&1
  python tools/prof_summary.py $O/kt_$name/run_kernel_trace.csv --steps 4 --md > $O/k_$name.md
  rm -rf $O/kt_$name
}
kt def CPX_X3_P32_TOUCH=1
kt nt CPX_LIB=$R/tools/_var/libcpx_nt.so
echo done
