# Round 5: k_obj_stage 4-pixel groups as 16-byte buffer loads (tools/_var/libcpx_sv4.so) vs the
# default library (now k_dyn_follow 2 x paired gathers): feature parity tests with the variant,
# tools/tex_bench.py for both, one-pipeline kernel traces, and the default bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05n
mkdir -p $O
cd $R
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 env CPX_LIB=$R/tools/_var/libcpx_sv4.so $T tests/test_gpu_features_pair.py tests/test_gpu_parity.py > $O/t_sv4.log 2>&1
timeout -k 10 200 python -u tools/tex_bench.py --batch 16 --reps 3 > $O/tex_def.log 2>&1
timeout -k 10 200 env CPX_LIB=$R/tools/_var/libcpx_sv4.so python -u tools/tex_bench.py --batch 16 --reps 3 > $O/tex_sv4.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R
kt() {  # name, then env assignments
  name=$1; shift
  timeout -k 10 300 env "$@" rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$name -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt_$name.log 2>&1
  python tools/prof_summary.py $O/kt_$name/run_kernel_trace.csv --steps 4 --md > $O/k_$name.md
  rm -rf $O/kt_$name
}
kt def CPX_FOLLOW_NI=2
kt sv4 CPX_LIB=$R/tools/_var/libcpx_sv4.so
cd $R
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
echo done
