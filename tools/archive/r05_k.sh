# Round 5: k_obj_stage with bit-parallel AreaShape sums (default library), then block size /
# waves-per-SIMD variants (tools/_var/libcpx_st{B,C,D}.so: 512 threads at 3 blocks per CU for the
# single-set kernel; 256 threads at 6 / 4 and 8 / 5 blocks per CU single-set / twin): feature
# parity tests, tools/tex_bench.py per variant, one-pipeline kernel traces.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05k
mkdir -p $O
cd $R
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_features_pair.py tests/test_gpu_parity.py > $O/t.log 2>&1
timeout -k 10 200 env CPX_LIB=$R/tools/_var/libcpx_sprof.so python -u tools/tex_bench.py --batch 16 --reps 3 > $O/tex_sprof.log 2>&1
timeout -k 10 200 python -u tools/tex_bench.py --batch 16 --reps 3 > $O/tex_A.log 2>&1
for v in B C D; do
  timeout -k 10 200 env CPX_LIB=$R/tools/_var/libcpx_st$v.so python -u tools/tex_bench.py --batch 16 --reps 3 > $O/tex_$v.log 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd $R
kt() {  # name, then env assignments
  name=$1; shift
  timeout -k 10 300 env "$@" rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$name -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt_$name.log 2>&1
  python tools/prof_summary.py $O/kt_$name/run_kernel_trace.csv --steps 4 --md > $O/k_$name.md
  rm -rf $O/kt_$name
}
kt A CPX_X3_P32_TOUCH=1
kt C CPX_LIB=$R/tools/_var/libcpx_stC.so
kt D CPX_LIB=$R/tools/_var/libcpx_stD.so
echo done
