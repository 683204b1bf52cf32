# Where the deep-level convolution time goes: tools/conv_bench_x3.py on timing builds of
# k_conv_x3 that drop a piece (tools/build_variants.sh, CPX_X3_DIAG; wrong outputs).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04f
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/conv_bench_x3.py --tiles 432 --reps 5 --variants 0 > $O/conv_base.log 2>&1
for v in nodma nobar noepi mfmaonly; do
  CPX_LIB=$R/tools/_var/libcpx_$v.so timeout -k 10 200 python -u tools/conv_bench_x3.py --tiles 432 --reps 5 --variants 0 > $O/conv_$v.log 2>&1
done
echo done
