# A/B kernel traces of the round-4 changes (pipes 1, steps back to back): the new tree vs the
# folded projections / fused stem / small-item GLCM switched off, plus SQ counters of the CPnet
# convolutions (tools/conv_bench_x3.py).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04b
mkdir -p $O
cd $R
export TMPDIR=/tmp
run_kt() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$name -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/bench_kt_$name.log 2>&1
  python tools/prof_summary.py $O/kt_$name/run_kernel_trace.csv --steps 4 --md > $O/kernels_$name.md
  rm -rf $O/kt_$name
}
run_kt new
run_kt old CPX_X3_FOLD=0 CPX_X3_STEM=0 CPX_GLCM_SMALL=0
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/sqa -o run -- python -u tools/conv_bench_x3.py --tiles 432 --reps 1 --forward 1 --variants 0 > $O/sqa.log 2>&1
python tools/pmc_sq.py $O/sqa --match conv_x3 > $O/sqa.txt
rm -rf $O/sqa
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/sqb -o run -- python -u tools/conv_bench_x3.py --tiles 432 --reps 1 --forward 1 --variants 0 > $O/sqb.log 2>&1
python tools/pmc_sq.py $O/sqb --match conv_x3 > $O/sqb.txt
rm -rf $O/sqb
echo done
