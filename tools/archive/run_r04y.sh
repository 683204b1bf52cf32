# SQ counters of the flow-error kernels (register screening vs LDS) in one bench pass.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04y
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o run -- \
  python -u bench.py --pipes 1 --steps 3 --warmup 1 --no-cpu-baseline --stage-steps 1 > $O/bench_sq.log 2>&1
python tools/pmc_sq.py $O/sq --match flow_error > $O/sq_flow_error.txt
cat $O/sq_flow_error.txt
rm -rf $O/sq
