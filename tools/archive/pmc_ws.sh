# Development GPU pass: SQ counters of the Cells watershed kernels (one counter pass over ws_bench).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/wssq
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --output-format csv -d $O/pmc -o run -- python -u tools/ws_bench.py --reps 1 > $O/ws.log 2>&1
python tools/pmc_sq.py $O/pmc --match k_ws,k_edt > $O/sq.txt
rm -rf $O/pmc
echo done
