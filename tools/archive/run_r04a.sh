# Round-4 first GPU pass: recovery / x3 / streams tests, the default bench, then the CPnet
# convolutions in isolation (tools/conv_bench_x3.py) with two SQ counter passes.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04a
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cpnet_x3.py tests/test_gpu_recovery.py tests/test_gpu_streams.py tests/test_gpu_e2e.py -x -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
timeout -k 10 300 python -u tools/conv_bench_x3.py --tiles 432 --reps 5 --variants 0 > $O/conv.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sqa -o run -- python -u tools/conv_bench_x3.py --tiles 432 --reps 1 --forward 1 --variants 0 > $O/sqa.log 2>&1
python tools/pmc_sq.py $O/sqa --match conv_x3 > $O/sqa.txt
rm -rf $O/sqa
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d $O/sqb -o run -- python -u tools/conv_bench_x3.py --tiles 432 --reps 1 --forward 1 --variants 0 > $O/sqb.log 2>&1
python tools/pmc_sq.py $O/sqb --match conv_x3 > $O/sqb.txt
rm -rf $O/sqb
echo done
