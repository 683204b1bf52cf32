#!/bin/bash
# One GPU-box pass that produces the round's committed evidence (run via gpurun from the repo
# root): the default bench line (with cpu_baseline), a rocprofv3 kernel-trace + stats run of
# the same bench, and separate FETCH_SIZE / WRITE_SIZE counter passes (MI355X_MICROARCH.md:
# they do not fit one pass).  Outputs land under gpurun_out/round/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-round}
BATCH=${BATCH:-48}  # bench.py's default --batch
PREC=${PREC:-f16x3}  # bench.py's default --cpnet-precision
mkdir -p $O
cd $R
timeout -k 10 420 python -u bench.py > $O/bench_default.log 2>&1
timeout -k 10 200 python -u tools/flow_error_flops.py > $O/flow_error_flops.json 2> $O/flow_error_flops.log
cd /tmp && export TMPDIR=/tmp
cd $R
# per-kernel durations: one pipeline (steps run back to back, as the bench's instrumented
# stage timing that the roofline uses); the default two-pipeline run overlaps batches, so its
# kernel durations include co-resident work (kernels_concurrent.md)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/bench_kt.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt2 -o run -- \
  python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/bench_kt2.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- \
  python -u bench.py --pipes 1 --steps 3 --warmup 1 --no-cpu-baseline --stage-steps 1 > $O/bench_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- \
  python -u bench.py --pipes 1 --steps 3 --warmup 1 --no-cpu-baseline --stage-steps 1 > $O/bench_write.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/mfma -o run -- \
  python -u bench.py --pipes 1 --steps 3 --warmup 1 --no-cpu-baseline --stage-steps 1 > $O/bench_mfma.log 2>&1
# VALU instructions of the register flow-error kernels (bench.py's roofline_all.flow_error_reg)
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-include-regex k_flow_error_reg --output-format csv \
  -d $O/sqfe -o run -- python -u bench.py --pipes 1 --steps 3 --warmup 1 --no-cpu-baseline --stage-steps 1 > $O/bench_sqfe.log 2>&1

# summarise on the box (raw per-dispatch CSVs are too large to bring back)
python tools/prof_summary.py $O/kt/run_kernel_trace.csv --steps 4 --md > $O/kernels_steady.md
python tools/prof_summary.py $O/kt2/run_kernel_trace.csv --steps 4 --md > $O/kernels_concurrent.md
cp $O/kt/run_kernel_stats.csv $O/kernel_stats.csv
cp $O/kt2/run_kernel_stats.csv $O/kernel_stats_concurrent.csv
python tools/pmc_traffic.py $O/fetch $O/write --batch $BATCH --precision ${PREC:-f16x3} --out $O/pmc_traffic.json > $O/pmc_traffic.log
python tools/pmc_mfma.py $O/mfma --out $O/pmc_mfma.json > $O/pmc_mfma.log
python tools/sq_flow_error.py $O/sqfe --fovs $BATCH --out $O/sq_flow_error.json > $O/sq_flow_error.log
rm -rf $O/kt $O/kt2 $O/fetch $O/write $O/mfma $O/sqfe
echo done
