# Round 5: SQ counters of the CPnet convolutions (tools/conv_bench_x3.py, variant 0), normal build
# and the CPX_X3_DIAG=4 build (MFMA + fragment-read loop alone), to attribute the deep levels'
# MFMA-idle time.  Counters absent from this rocprofv3's list are dropped from the passes.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05b
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
pick() { local out=""; for c in "$@"; do grep -q "\b$c\b" $O/avail.txt && out="$out $c"; done; echo $out; }
P1=$(pick SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE)
P2=$(pick SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM)
P3=$(pick SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_WAIT_INST_VMEM SQ_INSTS_MFMA SQ_ACTIVE_INST_FLAT)
echo "P1=$P1" > $O/passes.txt; echo "P2=$P2" >> $O/passes.txt; echo "P3=$P3" >> $O/passes.txt
for lib in normal diag4; do
  if [ $lib = diag4 ]; then export CPX_LIB=$R/tools/_var/libcpx_diag4.so; else unset CPX_LIB; fi
  for p in 1 2 3; do
    eval C=\$P$p
    [ -z "$C" ] && continue
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/${lib}_p$p -o run -- \
      python tools/conv_bench_x3.py --tiles 144 --reps 2 --forward 1 --variants 0 > $O/${lib}_p$p.log 2>&1
  done
done
for lib in normal diag4; do for p in 1 2 3; do
  [ -d $O/${lib}_p$p ] && python tools/pmc_sq.py $O/${lib}_p$p --match k_conv_x3 > $O/sq_${lib}_p$p.txt 2>&1 || true
done; done
unset CPX_LIB
timeout -k 10 400 python -u tools/plate_bench.py --fovs 192 --repeat 4 --dir /tmp > $O/plate.log 2>&1
echo done
