# Development GPU pass: watershed + GLCM SQ counters, GLCM phase timing of the no-atomic /
# no-homogeneity-lookup timing variants (tools/_var, wrong results by construction).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/glcm2
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --output-format csv -d $O/pmc -o run -- python -u tools/ws_bench.py --reps 1 > $O/ws.log 2>&1
python tools/pmc_sq.py $O/pmc --match k_ws,k_edt > $O/ws_sq.txt
rm -rf $O/pmc
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU --output-format csv -d $O/pmc -o run -- python -u tools/tex_bench.py --batch 16 --reps 1 > $O/tex_pmc.log 2>&1
python tools/pmc_sq.py $O/pmc --match k_tex_glcm,k_obj_stage > $O/glcm_sq.txt
rm -rf $O/pmc
for v in gprof gnoatom gnohom gnoboth; do
  CPX_LIB=$R/tools/_var/libcpx_$v.so timeout -k 10 200 python -u tools/tex_bench.py --batch 16 > $O/tex_$v.log 2>&1
done
echo done
