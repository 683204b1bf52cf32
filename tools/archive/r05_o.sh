# Round 5: what bounds k_dyn_follow / k_obj_stage / k_tex_glcm (SQ and TA/TCP counter passes over
# one-pipeline bench steps), the LDS atomic micro-benchmark (the GLCM's roofline peak), and the
# parity tests of the current default library (16-byte group loads, paired follow gathers).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05o
mkdir -p $O
cd $R
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_features_pair.py tests/test_gpu_parity.py tests/test_gpu_seg.py > $O/t.log 2>&1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/micro/lds_atomic.hip -o $O/lds_atomic
timeout -k 10 120 $O/lds_atomic > $O/lds_atomic.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R
B="python -u bench.py --pipes 1 --steps 2 --warmup 1 --no-cpu-baseline --stage-steps 1"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD --output-format csv -d $O/sq -o run -- $B > $O/sq.log 2>&1
python tools/pmc_sq.py $O/sq --match k_dyn_follow,k_obj_stage,k_tex_glcm,k_conv_x3_p32,k_flow_error > $O/sq.txt
timeout -s KILL 180 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d $O/ta -o run -- $B > $O/ta.log 2>&1
python tools/pmc_sq.py $O/ta --match k_dyn_follow,k_obj_stage,k_tex_glcm,k_conv_x3_p32 > $O/ta.txt
rm -rf $O/sq $O/ta
echo done
