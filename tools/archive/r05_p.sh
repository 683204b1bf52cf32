# Round 5: SQ counters of k_dyn_follow / k_obj_stage / k_tex_glcm / p32 / flow error (one
# counter pass, summarised and its CSVs removed at once), the LDS atomic micro-benchmark (the
# GLCM's roofline peak), the plate CLI tests and the I/O-inclusive plate bench with the native
# CSV writer (768 FOVs).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05p
mkdir -p $O
cd $R
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -Wno-unused-value tools/micro/lds_atomic.hip -o /tmp/lds_atomic > /dev/null 2>&1
timeout -k 10 120 /tmp/lds_atomic > $O/lds_atomic.log 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_plate.py > $O/t_plate.log 2>&1
timeout -k 10 600 python -u tools/plate_bench.py --fovs 192 --repeat 4 --dir /tmp > $O/plate_bench.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R
B="python -u bench.py --pipes 1 --steps 2 --warmup 1 --no-cpu-baseline --stage-steps 1"
if ! timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD --output-format csv -d /tmp/sq -o run -- $B > $O/sq.log 2>&1; then
  rm -rf /tmp/sq; exit 1
fi
python tools/pmc_sq.py /tmp/sq --match k_dyn_follow,k_obj_stage,k_tex_glcm,k_conv_x3_p32,k_flow_error > $O/sq.txt
rm -rf /tmp/sq
echo done
