# Round 5: k_obj_stage L2 prefetch of the channel bboxes + GLCM chunk scatter without integer
# divisions: feature tests, the bench, and a one-pipeline kernel trace.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05h
mkdir -p $O
cd $R
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_features_pair.py tests/test_gpu_parity.py > $O/t.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/bench_kt.log 2>&1
python tools/prof_summary.py $O/kt/run_kernel_trace.csv --steps 4 --md > $O/kernels_steady.md
rm -rf $O/kt
echo done
