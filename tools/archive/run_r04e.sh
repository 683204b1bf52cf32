# New round-4 GPU tests (configs[3] job shape, widened ID bar, recovery) + the I/O-inclusive
# plate bench (tools/plate_bench.py) whose line backs DESIGN's plate throughput.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04e
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_config3_jobs.py tests/test_gpu_ids_wide.py -x -v -s --timeout 900 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python -u tools/plate_bench.py --fovs 96 --warm 48 --threads 16 > $O/plate_bench.log 2>&1
echo done
