# QC row/column FFT kernels at 320 threads (one P3 round) vs 256: parity of the 320 build on the
# QC tests, qc_bench A/B; then the bench under the HIP blit-engine setting (D2H result copies).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04t
mkdir -p $O
cd $R
CPX_LIB=$R/tools/_var/libcpx_qc320.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "qc or illum" -x -v --timeout 200 --timeout-method thread > $O/tests320.log 2>&1
tail -1 $O/tests320.log
for v in qc256 qc320 qc256 qc320; do
  CPX_LIB=$R/tools/_var/libcpx_$v.so timeout -k 10 120 python -u tools/qc_bench.py --fovs 48 --reps 10 > $O/$v.log 2>&1
  echo "$v: $(tail -1 $O/$v.log)"
done
for b in 0 3 0 3; do
  GPU_BLIT_ENGINE_TYPE=$b timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 16 > $O/bench_blit$b.log 2>&1
  python -c "import json; d=json.loads(open('$O/bench_blit$b.log').read().strip().splitlines()[-1]); print('blit $b', d['value'])"
done
echo done
