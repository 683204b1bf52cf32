# Round 5: the 224^2 persistent conv's grid sized for the CUs its (CU-masked) stream holds
# (CPX_X3_P32_MASKGRID, default on) vs per CU of the device: CPnet tests + same-box bench pairs.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05be
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cpnet_x3.py tests/test_gpu_streams.py > $O/t.log 2>&1
tail -1 $O/t.log
for i in 1 2; do
for g in 1 0; do
  timeout -k 10 300 env CPX_X3_P32_MASKGRID=$g python -u bench.py --no-cpu-baseline --steps 40 --stage-steps 1 > $O/b.log 2>&1
  tail -1 $O/b.log | tee -a $O/bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('maskgrid $g', d['value'], d['ms_per_step'])"
done
done
echo done
