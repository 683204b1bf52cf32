# Round 5: which stages to keep exclusive across the two batches in flight (default now
# cpnet,features): interleaved 60-step benches of a few sets, then the stream / pipeline tests.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05u
mkdir -p $O
cd $R
for i in 1 2; do
  for v in cpnet,features cpnet,features,cells cpnet,features,illum_qc cpnet,seg_post,features,cells cpnet,cells,features,illum_qc,seg_post; do
    timeout -k 10 300 env CPX_STAGE_EXCLUSIVE=$v python -u bench.py --no-cpu-baseline --steps 60 --stage-steps 1 > $O/bench_${v}_$i.log 2>&1
    tail -1 $O/bench_${v}_$i.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$v',$i,d['value'],d['ms_per_step'])"
  done
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_capacity.py tests/test_gpu_recovery.py > $O/t.log 2>&1
echo done
