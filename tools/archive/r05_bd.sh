# Round 5: CPnet variant 3 (BM 64 single-buffer for every >= 64-channel conv) under the CU-split
# pipelines, same-box pairs against the default.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05bd
mkdir -p $O
cd $R
for i in 1 2; do
for v in 0 3; do
  timeout -k 10 300 env CPX_X3_VARIANT=$v python -u bench.py --no-cpu-baseline --steps 40 --stage-steps 1 > $O/b.log 2>&1
  tail -1 $O/b.log | tee -a $O/bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('variant $v', d['value'], d['ms_per_step'])"
done
done
echo done
