# Round 5: (development) each pipeline's stream restricted to half of the CUs by a CU mask
# (interleaved CUs or contiguous halves) against the shared-CU default: two-pipeline benches.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05as
mkdir -p $O
cd $R
for cs in none interleave halves none interleave halves; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 --stage-steps 1 --cu-split $cs > $O/b.log 2>&1
  tail -1 $O/b.log | tee -a $O/bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cs', d['value'], d['ms_per_step'])"
done
echo done
