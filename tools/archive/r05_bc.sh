# Round 5: final-tree default bench lines (as the driver runs it) with a same-box --cu-split none pair.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05bc
mkdir -p $O
cd $R
for cs in auto none auto; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --cu-split $cs > $O/b.log 2>&1
  tail -1 $O/b.log | tee -a $O/bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cs', d['value'], d['ms_per_step'], d['steps'])"
done
echo done
