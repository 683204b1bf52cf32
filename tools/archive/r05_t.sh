# Round 5: longer interleaved A/B of CPX_STAGE_EXCLUSIVE=cpnet,features vs none (60 steps each).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05t
mkdir -p $O
cd $R
for i in 1 2 3; do
  for v in none cpnet,features; do
    e=$v; [ "$v" = none ] && e=""
    timeout -k 10 300 env CPX_STAGE_EXCLUSIVE=$e python -u bench.py --no-cpu-baseline --steps 60 --stage-steps 1 > $O/bench_${v}_$i.log 2>&1
    tail -1 $O/bench_${v}_$i.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$v',$i,d['value'],d['ms_per_step'])"
  done
done
echo done
