# Round 5: the plate CLI with CU-split pipeline streams vs unrestricted ones (1,536 FOVs, two rounds).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05az
mkdir -p $O
cd $R
for i in 1 2; do
for cs in halves none; do
  timeout -k 10 400 env CPX_CU_SPLIT=$cs python -u tools/plate_bench.py --fovs 192 --repeat 8 --dir /tmp > $O/pb.log 2>&1
  tail -1 $O/pb.log | tee -a $O/plate_bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cs', d['value'], d['value_excluding_csv'])"
done
done
echo done
