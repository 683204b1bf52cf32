# Round 5: does cpx.plate's own GPU_MAX_HW_QUEUES=8 default (set in Python before torch loads HIP)
# take effect?  plate bench (768 FOVs) with the variable unset, forced to 4 and forced to 8.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05an
mkdir -p $O
cd $R
for cfg in "CPX_NOP=1" "GPU_MAX_HW_QUEUES=4" "GPU_MAX_HW_QUEUES=8" "CPX_NOP=1" "GPU_MAX_HW_QUEUES=4"; do
  timeout -k 10 400 env $cfg python -u tools/plate_bench.py --fovs 192 --repeat 4 --dir /tmp > $O/pb.log 2>&1
  tail -1 $O/pb.log | tee -a $O/plate_bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg', d['value'], d['value_excluding_csv'])"
done
echo done
