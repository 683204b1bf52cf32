# Round 5: the plate with its uploads on the result-copy stream (four streams, the bench's count)
# vs the separate upload stream, both at HIP's 4 queues and the separate stream at 8: kernel
# overlap traces (env set in the shell, so rocprofv3's early HIP start sees it) and benches.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ap
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
for cfg in "CPX_PLATE_UPLOAD=copy CPX_PLATE_HW_QUEUES=4 GPU_MAX_HW_QUEUES=4" "CPX_PLATE_HW_QUEUES=4 GPU_MAX_HW_QUEUES=4"; do
  tag=$(echo $cfg | cut -c1-20 | tr '= ' '__')
  timeout -k 10 400 env $cfg rocprofv3 --kernel-trace --output-format csv -d /tmp/pt -o run -- \
    python -u tools/plate_bench.py --fovs 96 --repeat 4 --dir /tmp > $O/pt.log 2>&1
  S=$(grep '^{"metric"' $O/pt.log | python -c "import json,sys;print(json.loads(sys.stdin.read())['seconds'])")
  echo "$cfg"
  python tools/plate_overlap.py /tmp/pt/run_kernel_trace.csv --seconds $S | tee $O/overlap_$tag.txt | head -1
  rm -rf /tmp/pt
done
for i in 1 2; do
for cfg in "CPX_PLATE_UPLOAD=copy CPX_PLATE_HW_QUEUES=4" "CPX_PLATE_HW_QUEUES=4" "CPX_PLATE_HW_QUEUES=8"; do
  timeout -k 10 400 env $cfg python -u tools/plate_bench.py --fovs 192 --repeat 8 --dir /tmp > $O/pb.log 2>&1
  tail -1 $O/pb.log | tee -a $O/plate_bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg', d['value'], d['value_excluding_csv'])"
done
done
echo done
