# Round 5: why the plate CLI's two pipelines barely overlap on the GPU (r05ai: >= 2 kernels 3 % of
# the time, against 1.27x kernel-time / busy-time in the bench).  Kernel traces and benches of
# the plate with 8 hardware queues per process (is a fifth stream sharing a queue?) and with each
# upload on its pipeline's own stream (four streams).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05aj
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
for cfg in "GPU_MAX_HW_QUEUES=8" "CPX_PLATE_UPLOAD=pipeline"; do
  tag=$(echo $cfg | tr '=' '_')
  timeout -k 10 400 env $cfg rocprofv3 --kernel-trace --output-format csv -d /tmp/pt -o run -- \
    python -u tools/plate_bench.py --fovs 96 --repeat 4 --dir /tmp > $O/pt_$tag.log 2>&1
  grep '^{"metric"' $O/pt_$tag.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg', d['value'], d['seconds'])"
  S=$(grep '^{"metric"' $O/pt_$tag.log | python -c "import json,sys;print(json.loads(sys.stdin.read())['seconds'])")
  python tools/plate_overlap.py /tmp/pt/run_kernel_trace.csv --seconds $S | tee $O/overlap_$tag.txt
  rm -rf /tmp/pt
done
for cfg in "GPU_MAX_HW_QUEUES=8" "CPX_PLATE_UPLOAD=pipeline" "CPX_PLATE_UPLOAD=device"; do
  timeout -k 10 400 env $cfg python -u tools/plate_bench.py --fovs 192 --repeat 4 --dir /tmp > $O/pb.log 2>&1
  tail -1 $O/pb.log | tee -a $O/plate_bench.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg', d['value'], d['value_excluding_csv'])"
done
echo done
