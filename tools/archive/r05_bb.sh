# Round 5: rehearse bench.py's multi-rank path with the default two pipelines per rank (CU-masked
# streams) — two ranks on the box's one GPU (CPX_BENCH_DEVICE=0, 16 FOVs per step).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05bb
mkdir -p $O
cd $R
CPX_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --steps 8 --warmup 2 --no-cpu-baseline --batch 16 > $O/bench2.log 2>&1
tail -1 $O/bench2.log
echo done
