# Rehearse bench.py's multi-rank path (torchrun, gloo barrier, shared WorkQueue claims, max/sum
# over ranks) with two ranks on the one GPU of the box (CPX_BENCH_DEVICE=0; 16 FOVs per step and
# one pipeline per rank, so that two ranks fit one card).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04v
mkdir -p $O
cd $R
CPX_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 8 --warmup 2 --no-cpu-baseline --batch 16 --pipes 1 > $O/bench2.log 2>&1
tail -1 $O/bench2.log
CPX_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 8 --warmup 2 --no-cpu-baseline --batch 16 --pipes 1 --scheduler static > $O/bench2_static.log 2>&1
tail -1 $O/bench2_static.log
echo done
