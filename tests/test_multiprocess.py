"""World-size-2 CPU (gloo) checks of the multi-GPU split used by bench.py:
well-sharded FOVs with no data-path collective, max-over-ranks timing, summed FOV count."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cpx import shard


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fovs = shard.plate_fovs(plates=("P01", "P02"), n_wells=96, sites=(1, 2), times=(6, 24))
        mine = shard.shard(fovs, rank, world)
        got = [None] * world
        dist.all_gather_object(got, [tuple(f.__dict__.values()) for f in mine])
        t = shard.max_over_ranks(1.5 + rank)
        n = shard.sum_over_ranks(len(mine))
        if rank == 0:
            q.put((got, t, n, len(fovs)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_well_shards_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, t, n, total = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    flat = [f for part in got for f in part]
    assert len(flat) == total == n                # every FOV exactly once
    assert len(set(flat)) == total
    owner = {}
    for r, part in enumerate(got):
        for f in part:
            assert owner.setdefault((f[0], f[1]), r) == r   # wells are never split
    assert abs(len(got[0]) - len(got[1])) <= 8               # balanced to a well
    assert t == 1.5 + (world - 1)                             # max over ranks


def test_shard_single_rank_is_identity():
    fovs = shard.plate_fovs(n_wells=384)
    assert shard.shard(fovs, 0, 1) == fovs
    assert len(fovs) == 384 and fovs[0].well == "A01" and fovs[-1].well == "P24"
    assert shard.fov_seed(fovs[0]) != shard.fov_seed(fovs[1])
