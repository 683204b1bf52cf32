"""Multi-GPU work split for the per-FOV path.

FOVs are independent, so ranks share nothing on the data path: every rank (one process per
GPU) takes whole wells — all sites and time points of a well land on one GPU, so the well-level
aggregations downstream (Cellpose_GPU_s3fs.py:402-412, Pycyto_pertime.py:69-72) stay host-side
concatenations.  Well w goes to rank (w mod world).  Results are gathered on the host and sorted
by (plate, well, site, time), so output is identical for any world size.
"""
from __future__ import annotations

from dataclasses import dataclass

ROWS = "ABCDEFGHIJKLMNOP"


@dataclass(frozen=True, order=True)
class Fov:
    plate: str
    well: str
    site: int
    time: int


def plate_wells(n_wells: int = 384):
    """Well names in plate order: A01..A24, B01.. (384-well: 16 rows x 24 columns;
    96-well: 8 x 12)."""
    cols = 24 if n_wells == 384 else 12
    rows = n_wells // cols
    return [f"{ROWS[r]}{c + 1:02d}" for r in range(rows) for c in range(cols)]


def plate_fovs(plates=("P01",), n_wells=384, sites=(1,), times=(24,)):
    return [Fov(p, w, s, t) for p in plates for w in plate_wells(n_wells) for s in sites for t in times]


def shard(fovs, rank: int, world: int):
    """FOVs of `rank`: wells dealt round-robin in first-appearance order; all FOVs of a well
    stay together."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    order = {}
    for f in fovs:
        order.setdefault((f.plate, f.well), len(order))
    return [f for f in fovs if order[(f.plate, f.well)] % world == rank]


def fov_seed(f: Fov, channel: int = 0) -> int:
    """Deterministic per-FOV synthetic seed (0x5A6A ^ hash of the FOV key)."""
    h = 1469598103934665603
    for ch in f"{f.plate}|{f.well}|{f.site}|{f.time}|{channel}".encode():
        h = ((h ^ ch) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return (0x5A6A ^ h) & 0x7FFFFFFF


def max_over_ranks(value: float, device=None) -> float:
    """Largest `value` over all ranks (the bench's wall time); identity without a process group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: int, device=None) -> int:
    """Total of an integer count over ranks (FOVs processed by the whole job)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return int(value)
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())
