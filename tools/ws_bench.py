"""Same-box timing of cpx_watershed_cells on the bench's own batch (32 FOVs of 2080^2 Nuclei from
the pipeline), per-dispatch durations via rocprofv3 when run under it.

  python tools/ws_bench.py [--reps 5] [--rounds 16 16] [--check]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "image-processing-suite_amd"), os.path.join(REPO, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--rounds", type=int, nargs=2, default=[16, 16])
    ap.add_argument("--check", action="store_true", help="compare FOV 0 with the C heap oracle")
    a = ap.parse_args()
    from cpx import shard
    from cpx._lib import check
    from cpx.device import Device, _ptr
    from cpx.pipeline import FovPipeline, PipelineConfig
    from cpx.synth import synth_fovs, synth_illum
    dev = Device(0)
    H = W = 2080
    C, B = 5, a.batch
    weights = os.path.join(REPO, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
    cfg = PipelineConfig(H=H, W=W, C=C, batch=B, weights=weights, cells="expand")
    pipe = FovPipeline(dev, cfg, synth_illum(C, H, W, seed=1))
    first = shard.shard(shard.plate_fovs(n_wells=384), 0, 1)[0]
    raw = synth_fovs(B, C, H, W, dev.torch_device, seed=shard.fov_seed(first))
    pipe.run(raw)
    dev.sync()
    nuc, corr = pipe.labels["Nuclei"], pipe.corr
    cells = torch.empty_like(nuc)
    cyto = torch.empty_like(nuc)
    st = torch.zeros((B, 8), dtype=torch.int32, device=dev.torch_device)
    ms = []
    for r in range(a.reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        check(dev.lib.cpx_watershed_cells(dev.h, _ptr(nuc), _ptr(corr), B, C, 3, H, W, 15, a.rounds[0],
                                          a.rounds[1], _ptr(cells), _ptr(cyto), _ptr(st), 8), "ws")
        e1.record()
        dev.sync()
        if r:
            ms.append(e0.elapsed_time(e1))
    status = st[:, 0].cpu().numpy()
    out = {"ms": [round(x, 3) for x in ms], "status_min": int(status.min()), "status_max": int(status.max()),
           "rounds": a.rounds, "free_px_per_fov": None}
    if a.check:
        import ws_oracle as wo
        ref, _ = wo.cells_watershed(nuc[0].cpu().numpy(), corr[0, 3].cpu().numpy(), 15)
        out["fov0_equal"] = bool(np.array_equal(ref, cells[0].cpu().numpy()))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
