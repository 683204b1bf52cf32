"""Segmentation diagnostics on one bench batch (GPU): per-stage times (HIP events) for a CPnet
precision, and the size distribution of the Nuclei masks against the flow-error kernels' LDS
capacity (bbox cells (bh + 2) x stride > 20224 go to the large-object path)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from cpx import shard  # noqa: E402
from cpx.device import Device  # noqa: E402
from cpx.pipeline import FovPipeline, PipelineConfig  # noqa: E402
from cpx.synth import synth_fovs, synth_illum  # noqa: E402


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "f16x3"
    B = int(os.environ.get("BATCH", "48"))
    dev = Device(0)
    w = os.path.join(REPO, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
    cfg = PipelineConfig(H=2080, W=2080, C=5, batch=B, weights=w, cpnet_precision=prec)
    pipe = FovPipeline(dev, cfg, synth_illum(5, 2080, 2080, seed=1))
    mine = shard.shard(shard.plate_fovs(n_wells=384), 0, 1)
    out = {"precision": prec, "batch": B, "batches": []}
    for i in range(int(os.environ.get("NB", "2"))):
        raw = synth_fovs(B, 5, 2080, 2080, dev.torch_device, seed=shard.fov_seed(mine[(i * B) % len(mine)]) + 7919 * i)
        pipe.run(raw)
        res = pipe.fetch()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        pipe.seg.prepare(pipe.corr)
        ev[1].record()
        pipe.seg._run_net()
        ev[2].record()
        pipe.seg.postprocess(pipe.labels["Nuclei"])
        ev[3].record()
        torch.cuda.synchronize()
        cells = []
        for b in range(B):
            o = res.objects["Nuclei"][b]
            bh = o["bbox"][:, 2] - o["bbox"][:, 0]
            bw = o["bbox"][:, 3] - o["bbox"][:, 1]
            cells.append((bh + 2) * ((bw + 3) & ~1))
        allc = np.concatenate(cells)
        per_fov_big = [int((c > 20224).sum()) for c in cells]
        st = res.seg_stats
        out["batches"].append({
            "ms": {"prep": ev[0].elapsed_time(ev[1]), "cpnet": ev[1].elapsed_time(ev[2]),
                   "seg_post": ev[2].elapsed_time(ev[3])},
            "n_objects_mean": float(np.mean([len(c) for c in cells])),
            "bbox_cells_pct_50_90_99_max": [int(v) for v in np.percentile(allc, [50, 90, 99, 100])],
            "big_objects_total": int((allc > 20224).sum()), "big_per_fov_max": max(per_fov_big),
            "largest_bbox": [int(v) for v in sorted(allc)[-5:]],
            "n_moving_mean": float(st["n_moving"].mean()), "n_bad_flow_total": int(st["n_bad_flow"].sum()),
            "n_final_mean": float(st["n_final"].mean())})
        print(json.dumps(out["batches"][-1]), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", f"seg_diag_{prec}.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
