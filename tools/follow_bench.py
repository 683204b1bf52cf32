"""Same-box timing of the segmentation post-processing (cpx_seg_masks) on the bench's own
network outputs: 32 FOVs of the synthetic plate through CPnet once, then the masks call timed
with HIP events; every repetition's labels are compared with the first (determinism)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))

import torch  # noqa: E402

from cpx import shard  # noqa: E402
from cpx.device import Device  # noqa: E402
from cpx.pipeline import FovPipeline, PipelineConfig  # noqa: E402
from cpx.synth import synth_fovs, synth_illum  # noqa: E402


def main():
    B = int(os.environ.get("BATCH", "32"))
    dev = Device(0)
    w = os.path.join(REPO, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
    cfg = PipelineConfig(H=2080, W=2080, C=5, batch=B, weights=w)
    pipe = FovPipeline(dev, cfg, synth_illum(5, 2080, 2080, seed=1))
    raw = synth_fovs(B, 5, 2080, 2080, dev.torch_device, seed=shard.fov_seed(shard.plate_fovs()[0]))
    pipe.run(raw)
    torch.cuda.synchronize()
    seg = pipe.seg
    lab = pipe.labels["Nuclei"]
    ts, n_final, same = [], [], []
    ref = None
    for i in range(int(os.environ.get("REPS", "4"))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        seg.postprocess(lab)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
        n_final.append(int(seg.seg_stats()["n_final"].sum()))
        if ref is None:
            ref = lab.clone()
        else:  # labels of every repetition vs the first: pixels that differ
            same.append(int((lab != ref).sum().item()))
    print(json.dumps({"seg_post_ms": ts, "n_final": n_final, "label_px_diff_vs_first": same}))


if __name__ == "__main__":
    main()
