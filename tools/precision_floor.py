"""Noise floor of the reference's own segmentation (CPU only): the same FOVs through Cellpose's
CPnet in fp32 and in fp64 on the CPU, each followed by the restated dynamics; counts the pixels
and objects whose masks differ.  Shows how many boundary pixels flip under rounding-level
changes of the network output alone."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import cpx_oracle as orc  # noqa: E402
import seg_oracle as so  # noqa: E402
from cpx.cpnet import build_cpnet  # noqa: E402
from cpx.synth import synth_fovs, synth_illum  # noqa: E402


def main():
    B = int(os.environ.get("B", "8"))
    H = W = 2080
    torch.set_num_threads(int(os.environ.get("THREADS", "8")))
    w = os.path.join(REPO, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
    net32 = build_cpnet(state_dict_path=w).float()
    net64 = build_cpnet(state_dict_path=w).double()
    raw = synth_fovs(B, 5, H, W, "cpu", seed=int(os.environ.get("SEED", "31"))).numpy().view(np.uint16).reshape(B, 5, H, W)
    illum = synth_illum(5, H, W, seed=1)
    Ly, Lx = so.net_size(H, W)
    tot = {"fovs": 0, "objects": 0, "pixels_differing": 0, "objects_differing": 0}
    for b in range(B):
        corr = np.stack([orc.illum_correct_producer(raw[b, c], illum[c]) for c in range(5)])
        tiles, g = so.make_net_input(corr, Ly, Lx)
        with torch.no_grad():
            y32 = net32(torch.from_numpy(tiles)).numpy()
            y64 = net64(torch.from_numpy(tiles).double()).numpy()
        m32 = so.compute_masks(so.average_tiles(y32, g), H, W)
        # fp64 network rounded to fp32 once at the output (the flows then follow the fp32 path)
        m64 = so.compute_masks(so.average_tiles(y64.astype(np.float32), g), H, W)
        diff = m32 != m64
        objs = np.unique(np.concatenate([m32[diff], m64[diff]]))
        r = {"fov": b, "objects": int(m32.max()), "pixels_differing": int(diff.sum()),
             "objects_differing": int((objs > 0).sum()), "max_abs_out_diff": float(np.abs(y32 - y64).max())}
        print(json.dumps(r), flush=True)
        tot["fovs"] += 1
        tot["objects"] += r["objects"]
        tot["pixels_differing"] += r["pixels_differing"]
        tot["objects_differing"] += r["objects_differing"]
    print(json.dumps({"total": tot}))


if __name__ == "__main__":
    main()
