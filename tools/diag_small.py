"""Small-FOV segmentation check (GPU): a 768^2 batch through the Segmenter at each CPnet precision
vs the CPU path (fp32 CPnet on the CPU + the restated dynamics): seg stats, labels agreement and
the network output error of each precision against the CPU network."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import seg_oracle as so  # noqa: E402
from cpx.cpnet import build_cpnet  # noqa: E402
from cpx.device import Device  # noqa: E402
from cpx.segment import Segmenter  # noqa: E402
from cpx.synth import synth_fovs, synth_illum  # noqa: E402
import cpx_oracle as orc  # noqa: E402


def main():
    H = W = int(os.environ.get("SIZE", "768"))
    B, C = 2, 5
    dev = Device(0)
    w = os.path.join(REPO, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
    raw = synth_fovs(B, C, H, W, dev.torch_device, seed=3, nuclei=(30, 45)).cpu().numpy().view(np.uint16).reshape(B, C, H, W)
    illum = synth_illum(C, H, W, seed=1)
    corr = np.stack([np.stack([orc.illum_correct_producer(raw[b, c], illum[c]) for c in range(C)]) for b in range(B)])
    net = build_cpnet(state_dict_path=w)
    torch.set_num_threads(16)
    Ly, Lx = so.net_size(H, W)
    cpu_masks, cpu_yf = [], []
    for b in range(B):
        tiles, g = so.make_net_input(corr[b], Ly, Lx)
        with torch.no_grad():
            y = net(torch.from_numpy(tiles)).numpy()
        yf = so.average_tiles(y, g)
        cpu_yf.append(yf)
        cpu_masks.append(so.compute_masks(yf, H, W))
    out = {"size": H, "tiles": [g.by, g.bx, len(g.tiles)], "cpu_objects": [int(m.max()) for m in cpu_masks]}
    for prec in ("f16x3", "bf16", "fp32"):
        seg = Segmenter(dev, H, W, B, weights=w, use_graph=False, precision=prec)
        lab = seg.segment(torch.from_numpy(corr).to(dev.torch_device)).cpu().numpy()
        st = seg.seg_stats()
        yf = seg.yf.cpu().numpy()
        out[prec] = {"stats": [[int(st[b][k]) for k in ("n_moving", "n_seeds", "n_masks", "n_bad_flow", "n_final")]
                               for b in range(B)],
                     "objects": [int(l.max()) for l in lab],
                     "px_diff_vs_cpu": [int((lab[b] != cpu_masks[b]).sum()) for b in range(B)],
                     "max_abs_yf_diff": [float(np.abs(yf[b] - cpu_yf[b]).max()) for b in range(B)]}
        print(prec, json.dumps(out[prec]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
