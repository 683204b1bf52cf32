"""Analysis of the full-resolution follow_flows dynamics on reference-precision (fp32 CPU
network) flows: fixed-point steps, Brent cycle detection (period, detection step) and whether the
cycle shortcut reproduces the full loop (tools/probe/dyn_probe.c).  CPU only."""
import ctypes as ct
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import seg_oracle as so  # noqa: E402
import cpx_oracle as orc  # noqa: E402
from cpx.cpnet import build_cpnet  # noqa: E402
from cpx.synth import synth_fovs, synth_illum  # noqa: E402


def main():
    B = int(os.environ.get("B", "2"))
    H = W = 2080
    torch.set_num_threads(8)
    w = os.path.join(REPO, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
    net = build_cpnet(model="nuclei", state_dict_path=w)
    dtype = os.environ.get("NET", "fp32")
    if dtype == "bf16":
        net = net.to(torch.bfloat16)
    raw = synth_fovs(B, 5, H, W, "cpu", seed=int(os.environ.get("SEED", "77"))).numpy().view(np.uint16).reshape(B, 5, H, W)
    illum = synth_illum(5, H, W, seed=1)
    lib = ct.CDLL(os.path.join(REPO, "tools", "probe", "libdynprobe.so"))
    P = ct.c_void_p
    niter = so.default_niter()
    out = []
    for b in range(B):
        corr = np.stack([orc.illum_correct_producer(raw[b, c], illum[c]) for c in range(5)])
        Ly, Lx = so.net_size(H, W)
        tiles, g = so.make_net_input(corr, Ly, Lx)
        t0 = time.time()
        with torch.no_grad():
            x = torch.from_numpy(tiles)
            y = net(x.to(torch.bfloat16)).float().numpy() if dtype == "bf16" else net(x).numpy()
        yf = so.average_tiles(y, g)
        yfu = so.upsample_flows(yf, H, W)
        dP, cp = yfu[:2], yfu[2] > 0
        dPs = np.ascontiguousarray((dP * cp / np.float32(5.0)).astype(np.float32))
        inds = np.array(np.nonzero(np.abs(dPs[0]) > 1e-3)).T
        py = inds[:, 0].astype(np.float32).copy()
        px = inds[:, 1].astype(np.float32).copy()
        n = py.size
        fix, det, per, ok = (np.zeros(n, np.int32) for _ in range(4))
        t1 = time.time()
        lib.probe(dPs.ctypes.data_as(P), H, W, ct.c_int64(n), niter, py.ctypes.data_as(P), px.ctypes.data_as(P),
                  fix.ctypes.data_as(P), det.ctypes.data_as(P), per.ctypes.data_as(P), ok.ctypes.data_as(P))
        t2 = time.time()
        # effective stop step per pixel: fixed point, else cycle detection, else niter
        stop = np.where(fix >= 0, fix + 1, np.where(det >= 0, det, niter))
        stop_fix_only = np.where(fix >= 0, fix + 1, niter)
        r = {"fov": b, "net": dtype, "n_moving": int(n), "net_s": round(t1 - t0, 1), "probe_s": round(t2 - t1, 1),
             "frac_fixed": float((fix >= 0).mean()), "frac_cycle": float((det >= 0).mean()),
             "frac_neither": float(((fix < 0) & (det < 0)).mean()),
             "cycle_shortcut_all_ok": bool((ok[det >= 0] == 1).all()),
             "mean_steps_fix_only": float(stop_fix_only.mean()), "mean_steps_fix_or_cycle": float(stop.mean()),
             "fix_pct": [int(v) for v in np.percentile(np.where(fix >= 0, fix, niter), [50, 90, 99, 99.9])],
             "det_pct_of_cycled": [int(v) for v in np.percentile(det[det >= 0], [50, 90, 99, 99.9])] if (det >= 0).any() else None,
             "period_counts": {int(k): int(v) for k, v in zip(*np.unique(per[(det >= 0) & (fix < 0)], return_counts=True))}}
        # histogram of remaining (moving) pixels after step s with both exits
        r["remaining_after"] = {s: int((stop > s).sum()) for s in (16, 32, 64, 128, 256, 384, 512, 768, 1024)}
        r["remaining_after_fix_only"] = {s: int((stop_fix_only > s).sum()) for s in (16, 32, 64, 128, 256, 384, 512, 768, 1024)}
        print(json.dumps(r), flush=True)
        out.append(r)
        if os.environ.get("SAVE"):
            np.save(f"/tmp/yf_{dtype}_{b}.npy", yf)


if __name__ == "__main__":
    main()
