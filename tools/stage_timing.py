"""Development timing of the libcpx stages on synthetic full-size FOVs (GPU box).

python tools/stage_timing.py --fovs 8 --iters 5
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from cpx.device import Device, as_numpy, n_features  # noqa: E402
import synth_golden as sg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fovs", type=int, default=8)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--H", type=int, default=2080)
    a = ap.parse_args()
    dev = Device(0)
    B, C, H, W = a.fovs, 5, a.H, a.H
    d = dev.torch_device
    raw1, ill = sg.full_case(7, H, W, C, 300)
    raw = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(raw1, (B,) + raw1.shape)).view(np.int16)).to(d)
    il = torch.from_numpy(ill).to(d)
    lab1 = sg.labels(3, H, W, n=300, rmin=15, rmax=50)
    lab = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(lab1, (B, H, W)))).to(d)
    ML = 512
    corr = torch.empty((B, C, H, W), dtype=torch.float32, device=d)
    stats, qc = dev.empty_bytes(64 * B * C), dev.empty_bytes(24 * B * C)
    lst, obj, hdr = dev.empty_bytes(64 * B * (ML + 1)), dev.empty_bytes(56 * B * ML), dev.empty_bytes(16 * B)
    feats = torch.zeros((B, ML, n_features(C)), dtype=torch.float64, device=d)
    stages = {
        "illum": lambda: dev.illum_correct(raw.view(B * C, H, W), il, C, corr, stats),
        "qc_rps": lambda: dev.qc_rps(raw.view(B * C, H, W), il, C, stats, qc),
        "objects": lambda: dev.objects(lab, ML, 200, lst, obj, hdr),
        "features": lambda: dev.features(lab, corr, C, ML, obj, hdr, feats),
    }
    for name, fn in stages.items():
        fn()
    torch.cuda.synchronize()
    print("objects per FOV:", as_numpy(hdr, "hdr")[0])
    for name, fn in stages.items():
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(a.iters):
            fn()
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / a.iters
        print(f"{name:10s} {ms:8.3f} ms / batch of {B} FOV  -> {ms / B * 1000:8.1f} us/FOV")
    t0 = time.time()
    for _ in range(a.iters):
        for fn in stages.values():
            fn()
    torch.cuda.synchronize()
    dt = (time.time() - t0) / a.iters
    print(f"all stages: {dt * 1e3:.3f} ms/batch -> {B / dt:.1f} FOV/s (no seg)")


if __name__ == "__main__":
    main()
