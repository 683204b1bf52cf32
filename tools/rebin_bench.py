"""Re-binning throughput: G planes 2080^2 -> 1080^2 per call, HIP events
on the launch stream; algorithmic bytes = 2 B read per source pixel + 2 B written per output
pixel.  python tools/rebin_bench.py [--planes 80 --size 2080 --res 1080 --reps 10]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))
import torch  # noqa: E402

from cpx.device import Device  # noqa: E402
from cpx.synth import synth_fovs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--planes", type=int, default=80)
    ap.add_argument("--size", type=int, default=2080)
    ap.add_argument("--res", type=int, default=1080)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cpu", type=int, default=0,
                    help="also time Pillow's own resize (what the reference calls) on this many planes")
    a = ap.parse_args()
    dev = Device(0)
    td = dev.torch_device
    src = synth_fovs(a.planes // 5, 5, a.size, a.size, td, seed=3)
    out = torch.empty((src.shape[0], a.res, a.res), dtype=torch.int16, device=td)
    dev.rebin(src, a.res, a.res, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        dev.rebin(src, a.res, a.res, out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    G = src.shape[0]
    byt = G * (a.size * a.size * 2 + a.res * a.res * 2)
    res = {"planes": G, "ms_per_call": round(ms, 4), "planes_per_s": round(G / ms * 1e3, 1),
           "fovs_per_s_5ch": round(G / 5 / ms * 1e3, 1), "achieved_GBs": round(byt / ms / 1e6, 1),
           "hbm_frac": round(byt / ms / 1e6 / 8000.0, 4)}
    if a.cpu:
        import time
        from PIL import Image
        host = src[:a.cpu].cpu().numpy().view("uint16")
        t0 = time.perf_counter()
        for p in host:
            Image.fromarray(p).resize((a.res, a.res), Image.LANCZOS)
        dt = time.perf_counter() - t0
        res["cpu_pillow"] = {"planes_per_s": round(a.cpu / dt, 2), "cores": 1, "kind": "reference",
                             "sample": f"{a.cpu} planes {a.size}^2 -> {a.res}^2, PIL Image.resize LANCZOS"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
