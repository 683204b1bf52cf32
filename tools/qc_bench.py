"""Development timing of cpx_qc_rps (ImageQuality_PowerLogLogSlope) alone on the bench's plane
batch: N FOVs x C channels of H x W synthetic uint16 planes with an fp32 flat-field, one
cpx_illum_correct for the plane statistics, then `reps` cpx_qc_rps calls between HIP events.

python tools/qc_bench.py [--fovs 48] [--reps 10]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))
import torch  # noqa: E402

from cpx.device import Device  # noqa: E402
from cpx.synth import synth_fovs, synth_illum  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fovs", type=int, default=48)
    ap.add_argument("--C", type=int, default=5)
    ap.add_argument("--H", type=int, default=2080)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = Device(0)
    td = dev.torch_device
    C, H = a.C, a.H
    raw = synth_fovs(a.fovs, C, H, H, td, seed=3).reshape(a.fovs * C, H, H)
    illum = torch.from_numpy(synth_illum(C, H, H, seed=1)).to(td)
    n = a.fovs * C
    stats = dev.empty_bytes(64 * n)
    qc = dev.empty_bytes(24 * n)
    corr = torch.empty((n, H, H), dtype=torch.float32, device=td)
    dev.illum_correct(raw, illum, C, corr, stats)
    del corr
    dev.qc_rps(raw, illum, C, stats, qc)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        dev.qc_rps(raw, illum, C, stats, qc)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    print(f"cpx_qc_rps: {n} planes of {H}x{H}: {ms:.3f} ms per call ({ms / a.fovs * 48:.3f} ms per 48 FOVs)")


if __name__ == "__main__":
    main()
