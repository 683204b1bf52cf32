"""Development: FOV/s of the bench workload with P pipelines on P HIP streams of one GPU
(step i runs on pipeline i % P), to measure how much two batches in flight overlap.

python tools/streams_bench.py [--pipes 2 --steps 16 --batch 16]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))
import torch  # noqa: E402

from cpx.device import Device  # noqa: E402
from cpx.pipeline import FovPipeline, PipelineConfig  # noqa: E402
from cpx.synth import synth_fovs, synth_illum  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pipes", type=int, default=2)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    H = W = 2080
    C, B = 5, a.batch
    w = os.path.join(REPO, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
    illum = synth_illum(C, H, W, seed=1)
    streams = [torch.cuda.Stream() for _ in range(a.pipes)]
    pipes, pools = [], []
    for p in range(a.pipes):
        with torch.cuda.stream(streams[p]):
            dev = Device(0)
            pipes.append(FovPipeline(dev, PipelineConfig(H=H, W=W, C=C, batch=B, weights=w), illum))
            pools.append(synth_fovs(B, C, H, W, dev.torch_device, seed=11 + p))
    torch.cuda.synchronize()

    def run(n):
        pend = []
        for i in range(n):
            p = i % a.pipes
            with torch.cuda.stream(streams[p]):
                slot = pipes[p].run(pools[p])
            pend.append((p, slot))
            if len(pend) > a.pipes:     # fetch the oldest step while the newer ones run
                q, sl = pend.pop(0)
                pipes[q].fetch(sl)
        for q, sl in pend:
            pipes[q].fetch(sl)

    run(2 * a.pipes)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(a.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"pipes {a.pipes}: {a.steps * B / dt:.1f} FOV/s ({dt / a.steps * 1e3:.2f} ms/step)")


if __name__ == "__main__":
    main()
