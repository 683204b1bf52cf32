"""Development timing of the native EfficientNetV2-L forward (cpx.effnet_hip on k_effnet.hip):
images/s and TFLOP/s (count_flops) for a batch of 384^2 pixel-value images, beside the
PyTorch/MIOpen fp16-autocast module on the same weights.

python tools/effnet_bench.py [--batch 64] [--reps 3]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))
import torch  # noqa: E402

from cpx import effnet  # noqa: E402
from cpx.device import Device  # noqa: E402
from cpx.effnet_hip import EffNetHip  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--size", type=int, default=effnet.INPUT_SIZE)
    a = ap.parse_args()
    dev = Device(0)
    td = dev.torch_device
    m = effnet.build_effnet(seed=1)
    net = EffNetHip(m, dev)
    x = torch.rand(a.batch, 3, a.size, a.size, device=td).half() * 2 - 1
    ms = timed(lambda: net(x), a.reps)
    flops = effnet.count_flops(a.size) * a.batch
    mt = m.to(td).to(memory_format=torch.channels_last)

    def torch_fwd():
        with torch.no_grad(), torch.autocast(device_type="cuda", dtype=torch.float16):
            return mt(x.contiguous(memory_format=torch.channels_last))
    ms_t = timed(torch_fwd, a.reps)
    a_n, a_t = net(x), torch_fwd().float()
    cos = torch.nn.functional.cosine_similarity(a_n, a_t, dim=1)
    rel = float((a_n - a_t).norm() / a_t.norm())
    spread = float(a_t.std(dim=1).mean() / a_t.abs().mean())  # features not all alike
    print(json.dumps({"batch": a.batch, "size": a.size, "native_ms": round(ms, 3),
                      "native_images_per_s": round(a.batch / ms * 1e3, 1),
                      "native_tflops": round(flops / ms / 1e9, 1), "torch_ms": round(ms_t, 3),
                      "torch_images_per_s": round(a.batch / ms_t * 1e3, 1),
                      "cosine_native_vs_torch_min": round(float(cos.min()), 6),
                      "rel_l2_native_vs_torch": round(rel, 6), "feature_spread": round(spread, 4)}))


if __name__ == "__main__":
    main()
