import sys, os, time
sys.path.insert(0, "image-processing-suite_amd")
import torch, numpy as np
from cpx.device import Device
from cpx.synth import synth_fovs, synth_illum
dev = Device(0); td = dev.torch_device
B, C, H, W = 16, 5, 2080, 2080
raw = synth_fovs(B, C, H, W, td, seed=3)
il = torch.from_numpy(synth_illum(C, H, W, seed=1)).to(td)
corr = torch.empty((B, C, H, W), dtype=torch.float32, device=td)
stats, qc = dev.empty_bytes(64 * B * C), dev.empty_bytes(24 * B * C)
dev.illum_correct(raw, il, C, corr, stats)
for _ in range(2): dev.qc_rps(raw, il, C, stats, qc)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5): dev.qc_rps(raw, il, C, stats, qc)
e1.record(); torch.cuda.synchronize()
print("qc_rps ms per 16 FOV:", e0.elapsed_time(e1) / 5)
