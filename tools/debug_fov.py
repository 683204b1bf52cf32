"""Debug: FovSession submit after a batch pipeline run in the same process."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "image-processing-suite_amd"))
import numpy as np
import torch
from cpx.fov import FovSession
from cpx.device import Device
from cpx.pipeline import FovPipeline, PipelineConfig
from cpx.synth import synth_fovs
s = FovSession(0)
p = np.random.default_rng(0).integers(0, 5000, (64, 80), dtype=np.uint16)
s.submit([p], C=1); print("submit 1 ok", s.qc())
dev = Device(0)
cfg = PipelineConfig(H=384, W=416, C=2, batch=2)
pipe = FovPipeline(dev, cfg, None)
pipe.raw.copy_(synth_fovs(2, 2, 384, 416, dev.torch_device, seed=5))
pipe.run(); pipe.fetch(); print("pipeline ok")
print("current stream", torch.cuda.current_stream().cuda_stream)
try:
    s.submit([p], C=1); print("submit 2 ok", s.qc())
except Exception as e:
    print("submit 2 failed:", e)
del pipe, dev
import gc; gc.collect()
try:
    s.submit([p], C=1); print("submit 3 ok", s.qc())
except Exception as e:
    print("submit 3 failed:", e)
