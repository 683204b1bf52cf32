"""Development probe: does a CU-masked HIP stream (cpx.device.pipeline_streams) work under
rocprofv3's kernel tracer?  Creates two masked streams, runs a torch op on each, synchronises."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "image-processing-suite_amd"))
import torch  # noqa: E402

from cpx.device import pipeline_streams  # noqa: E402

td = torch.device("cuda", 0)
print("env LD_PRELOAD:", os.environ.get("LD_PRELOAD", ""), flush=True)
print("env ROCP*:", sorted(k for k in os.environ if k.startswith("ROCP")), flush=True)
ss = pipeline_streams(td, 2, sys.argv[1] if len(sys.argv) > 1 else "halves")
print("streams", [s.cuda_stream for s in ss], flush=True)
x = torch.ones(1 << 20, device=td)
for s in ss:
    with torch.cuda.stream(s):
        y = x * 2
torch.cuda.synchronize()
print("ok", float(y.sum()), flush=True)
