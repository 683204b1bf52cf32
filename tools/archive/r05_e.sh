# Round 5: the max-pool fused into each down block's last convolution — the forward must be
# bit-identical to the separate pool kernel; cpnet_x3 / e2e-ID tests; bench with fusion off / on.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05e
mkdir -p $O
cd $R
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 python -u - > $O/pool_check.log 2>&1 <<'PY'
import os, sys, torch
sys.path.insert(0, "image-processing-suite_amd")
import cpx.cpnet_x3 as cx
from cpx.cpnet import build_cpnet
from cpx.device import Device
dev = Device(0)
w = "image-processing-suite_amd/cpx/weights/cpnet_nuclei_synth.pt"
net = build_cpnet(state_dict_path=w if os.path.exists(w) else None)
x = torch.rand(36, 224, 224, 2, device=dev.torch_device)
f = cx.FusedCPnetX3(net, dev)
outs = []
for fuse in (False, True):
    cx.X3_POOL_FUSE = fuse
    outs.append(f(x).clone())
torch.cuda.synchronize()
print("fused-pool forward bit-identical to the separate pool:", bool(torch.equal(outs[0], outs[1])), flush=True)
PY
timeout -k 10 600 $T tests/test_gpu_cpnet_x3.py tests/test_gpu_e2e.py > $O/t.log 2>&1
CPX_X3_POOL_FUSE=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_off.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_on.log 2>&1
echo done
