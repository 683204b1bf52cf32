# Round 5: (1) z-only convolutions in variant 3, (2) Cells + Cytoplasm features in one pass,
# (3) the max-pool fused into each down block's last convolution: bit-identity checks, the
# affected GPU tests, and the bench with all three off / on (same box).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05f
mkdir -p $O
cd $R
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 python -u - > $O/checks.log 2>&1 <<'PY'
import os, sys, torch
sys.path.insert(0, "image-processing-suite_amd")
import cpx.cpnet_x3 as cx
from cpx.cpnet import build_cpnet
from cpx.device import Device
dev = Device(0)
w = "image-processing-suite_amd/cpx/weights/cpnet_nuclei_synth.pt"
net = build_cpnet(state_dict_path=w if os.path.exists(w) else None)
x = torch.rand(36, 224, 224, 2, device=dev.torch_device)
cx.X3_POOL_FUSE = False
ref = cx.FusedCPnetX3(net, dev, variant=0, zvariant=-1)(x).clone()
mix = cx.FusedCPnetX3(net, dev, variant=0, zvariant=3)(x).clone()
cx.X3_POOL_FUSE = True
both = cx.FusedCPnetX3(net, dev)(x).clone()
torch.cuda.synchronize()
print("z-only variant 3 forward bit-identical:", bool(torch.equal(ref, mix)), flush=True)
print("fused-pool + variant-3 forward bit-identical:", bool(torch.equal(ref, both)), flush=True)
PY
timeout -k 10 300 python -u tools/conv_bench_x3.py --tiles 144 --variants 0 > $O/conv.log 2>&1
timeout -k 10 900 $T tests/test_gpu_features_pair.py tests/test_gpu_parity.py tests/test_gpu_streams.py tests/test_gpu_cpnet_x3.py tests/test_gpu_e2e.py > $O/t.log 2>&1
CPX_PAIR_FEATURES=0 CPX_X3_ZVARIANT=-1 CPX_X3_POOL_FUSE=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_base.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_new.log 2>&1
echo done
