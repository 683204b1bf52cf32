# Round 5: (c) z-only convolutions in variant 3 vs all in variant 0 (bit-identical forward, conv
# sums), (d) Cells + Cytoplasm features in one pass (bit-identity tests, the feature parity suite),
# the cpnet_x3 tests, and the bench with the pair path off / on (same box).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05cd
mkdir -p $O
cd $R
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
timeout -k 10 300 python -u - > $O/mix_check.log 2>&1 <<'PY'
import os, sys, torch
sys.path.insert(0, "image-processing-suite_amd")
from cpx.cpnet import build_cpnet
from cpx.cpnet_x3 import FusedCPnetX3
from cpx.device import Device
dev = Device(0)
w = "image-processing-suite_amd/cpx/weights/cpnet_nuclei_synth.pt"
net = build_cpnet(state_dict_path=w if os.path.exists(w) else None)
x = torch.rand(36, 224, 224, 2, device=dev.torch_device)
outs = [FusedCPnetX3(net, dev, variant=0, zvariant=z)(x).clone() for z in (-1, 3)]
torch.cuda.synchronize()
print("mixed forward bit-identical to variant 0:", bool(torch.equal(outs[0], outs[1])), flush=True)
PY
timeout -k 10 300 python -u tools/conv_bench_x3.py --tiles 144 --variants 0 --zvariant -1 > $O/conv_v0.log 2>&1
timeout -k 10 300 python -u tools/conv_bench_x3.py --tiles 144 --variants 0 > $O/conv_mix.log 2>&1
timeout -k 10 600 $T tests/test_gpu_features_pair.py tests/test_gpu_parity.py tests/test_gpu_streams.py tests/test_gpu_cpnet_x3.py > $O/t.log 2>&1
CPX_PAIR_FEATURES=0 CPX_X3_ZVARIANT=-1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_base.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_new.log 2>&1
echo done
