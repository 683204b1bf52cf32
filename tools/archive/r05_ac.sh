# Round 5: defaults now unroll the BM 64 tap loop (CIN >= 64) and build the membership masks
# from 16-byte label loads: output hash, CPnet / features / seg tests, kernel trace, bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ac
mkdir -p $O
cd $R
cat > /tmp/hash.py <<'PY'
import hashlib, os, sys
sys.path.insert(0, "image-processing-suite_amd")
import torch
from cpx.cpnet import build_cpnet
from cpx.cpnet_x3 import FusedCPnetX3
from cpx.device import Device
dev = Device(0)
torch.manual_seed(0)
net = build_cpnet(state_dict_path="image-processing-suite_amd/cpx/weights/cpnet_nuclei_synth.pt")
x = torch.rand(24, 224, 224, 2).to(dev.torch_device)
y = FusedCPnetX3(net, dev)(x)
dev.sync()
print("hash", hashlib.sha1(y.cpu().numpy().tobytes()).hexdigest(), flush=True)
PY
timeout -k 10 120 python -u /tmp/hash.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cpnet_x3.py tests/test_gpu_features_pair.py tests/test_gpu_parity.py tests/test_gpu_e2e.py > $O/t.log 2>&1
tail -1 $O/t.log
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt -o run -- \
  python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt.log 2>&1
python tools/prof_summary.py /tmp/kt/run_kernel_trace.csv --steps 4 --md > $O/kernels_steady.md
rm -rf /tmp/kt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 60 --stage-steps 1 > $O/bench.log 2>&1
tail -1 $O/bench.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('bench',d['value'],d['ms_per_step'],d['stage_ms_per_step'])"
echo done
