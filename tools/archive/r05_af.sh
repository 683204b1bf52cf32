# Round 5: every >= 64-channel convolution in the BM 64 tile (CPX_X3_VARIANT=3) now that its tap
# loop is unrolled: output hash vs default, one-pipeline kernel traces, benches.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05af
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
print(os.environ.get("CPX_X3_VARIANT", "default"), hashlib.sha1(y.cpu().numpy().tobytes()).hexdigest(), flush=True)
PY
timeout -k 10 120 python -u /tmp/hash.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 env CPX_X3_VARIANT=3 python -u /tmp/hash.py 2>&1 | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp && cd $R
for v in 0 3; do
  timeout -k 10 300 env CPX_X3_VARIANT=$v rocprofv3 --kernel-trace --output-format csv -d /tmp/kt_$v -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt_$v.log 2>&1
  python tools/prof_summary.py /tmp/kt_$v/run_kernel_trace.csv --steps 4 --md > $O/k_$v.md
  rm -rf /tmp/kt_$v
done
for v in 3 0; do
  timeout -k 10 300 env CPX_X3_VARIANT=$v python -u bench.py --no-cpu-baseline --steps 60 --stage-steps 1 > $O/bench_$v.log 2>&1
  tail -1 $O/bench_$v.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('variant',$v,d['value'],d['ms_per_step'],d['stage_ms_per_step']['cpnet'])"
done
echo done
