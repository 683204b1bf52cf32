# Round 5: iglp_opt(0) now default in the single-fragment tap loop; the same hint also in the
# multi-fragment loop and the 224^2 persistent kernel (tools/_var/libcpx_schedall.so): output
# hashes, CPnet tests, one-pipeline kernel traces.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05z
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
print(os.path.basename(os.environ.get("CPX_LIB", "default")), hashlib.sha1(y.cpu().numpy().tobytes()).hexdigest(), flush=True)
PY
timeout -k 10 120 python -u /tmp/hash.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 env CPX_LIB=$R/tools/_var/libcpx_schedall.so python -u /tmp/hash.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cpnet_x3.py > $O/t.log 2>&1
tail -1 $O/t.log
cd /tmp && export TMPDIR=/tmp && cd $R
for L in default schedall; do
  if [ $L = default ]; then e="CPX_X3_NT=1"; else e="CPX_LIB=$R/tools/_var/libcpx_$L.so"; fi
  timeout -k 10 300 env $e rocprofv3 --kernel-trace --output-format csv -d /tmp/kt_$L -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt_$L.log 2>&1
  python tools/prof_summary.py /tmp/kt_$L/run_kernel_trace.csv --steps 4 --md > $O/k_$L.md
  rm -rf /tmp/kt_$L
done
echo done
