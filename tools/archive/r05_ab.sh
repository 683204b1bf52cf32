# Round 5: the multi-fragment (BM 64) tap loop unrolled 3 or 9 taps per iteration with iglp_opt(0) (tools/_var/libcpx_mu{3,9}.so): output
# hash, one-pipeline kernel traces against the default; then the 16-byte label loads of
# k_obj_stage's membership masks.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ab
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
timeout -k 10 120 env CPX_LIB=$R/tools/_var/libcpx_mu3.so python -u /tmp/hash.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 env CPX_LIB=$R/tools/_var/libcpx_mu9.so python -u /tmp/hash.py 2>&1 | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp && cd $R
for L in default mu3 mu9; do
  if [ $L = default ]; then e="CPX_X3_NT=1"; else e="CPX_LIB=$R/tools/_var/libcpx_$L.so"; fi
  timeout -k 10 300 env $e rocprofv3 --kernel-trace --output-format csv -d /tmp/kt_$L -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt_$L.log 2>&1
  python tools/prof_summary.py /tmp/kt_$L/run_kernel_trace.csv --steps 4 --md > $O/k_$L.md
  rm -rf /tmp/kt_$L
done
# k_obj_stage membership words from 16-byte label loads (tools/_var/libcpx_mask16.so): feature
# parity with the variant, tex_bench both, kernel trace of the variant
cd $R
timeout -k 10 600 env CPX_LIB=$R/tools/_var/libcpx_mask16.so python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_features_pair.py tests/test_gpu_parity.py tests/test_gpu_capacity.py > $O/t_mask16.log 2>&1
tail -1 $O/t_mask16.log
timeout -k 10 200 python -u tools/tex_bench.py --batch 16 --reps 3 2>&1 | grep "features\[" > $O/tex_def.log
timeout -k 10 200 env CPX_LIB=$R/tools/_var/libcpx_mask16.so python -u tools/tex_bench.py --batch 16 --reps 3 2>&1 | grep "features\[" > $O/tex_mask16.log
cat $O/tex_def.log $O/tex_mask16.log
echo done
