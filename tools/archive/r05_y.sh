# Round 5: scheduling hints in the single-fragment conv tap loop (tools/_var/libcpx_sched{1,2}.so:
# iglp_opt(0), or sched_group_barrier groups that issue the next tap's fragment reads before this
# tap's MFMAs): CPnet output hash per library (must agree), one-pipeline kernel traces, benches.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05y
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
for L in default sched1 sched2; do
  if [ $L = default ]; then e=""; else e="CPX_LIB=$R/tools/_var/libcpx_$L.so"; fi
  timeout -k 10 120 env $e python -u /tmp/hash.py 2>&1 | grep -v amdgpu.ids
done
cd /tmp && export TMPDIR=/tmp && cd $R
for L in default sched1 sched2; do
  if [ $L = default ]; then e="CPX_X3_NT=1"; else e="CPX_LIB=$R/tools/_var/libcpx_$L.so"; fi
  timeout -k 10 300 env $e rocprofv3 --kernel-trace --output-format csv -d /tmp/kt_$L -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt_$L.log 2>&1
  python tools/prof_summary.py /tmp/kt_$L/run_kernel_trace.csv --steps 4 --md > $O/k_$L.md
  rm -rf /tmp/kt_$L
done
for L in default sched2 sched1; do
  if [ $L = default ]; then e="CPX_X3_NT=1"; else e="CPX_LIB=$R/tools/_var/libcpx_$L.so"; fi
  timeout -k 10 300 env $e python -u bench.py --no-cpu-baseline --steps 60 --stage-steps 1 > $O/bench_$L.log 2>&1
  tail -1 $O/bench_$L.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$L',d['value'],d['ms_per_step'],d['stage_ms_per_step']['cpnet'])"
done
echo done
