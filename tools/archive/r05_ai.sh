# Round 5: the 224^2 persistent convolution with register-resident weights and double-buffered
# tiles (k_conv_x3_p32r, CPX_X3_P32R=1): output hash (must equal 5c491ed9...), CPnet tests,
# one-pipeline kernel traces and two-pipeline benches against the default; then the plate CLI's
# kernel trace (how much its two pipelines overlap on the GPU).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ai
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
print("p32r", os.environ.get("CPX_X3_P32R", "0"), hashlib.sha1(y.cpu().numpy().tobytes()).hexdigest(), flush=True)
PY
timeout -k 10 120 env CPX_X3_P32R=1 python -u /tmp/hash.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 env CPX_X3_P32R=1 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cpnet_x3.py > $O/t_cpnet.log 2>&1
tail -1 $O/t_cpnet.log
cd /tmp && export TMPDIR=/tmp && cd $R
for v in 1 0; do
  timeout -k 10 300 env CPX_X3_P32R=$v rocprofv3 --kernel-trace --output-format csv -d /tmp/kt_$v -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt_$v.log 2>&1
  python tools/prof_summary.py /tmp/kt_$v/run_kernel_trace.csv --steps 4 --md > $O/k_$v.md
  rm -rf /tmp/kt_$v
  grep -E "p32|total" $O/k_$v.md
done
for v in 1 0; do
  timeout -k 10 300 env CPX_X3_P32R=$v python -u bench.py --no-cpu-baseline --steps 60 --stage-steps 1 > $O/bench_$v.log 2>&1
  tail -1 $O/bench_$v.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('p32r',$v,d['value'],d['ms_per_step'],d['stage_ms_per_step']['cpnet'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/pt -o run -- \
  python -u tools/plate_bench.py --fovs 96 --repeat 4 --dir /tmp > $O/pt.log 2>&1
grep '^{"metric"' $O/pt.log
S=$(grep '^{"metric"' $O/pt.log | python -c "import json,sys;print(json.loads(sys.stdin.read())['seconds'])")
python tools/plate_overlap.py /tmp/pt/run_kernel_trace.csv --seconds $S | tee $O/overlap.txt
rm -rf /tmp/pt
echo done
