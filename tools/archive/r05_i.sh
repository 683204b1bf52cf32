# Round 5: L2 prefetch ("touch") in the f16x3 convolutions.  p32 (224^2 level): this tile's
# residual + the next tile's halo, on/off by CPX_X3_P32_TOUCH; deep k_conv_x3: every later slab's
# halo after the first slab lands (tools/_var/libcpx_touch1.so: single-fragment waves only,
# touch2: all).  Output hash of one CPnet forward per configuration (must agree), then a
# one-pipeline kernel trace per configuration.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05i
mkdir -p $O
cd $R
cat > $O/hash.py <<'PY'
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
print(os.environ.get("CPX_LIB", "default"), os.environ.get("CPX_X3_P32_TOUCH", "1"),
      hashlib.sha1(y.cpu().numpy().tobytes()).hexdigest(), flush=True)
PY
timeout -k 10 120 env CPX_X3_P32_TOUCH=0 python -u $O/hash.py > $O/hash.log 2>&1
timeout -k 10 120 python -u $O/hash.py >> $O/hash.log 2>&1
timeout -k 10 120 env CPX_LIB=$R/tools/_var/libcpx_touch1.so python -u $O/hash.py >> $O/hash.log 2>&1
timeout -k 10 120 env CPX_LIB=$R/tools/_var/libcpx_touch2.so python -u $O/hash.py >> $O/hash.log 2>&1
cat $O/hash.log
cd /tmp && export TMPDIR=/tmp && cd $R
kt() {  # name, then env assignments
  name=$1; shift
  timeout -k 10 300 env "$@" rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$name -o run -- \
    python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt_$name.log 2>&1
  python tools/prof_summary.py $O/kt_$name/run_kernel_trace.csv --steps 4 --md > $O/k_$name.md
  rm -rf $O/kt_$name
}
kt off CPX_X3_P32_TOUCH=0
kt p32 CPX_X3_P32_TOUCH=1
kt t1 CPX_LIB=$R/tools/_var/libcpx_touch1.so
kt t2 CPX_LIB=$R/tools/_var/libcpx_touch2.so
echo done
