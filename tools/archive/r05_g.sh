# Round 5 profile pass: per-kernel durations (one pipeline, back to back), the concurrent run,
# HBM traffic and MFMA passes (tools/profile_round.sh), plus how many Cytoplasm objects share
# their cell's bbox (the cpx_features_pair fast path).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r05g
timeout -k 10 300 python -u - > gpurun_out/r05g/twins.log 2>&1 <<'PY'
import os, sys, numpy as np
sys.path.insert(0, "image-processing-suite_amd")
from cpx import shard
from cpx.device import Device
from cpx.pipeline import FovPipeline, PipelineConfig
from cpx.synth import synth_fovs, synth_illum
dev = Device(0)
w = "image-processing-suite_amd/cpx/weights/cpnet_nuclei_synth.pt"
cfg = PipelineConfig(H=2080, W=2080, C=5, batch=8, weights=w)
p = FovPipeline(dev, cfg, synth_illum(5, 2080, 2080, seed=1))
raw = synth_fovs(8, 5, 2080, 2080, dev.torch_device, seed=shard.fov_seed(shard.plate_fovs(n_wells=384)[0]))
r = p.fetch(p.run(raw))
same = tot = 0; areas = {s: [] for s in ("Nuclei", "Cells", "Cytoplasm")}
for b in range(8):
    cb = {int(o["label"]): tuple(o["bbox"]) for o in r.objects["Cells"][b]}
    for o in r.objects["Cytoplasm"][b]:
        tot += 1; same += cb.get(int(o["label"])) == tuple(o["bbox"])
    for s in areas:
        for o in r.objects[s][b]:
            bb = o["bbox"]; areas[s].append((bb[2] - bb[0]) * (bb[3] - bb[1]))
print("cytoplasm objects sharing the cell bbox:", same, "of", tot)
for s, a in areas.items():
    a = np.array(a); print(s, "objects", len(a), "bbox px percentiles 10/50/90/99:", np.percentile(a, [10, 50, 90, 99]).astype(int).tolist())
PY
PREC=f16x3 bash tools/profile_round.sh
echo done
