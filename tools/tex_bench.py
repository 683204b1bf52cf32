"""Development timing of the feature stage (cpx_features) on the bench workload.

Runs the pipeline once on a synthetic batch, then times cpx_features per object set with HIP
events; with a -DCPX_GLCM_PROF build (tools/build_variants.sh, CPX_LIB=...) also prints the
k_tex_glcm phase breakdown, with -DCPX_STAGE_PROF the k_obj_stage one.  --dump writes FOV 0's Cells labels + corrected planes (fp16).
"""
import argparse
import ctypes as ct
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))

from cpx.device import Device  # noqa: E402
from cpx.pipeline import OBJECT_SETS, FovPipeline, PipelineConfig  # noqa: E402
from cpx.synth import synth_fovs, synth_illum  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--dump", default=None)
    a = ap.parse_args()
    dev = Device(0)
    td = dev.torch_device
    H = W = 2080
    C = 5
    w = os.path.join(REPO, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
    cfg = PipelineConfig(H=H, W=W, C=C, batch=a.batch, weights=w)
    pipe = FovPipeline(dev, cfg, synth_illum(C, H, W, seed=1))
    raw = synth_fovs(a.batch, C, H, W, td, seed=101)
    pipe.run(raw)
    res = pipe.fetch()
    for s in OBJECT_SETS:
        n = res.hdr[s]["n_objects"]
        areas = np.concatenate([(o["bbox"][:, 2] - o["bbox"][:, 0]) * (o["bbox"][:, 3] - o["bbox"][:, 1])
                                for o in res.objects[s]])
        print(f"{s}: objects/FOV min {n.min()} mean {n.mean():.1f} max {n.max()}; bbox px "
              f"p10 {np.percentile(areas, 10):.0f} p50 {np.percentile(areas, 50):.0f} "
              f"p90 {np.percentile(areas, 90):.0f} max {areas.max()}; > 12288: {(areas > 12288).mean():.2f}")
        # the fallback kernels' share: bbox > 65535 px (texture) or a membership mask over 4096 words
        fb = [int(((o["bbox"][:, 2] - o["bbox"][:, 0]) * (o["bbox"][:, 3] - o["bbox"][:, 1]) > 65535).sum() +
                  ((o["bbox"][:, 2] - o["bbox"][:, 0] + 4) * ((o["bbox"][:, 3] - o["bbox"][:, 1] + 35) // 32)
                   > 4096).sum()) for o in res.objects[s]]
        print(f"{s}: fallback objects per FOV {fb}")
    try:
        prof = dev.lib.cpx_debug_glcm_prof
        prof.argtypes = [ct.c_void_p, ct.c_int]
    except AttributeError:
        prof = None
    try:
        sprof = dev.lib.cpx_debug_stage_prof
        sprof.argtypes = [ct.c_void_p, ct.c_int]
    except AttributeError:
        sprof = None
    buf = (ct.c_ulonglong * 8)()
    sbuf = (ct.c_ulonglong * 8)()
    for s in OBJECT_SETS:
        dev.objects(pipe.labels[s], cfg.max_objects, cfg.box, pipe.lstats, pipe.objects[s], pipe.hdr[s])
        torch.cuda.synchronize()
        if prof:
            prof(buf, 1)
        if sprof:
            sprof(sbuf, 1)
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            dev.features(pipe.labels[s], pipe.corr, C, cfg.max_objects, pipe.objects[s], pipe.hdr[s],
                         pipe.feats[s])
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        line = f"features[{s}] ms: median {np.median(ts):.3f} min {min(ts):.3f}"
        if prof:
            prof(buf, 1)
            items = max(buf[5], 1)
            names = ["reduce", "zero", "count", "scan", "props"]
            line += " | cycles/item " + " ".join(f"{nm}={buf[k] / items:.0f}" for k, nm in enumerate(names))
            line += f" | items {buf[5] // a.reps} px/item {buf[6] / items:.0f} global {buf[7] / items:.2f}"
        if sprof:
            sprof(sbuf, 1)
            objs = max(sbuf[6], 1)
            names = ["queue", "masks", "shape", "reads", "reduce", "crop"]
            line += " | k_obj_stage cycles/object " + " ".join(f"{nm}={sbuf[k] / objs:.0f}" for k, nm in enumerate(names))
            line += f" | objects {sbuf[6] // a.reps} groups/object {sbuf[7] / objs:.0f}"
        print(line)
    if a.dump:
        lab = pipe.labels["Cells"][0].cpu().numpy()
        corr = pipe.corr[0].cpu().numpy().astype(np.float16)
        np.savez_compressed(a.dump, cells=lab, nuclei=pipe.labels["Nuclei"][0].cpu().numpy(),
                            cyto=pipe.labels["Cytoplasm"][0].cpu().numpy(), corr=corr)


if __name__ == "__main__":
    main()
