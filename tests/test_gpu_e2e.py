"""GPU end to end on the headline workload (BASELINE configs[1]: 2080x2080x5ch synthetic FOVs of
the bench's own plate, shipped CPnet weights): FovPipeline vs the CPU restatement, stage by stage
on the same inputs.

  * QC: PercentMaximal exact, PowerLogLogSlope rel 1e-9 (oracle = the reference's arithmetic);
  * segmentation post-processing: seg_oracle.compute_masks (resample=True, niter 1176) fed the
    GPU's own tile-averaged flows gives bit-identical Nuclei labels at 2080^2;
  * Cells / Cytoplasm (marker watershed) bit-identical to ws_oracle.cells_watershed of those
    Nuclei (the sequential heap flood, pinned to skimage 0.18.3);
  * object tables bit-exact and all three feature tables within rtol 1e-5 of cpx_oracle.features;
  * pipeline parity at the reference's precision: with the default CPnet (f16x3) every object ID
    of 8 FOVs of a bench batch equals the fp32 CPU network + the restated dynamics, masks equal up
    to the fp32 rounding-noise floor (a few boundary pixels); two runs bit-identical; the fp32
    (eager) and bf16 variants recorded beside it.
"""
import json
import os

import numpy as np
import pytest
import torch

import cpx_oracle as orc
import seg_oracle as so
import ws_oracle as wo

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def e2e(dev):
    from cpx import shard
    from cpx.pipeline import FovPipeline, PipelineConfig
    from cpx.synth import synth_fovs, synth_illum
    H = W = 2080
    C, B = 5, 2
    weights = os.path.join(REPO, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
    cfg = PipelineConfig(H=H, W=W, C=C, batch=B, weights=weights if os.path.exists(weights) else None)
    illum = synth_illum(C, H, W, seed=1)
    pipe = FovPipeline(dev, cfg, illum)
    first = shard.shard(shard.plate_fovs(n_wells=384), 0, 1)[0]
    raw = synth_fovs(B, C, H, W, dev.torch_device, seed=shard.fov_seed(first))
    slot = pipe.run(raw)
    res = pipe.fetch(slot)
    dev.sync()
    out = dict(cfg=cfg, illum=illum, res=res, pipe=pipe,
               raw=raw.cpu().numpy().view(np.uint16).reshape(B, C, H, W),
               corr=pipe.corr.cpu().numpy(), yf=pipe.seg.yf.cpu().numpy(),
               labels={s: pipe.labels[s].cpu().numpy() for s in ("Nuclei", "Cells", "Cytoplasm")})
    return out


def test_e2e_qc(e2e):
    raw, illum, res = e2e["raw"], e2e["illum"], e2e["res"]
    B, C = raw.shape[:2]
    for b in range(B):
        for c in range(C):
            ref = orc.calculate_qc_metrics(orc.illum_correct_qc(raw[b, c], illum[c]), "x")
            q = res.qc[b * C + c]
            assert q["pct_max"] == ref["ImageQuality_PercentMaximal_x"]
            s = ref["ImageQuality_PowerLogLogSlope_x"]
            assert abs(q["slope"] - s) <= 1e-9 * abs(s)
            np.testing.assert_array_equal(e2e["corr"][b, c], orc.illum_correct_producer(raw[b, c], illum[c]))


def test_e2e_nuclei_bit_exact_on_gpu_flows(e2e):
    H, W = e2e["cfg"].H, e2e["cfg"].W
    for b in range(e2e["yf"].shape[0]):
        ref = so.compute_masks(e2e["yf"][b], H, W)  # resample=True, niter 1176
        got = e2e["labels"]["Nuclei"][b]
        np.testing.assert_array_equal(got, ref, err_msg=f"fov {b}")
        assert ref.max() >= 150  # a realistic FOV: hundreds of nuclei
        assert e2e["res"].seg_stats[b]["n_final"] == ref.max()
        assert e2e["res"].seg_stats[b]["cells_status"] > 0


def test_e2e_cells_cytoplasm_bit_exact(e2e):
    for b in range(e2e["yf"].shape[0]):
        cfg = e2e["cfg"]
        assert cfg.cells == "watershed"
        cells, cyto = wo.cells_watershed(e2e["labels"]["Nuclei"][b], e2e["corr"][b, cfg.ws_channel()],
                                         cfg.cell_expand)
        np.testing.assert_array_equal(e2e["labels"]["Cells"][b], cells)
        np.testing.assert_array_equal(e2e["labels"]["Cytoplasm"][b], cyto)


@pytest.mark.parametrize("objset", ["Nuclei", "Cells", "Cytoplasm"])
def test_e2e_objects_and_features(e2e, objset):
    res = e2e["res"]
    for b in range(e2e["yf"].shape[0]):
        lab = e2e["labels"][objset][b]
        tab = orc.object_table(lab, e2e["cfg"].box)
        got = res.objects[objset][b]
        assert [t["label"] for t in tab] == list(got["label"])
        assert [t["yc"] for t in tab] == list(got["yc"]) and [t["xc"] for t in tab] == list(got["xc"])
        ref = orc.features(lab, e2e["corr"][b])
        np.testing.assert_allclose(res.feats[objset][b], ref, rtol=1e-5, atol=1e-9)


def _agreement(a, b):
    """Objects of label image a vs b: identical pixel set AND label; one-to-one matches by
    IoU >= 0.5 (with the matched label's id equal or not) and their mean IoU."""
    ids = np.unique(a[a > 0])
    same = matched = same_id = 0
    ious = []
    for l in ids:
        m = a == l
        if np.array_equal(m, b == l):
            same += 1
        cand = b[m]
        cand = cand[cand > 0]
        if cand.size == 0:
            continue
        k = np.bincount(cand).argmax()
        mb = b == k
        iou = np.logical_and(m, mb).sum() / np.logical_or(m, mb).sum()
        if iou >= 0.5:
            matched += 1
            same_id += int(k == l)
            ious.append(iou)
    n = max(len(ids), 1)
    return {"objects": int(len(ids)), "identical_mask_and_id": int(same), "fraction_identical": same / n,
            "matched_iou50": int(matched), "fraction_matched": matched / n,
            "matched_same_id": int(same_id), "mean_iou_matched": float(np.mean(ious)) if ious else 0.0}


@pytest.fixture(scope="module")
def ids8(dev):
    """8 FOVs of the bench plate through the default pipeline (CPnet f16x3) twice, and the same
    FOVs through Cellpose's CPnet in fp32 on the CPU followed by the restated dynamics."""
    from cpx import shard
    from cpx.cpnet import build_cpnet
    from cpx.pipeline import FovPipeline, PipelineConfig
    from cpx.synth import synth_fovs, synth_illum
    H = W = 2080
    C, B = 5, 8
    weights = os.path.join(REPO, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
    cfg = PipelineConfig(H=H, W=W, C=C, batch=B, weights=weights if os.path.exists(weights) else None)
    assert cfg.cpnet_precision == "f16x3"
    illum = synth_illum(C, H, W, seed=1)
    pipe = FovPipeline(dev, cfg, illum)
    mine = shard.shard(shard.plate_fovs(n_wells=384), 0, 1)
    raw = synth_fovs(B, C, H, W, dev.torch_device, seed=shard.fov_seed(mine[0]) + 7919)  # bench batch 1
    runs = []
    for _ in range(2):
        pipe.fetch(pipe.run(raw))
        dev.sync()
        runs.append(pipe.labels["Nuclei"].cpu().numpy().copy())
    corr = pipe.corr.cpu().numpy()
    del pipe
    torch.set_num_threads(16)
    net = build_cpnet(seed=cfg.seed, model=cfg.model, state_dict_path=cfg.weights)
    Ly, Lx = so.net_size(H, W, cfg.model, cfg.diameter)
    cpu = []
    for b in range(B):
        tiles, g = so.make_net_input(corr[b], Ly, Lx)
        with torch.no_grad():
            y = net(torch.from_numpy(tiles)).numpy()
        cpu.append(so.compute_masks(so.average_tiles(y, g), H, W))
    return dict(runs=runs, cpu=cpu, corr=corr, cfg=cfg)


# rounding-noise floor of the reference itself: Cellpose's CPnet in fp32 vs in fp64 on the CPU,
# each followed by the restated dynamics, flips ~0.2 boundary pixels per 2080^2 FOV (1 pixel in
# 5 FOVs, tools/precision_floor.py); any two fp32 implementations of the network
# differ at that rate.  The bar below: every object ID identical, masks identical up to a few
# such boundary pixels.
MAX_FLIPPED_PIXELS_PER_FOV = 8


@pytest.mark.timeout(900)
def test_e2e_object_ids_identical_to_fp32_cpu(ids8):
    """north_star's bar: object IDs identical to the CPU path.  The reference runs the U-Net in
    fp32 (Cellpose_GPU_s3fs.py:108,143); with the default CPnet precision (f16x3, native
    split-fp16 MFMA kernels) every object of 8 FOVs of a bench batch keeps its ID (same count,
    same label, IoU >= 0.5 one-to-one) against the fp32 CPU network + the restated dynamics, and
    at most MAX_FLIPPED_PIXELS_PER_FOV boundary pixels differ (the fp32 rounding-noise floor;
    recorded in gpurun_out/e2e_seg_agreement.json)."""
    rows = []
    for b, m_cpu in enumerate(ids8["cpu"]):
        got = ids8["runs"][0][b]
        r = {"fov": b, "objects": int(m_cpu.max()), "f16x3_gpu_vs_fp32_cpu": _agreement(m_cpu, got),
             "pixels_differing": int((got != m_cpu).sum())}
        rows.append(r)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "e2e_seg_agreement.json"), "w") as f:
        json.dump(rows, f, indent=1)
    print(json.dumps(rows))
    for b, r in enumerate(rows):
        a = r["f16x3_gpu_vs_fp32_cpu"]
        assert r["objects"] >= 150
        assert int(ids8["runs"][0][b].max()) == r["objects"], r
        assert a["matched_same_id"] == a["objects"] == r["objects"], r
        assert r["pixels_differing"] <= MAX_FLIPPED_PIXELS_PER_FOV, r


def test_e2e_default_cpnet_deterministic(ids8):
    """Two runs of the default pipeline on one batch: bit-identical masks (no float atomics in
    the CPnet or the dynamics)."""
    np.testing.assert_array_equal(ids8["runs"][0], ids8["runs"][1])


@pytest.mark.timeout(600)
def test_e2e_other_precisions_recorded(ids8, dev):
    """The named variants beside the default, recorded against the same fp32-CPU masks
    (gpurun_out/e2e_seg_agreement_variants.json): "fp32" (the eager PyTorch/MIOpen module — an
    independent fp32 implementation, so its boundary-pixel flips show the fp32 noise floor on the
    GPU) and "bf16" (native bf16 kernels: boundary pixels and IDs move).  Bar for bf16: >= 90 % of
    the objects matched one-to-one (IoU >= 0.5); fp32: every ID kept, as the default."""
    from cpx.segment import Segmenter
    cfg = ids8["cfg"]
    H, W, B = cfg.H, cfg.W, len(ids8["cpu"])
    out = {}
    for prec in ("fp32", "bf16"):
        seg = Segmenter(dev, H, W, B, model=cfg.model, diameter=cfg.diameter, weights=cfg.weights, seed=cfg.seed,
                        use_graph=False, max_objects=cfg.max_objects, precision=prec)
        lab = seg.segment(torch.from_numpy(ids8["corr"]).to(dev.torch_device)).cpu().numpy()
        del seg
        out[prec] = [dict(_agreement(m, lab[b]), pixels_differing=int((lab[b] != m).sum()))
                     for b, m in enumerate(ids8["cpu"])]
    with open(os.path.join(REPO, "gpurun_out", "e2e_seg_agreement_variants.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: [(r["pixels_differing"], r["matched_same_id"], r["objects"]) for r in v] for k, v in out.items()}))
    for r in out["bf16"]:
        assert r["fraction_matched"] >= 0.9, r
    for r in out["fp32"]:
        assert r["matched_same_id"] == r["objects"], r


def test_e2e_csv_tables(e2e, tmp_path):
    """north_star's CSV parity: the four result tables (Image / Nuclei / Cells / Cytoplasm, as
    Pycyto_pertime.py reads them) written from the GPU results vs written from the CPU pipeline
    (oracle/cpu_pipeline.run_fov) on the same raw FOV and the GPU's own flows.  ObjectNumber /
    ImageNumber columns and counts identical, PercentMaximal exact, PowerLogLogSlope rel 1e-9,
    every feature column within rtol 1e-5."""
    import pandas as pd
    import cpu_pipeline
    from csv_tables import cpu_tables, gpu_tables
    cfg, res = e2e["cfg"], e2e["res"]
    for b in range(e2e["yf"].shape[0]):
        ref = cpu_pipeline.run_fov(e2e["raw"][b], e2e["illum"], None, cell_expand=cfg.cell_expand,
                                   cell_channel=cfg.ws_channel(), flows=e2e["yf"][b])
        dirs = {}
        for side, t in (("cpu", cpu_tables(ref, image_number=b + 1)), ("gpu", gpu_tables(res, b, image_number=b + 1))):
            dirs[side] = t.write(str(tmp_path / side), "P01", 24)
        for name in ("Image", "Nuclei", "Cells", "Cytoplasm"):
            c = pd.read_csv(os.path.join(dirs["cpu"], f"{name}.csv"))
            g = pd.read_csv(os.path.join(dirs["gpu"], f"{name}.csv"))
            assert list(c.columns) == list(g.columns), name
            assert len(c) == len(g) and len(c) > 0, (name, len(c), len(g))
            exact = [k for k in c.columns if k in ("ImageNumber", "ObjectNumber", "Number_Object_Number")
                     or k.startswith(("Count_", "ImageQuality_PercentMaximal", "Metadata_"))]
            for k in exact:
                assert (c[k].to_numpy() == g[k].to_numpy()).all(), (name, k)
            rest = [k for k in c.columns if k not in exact]
            rtol = 1e-9 if name == "Image" else 1e-5
            np.testing.assert_allclose(g[rest].to_numpy(np.float64), c[rest].to_numpy(np.float64),
                                       rtol=rtol, atol=1e-9, err_msg=name)
