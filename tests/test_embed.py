"""f3 embeddings: EfficientNetV2-L restated (timm tf_efficientnetv2_l
architecture, parameter count exact), the preprocessing restatement pinned to Pillow, the HIP
preprocessing kernel bit-exact vs the restatement, the native fp16 forward (k_effnet.hip,
cpx.effnet_hip) vs the fp32 PyTorch module on the CPU, and the reference's parquet / CSV layout
(Cellpose_GPU_s3fs.py:326-471)."""
import numpy as np
import pytest
import torch

import embed_oracle as eo
from cpx import effnet


def test_effnet_v2_l_architecture():
    m = effnet.EfficientNetV2L()
    # timm tf_efficientnetv2_l: 118,515,272 parameters with the 1000-class head (1280 x 1000 + 1000)
    assert sum(p.numel() for p in m.parameters()) == 118515272 - 1281000
    assert effnet.count_flops(384) == pytest.approx(71.8e9, rel=2e-3)  # 35.9 GMACs at 384^2


@pytest.mark.parametrize("S,D", [(200, 384), (37, 64), (64, 37), (5, 9)])
def test_bicubic_u8_matches_pillow(S, D):
    from PIL import Image
    rng = np.random.default_rng(S + D)
    img = rng.integers(0, 256, (S, S + 3), dtype=np.uint8)
    img[: S // 3] = 0  # flat and saturated areas (masked crops are mostly 0 outside the cell)
    img[-2:] = 255
    ref = np.array(Image.fromarray(img).convert("RGB").resize((D + 1, D), Image.BICUBIC))
    got = eo.resize_bicubic_u8(img, D, D + 1)
    for c in range(3):
        np.testing.assert_array_equal(got, ref[..., c])


def test_effnet_seeded_forward_is_finite():
    m = effnet.build_effnet(seed=3)
    x = torch.from_numpy(np.stack([eo.pixel_values(np.full((20, 20), 7, np.uint8), 64)] * 2))
    with torch.no_grad():
        y = m(x)
    assert y.shape == (2, 1280) and torch.isfinite(y).all()


@pytest.mark.gpu
def test_preprocess_kernel_bit_exact(dev):
    """cpx_embed_preprocess == the Pillow-pinned restatement, rounded to fp16 (autocast)."""
    from cpx.embed import Embedder
    B, ML, C, S = 2, 3, 2, 200
    rng = np.random.default_rng(11)
    c8 = rng.integers(0, 256, (B, ML, C, S, S), dtype=np.uint8)
    c8[:, :, :, :60] = 0
    emb = Embedder.__new__(Embedder)
    emb.dev, emb.torch, emb.size = dev, torch, 384
    t = torch.from_numpy(c8).to(dev.torch_device)
    idx = [5, 0, 11, 7]
    got = emb.pixel_values(t, idx, S).cpu().numpy()
    flat = c8.reshape(-1, S, S)
    for j, i in enumerate(idx):
        ref = eo.pixel_values(flat[i], 384).astype(np.float16)
        np.testing.assert_array_equal(got[j].view(np.uint16), ref.view(np.uint16))


@pytest.mark.gpu
def test_effnet_fp16_gpu_vs_fp32_cpu(dev):
    """The native fp16 forward (libcpx k_effnet.hip kernels) on the GPU vs the fp32 module on the
    CPU, same weights."""
    m_cpu = effnet.build_effnet(seed=5)
    from cpx.embed import Embedder
    emb = Embedder(dev, seed=5)
    rng = np.random.default_rng(2)
    imgs = [rng.integers(0, 256, (200, 200), dtype=np.uint8) for _ in range(3)]
    x = torch.from_numpy(np.stack([eo.pixel_values(i) for i in imgs]))
    with torch.no_grad():
        ref = m_cpu(x).numpy()
    got = emb.forward(x.to(dev.torch_device).half()).cpu().numpy()
    for a, b in zip(got, ref):
        cos = float(a @ b / np.linalg.norm(a) / np.linalg.norm(b))
        assert cos > 0.999, cos
        assert np.linalg.norm(a - b) / np.linalg.norm(b) < 2e-2


@pytest.mark.gpu
def test_embed_cli_end_to_end(dev, tmp_path):
    """cpx.embed on a small plate: counts CSV, coords, well-aggregated and single-cell parquet in
    the reference's layout; one unreadable site is 'empty' (Cell_Count 0).  (The crops8 feeding
    the embedder are pinned by test_crops_and_scale8_bit_exact, the preprocessing by
    test_preprocess_kernel_bit_exact.)"""
    import os
    import pandas as pd
    import cpx_oracle as orc
    from cpx import embed, tiffio
    from cpx.synth import synth_fovs
    n, C, H, W = 3, 2, 640, 640
    raw = synth_fovs(n, C, H, W, dev.torch_device, seed=21).cpu().numpy().view(np.uint16)
    root = tmp_path / "s3"
    (root / "in").mkdir(parents=True)
    img = tmp_path / "img"
    img.mkdir()
    rows = []
    for f in range(n):
        row = {"Metadata_Plate": "P1", "Metadata_Well": "A01" if f < 2 else "A02", "Metadata_Site": f % 2 + 1,
               "Metadata_Timepoint": 24}
        for c, ch in enumerate(["DNA", "AGP"]):
            name = f"f{f}c{c}.tiff"
            if f != 2:
                tiffio.imwrite(str(img / name), raw[f * C + c])
            row[f"FileName_{ch}"] = name
        rows.append(row)
    pd.DataFrame(rows).to_csv(root / "in" / "ld.csv", index=False)
    out = embed.run(["--bucket_input", "in", "--data_base_path", str(img), "--load_data_key", "ld.csv",
                     "--channels", "DNA", "AGP", "--out_data_path", "res/emb.parquet", "--single_cell",
                     "--save_coords", "--local-root", str(root), "--batch", "2"])
    counts = pd.read_csv(root / "res" / "emb_counts.csv")
    assert counts["Cell_Count"].tolist()[2] == 0 and counts["Cell_Count"].sum() > 0
    coords = pd.read_parquet(root / "res" / "emb_coords.parquet")
    assert len(coords) == counts["Cell_Count"].sum()
    assert coords["Cell_ID"].iloc[0] == "A01_1_cell0"
    well = pd.read_parquet(root / "res" / "emb_well_aggregated.parquet")
    assert well["Metadata_Well"].tolist() == ["A01", "A02"]
    assert np.array(well["mean_features"].iloc[0].tolist()).shape == (C, 1280)
    sc = pd.read_parquet(root / "res" / "emb_single_cell.parquet")
    assert len(sc) == counts["Cell_Count"].sum() and len(sc["single_cell_features"].iloc[0]) == C * 1280
    assert sc["Cell_Index"].tolist()[:2] == [0, 1]
    assert any(p.endswith("_single_cell.parquet") for p in out)


@pytest.mark.gpu
def test_preprocess_table_survives_workspace_regrowth(dev):
    """the bicubic coefficient table lives in a workspace slot that is freed and
    re-allocated when a later call needs more room (more images); the table cache is keyed by
    the slot's allocation generation, so the regrown slot gets the table again even when the
    allocator hands back the same address.  Small N, then a much larger N: both bit-exact."""
    from cpx.embed import Embedder
    S = 200
    rng = np.random.default_rng(12)
    emb = Embedder.__new__(Embedder)
    emb.dev, emb.torch, emb.size = dev, torch, 384
    for n in (1, 24):
        c8 = rng.integers(0, 256, (n, S, S), dtype=np.uint8)
        t = torch.from_numpy(c8).to(dev.torch_device)
        idx = list(range(n))[::-1]
        got = emb.pixel_values(t, idx, S).cpu().numpy()
        for j, i in enumerate(idx):
            ref = eo.pixel_values(c8[i], 384).astype(np.float16)
            np.testing.assert_array_equal(got[j].view(np.uint16), ref.view(np.uint16))


@pytest.mark.parametrize("xgb,filt", [(False, False), (True, True), (True, False)])
def test_assemble_output_layout(tmp_path, xgb, filt):
    """assemble() against the output spec of Cellpose_GPU_s3fs.py:326-471, on hand-made per-site
    results (one empty site, one well with no cell): counts, coords, well means (float32 sums of
    the alive cells in row order / float32 count) and the single-cell explode."""
    import pandas as pd
    from cpx import embed
    C, L = 2, effnet.FEATURE_LENGTH
    rng = np.random.default_rng(4)
    ld = pd.DataFrame({"Metadata_Plate": ["P"] * 5, "Metadata_Well": ["B02", "A01", "B02", "A01", "C03"],
                       "Metadata_Site": [1, 1, 2, 2, 1], "Metadata_Timepoint": [6, 6, 6, 6, 6]},
                      index=[10, 11, 12, 13, 14])
    ncell = {10: 3, 11: 2, 12: 0, 13: 4, 14: 0}
    res = {}
    for i, n in ncell.items():
        if n == 0:
            res[i] = {"status": "empty", "n_cells": 0}
            continue
        res[i] = {"status": "success", "features": rng.standard_normal((n, C, L)).astype(np.float32),
                  "coords": [(int(y), int(x)) for y, x in rng.integers(0, 500, (n, 2))],
                  "is_dead": rng.random(n) < 0.4, "n_cells": n}
    out = str(tmp_path / "o" / "emb.parquet")
    written = embed.assemble(ld, res, ["DNA", "AGP"], out, save_coords=True, single_cell=True,
                             xgb=xgb, filter_dead_cells=filt)
    counts = pd.read_csv(tmp_path / "o" / "emb_counts.csv")
    drop = xgb and filt
    alive = {i: (~res[i]["is_dead"] if drop else np.ones(n, bool)) if n else np.zeros(0, bool)
             for i, n in ncell.items()}
    assert counts["Cell_Count"].tolist() == [int(alive[i].sum()) for i in ld.index]
    if xgb:
        assert counts["Dead_Cells"].tolist() == [int(res[i]["is_dead"].sum()) if ncell[i] else 0 for i in ld.index]
    coords = pd.read_parquet(tmp_path / "o" / "emb_coords.parquet")
    assert coords["Cell_ID"].tolist() == [f"{ld.at[i, 'Metadata_Well']}_{ld.at[i, 'Metadata_Site']}_cell{k}"
                                          for i in ld.index for k in range(ncell[i])]
    wname = "emb_filtered_well_aggregated.parquet" if filt else "emb_well_aggregated.parquet"
    well = pd.read_parquet(tmp_path / "o" / wname)
    assert list(well.columns) == ["Metadata_Well", "Cell_Count", "Metadata_Timepoint", "Metadata_Plate", "mean_features"]
    assert well["Metadata_Well"].tolist() == ["A01", "B02", "C03"]
    for _, r in well.iterrows():
        rows = [i for i in ld.index if ld.at[i, "Metadata_Well"] == r["Metadata_Well"]]
        tot, n = np.zeros((C, L), np.float32), 0
        for i in rows:
            if ncell[i]:
                s = np.zeros((C, L), np.float32)
                for k in np.flatnonzero(alive[i]):
                    s += res[i]["features"][k]
                tot += s
                n += int(alive[i].sum())
        got = np.array(r["mean_features"].tolist(), dtype=np.float64)
        want = (tot / np.float32(n)).astype(np.float64) if n else np.zeros((C, L))
        np.testing.assert_array_equal(got, want)
        assert r["Cell_Count"] == n
    sc = pd.read_parquet(tmp_path / "o" / "emb_single_cell.parquet")
    assert len(sc) == sum(ncell.values()) and "Cell_Count" not in sc.columns
    assert sc.index.tolist() == [i for i in ld.index for _ in range(ncell[i])]
    assert sc["Cell_Index"].tolist() == [k for i in ld.index for k in range(ncell[i])]
    # row 3 = the first cell of the second non-empty site (row 11)
    np.testing.assert_array_equal(np.stack(sc["single_cell_features"].to_numpy())[3], res[11]["features"][0].reshape(-1))
    assert ("is_dead_cell" in sc.columns) == xgb
    assert len(written) == 4
