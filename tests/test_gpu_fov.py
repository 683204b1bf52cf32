"""Per-FOV drop-in boundary (include/cpx.h "per-FOV drop-in boundary", cpx/fov.py, cpx/qc.py)
against the reference's own outputs (tests/golden/*) and the batch kernels."""
import json
import os

import numpy as np
import pandas as pd
import pytest

import synth_golden as sg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sess():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cpx import qc
    return qc.session()  # the CLI's process-wide session


@pytest.mark.parametrize("batch", [1, 2, 16])
def test_qc_cli_matches_reference_csv(sess, golden_dir, tmp_path, batch):
    """cpx.qc.main on the LoadData fixture == the reference CLI's CSV (same rows, columns,
    error strings; slopes to 1e-9 relative, PercentMaximal exactly), whether the sites go to the
    GPU one per call or batched (the fixture mixes clean sites with missing planes)."""
    from cpx import qc
    d = os.path.join(golden_dir, "qc_cli")
    out = tmp_path / "qc.csv"
    qc.main(["--load-data", os.path.join(d, "load_data.csv"), "--data-path", os.path.join(d, "images"),
             "--illum-path", os.path.join(d, "illum"), "--channels", "DNA", "AGP", "Mito",
             "--output", str(out), "--threads", "3", "--batch", str(batch)])
    got = pd.read_csv(out, float_precision="round_trip")
    exp = pd.read_csv(os.path.join(d, "expected_qc.csv"), float_precision="round_trip")
    assert list(got.columns) == list(exp.columns)
    assert len(got) == len(exp)
    for c in exp.columns:
        if c.startswith("ImageQuality_PowerLogLogSlope_"):
            np.testing.assert_allclose(got[c].to_numpy(float), exp[c].to_numpy(float), rtol=1e-9,
                                       equal_nan=True, err_msg=c)
        elif c.startswith("ImageQuality_PercentMaximal_"):
            np.testing.assert_array_equal(got[c].to_numpy(float), exp[c].to_numpy(float), err_msg=c)
        else:
            assert got[c].fillna("").astype(str).tolist() == exp[c].fillna("").astype(str).tolist(), c


def test_calculate_qc_metrics_float_image(sess, golden_dir):
    """calculate_qc_metrics(float image) (CPX_DTYPE_IMAGE_F64 path) vs the reference's values."""
    from cpx import qc
    arrays = np.load(os.path.join(golden_dir, "qc_cases.npz"))
    meta = json.load(open(os.path.join(golden_dir, "qc_cases.json")))
    n = 0
    for name, m in meta.items():
        if name == "full" or f"{name}_raw" not in arrays:
            continue
        raw = arrays[f"{name}_raw"].astype(np.float64)
        ill = arrays[f"{name}_illum"] if f"{name}_illum" in arrays else None
        img = raw / ill if ill is not None else raw
        res = qc.calculate_qc_metrics(img, "X")
        exp_s, exp_p = m["slope"], m["pct_max"]
        got_s = res["ImageQuality_PowerLogLogSlope_X"]
        if exp_s is None or (isinstance(exp_s, float) and np.isnan(exp_s)):
            assert np.isnan(got_s), name
        else:
            assert got_s == pytest.approx(exp_s, rel=1e-9, abs=1e-12), name
        np.testing.assert_equal(res["ImageQuality_PercentMaximal_X"], exp_p, err_msg=name)
        n += 1
    assert n > 0


def test_fov_zmax_and_tiff_match_reference(sess, golden_dir):
    """cpx_fov_submit(Z planes) + cpx_fov_read_plane + cpx.tiffio == the reference's max
    projection TIFF byte for byte (MaxProjection.max_projection golden)."""
    from cpx import tiffio
    d = np.load(os.path.join(golden_dir, "maxproj.npz"))
    planes = [d[f"plane{z}"] for z in range(5)]
    sess.set_illum(0, None)
    sess.submit(planes, C=1, Z=5)
    got = sess.read_plane(0)
    np.testing.assert_array_equal(got, d["expected"])
    assert tiffio.imwrite_bytes(got) == d["expected_tiff"].tobytes()


def test_fov_zmax_plane_major_channels(sess):
    """planes[z*C + c] order (MaxProjection.py chunk order) with C=3, Z=4."""
    C, Z, H, W = 3, 4, 40, 56
    planes = [sg.plane(700 + k, H, W, n_blobs=3) for k in range(C * Z)]
    for c in range(C):
        sess.set_illum(c, None)
    sess.submit(planes, C=C, Z=Z)
    for c in range(C):
        exp = np.maximum.reduce([planes[z * C + c] for z in range(Z)])
        np.testing.assert_array_equal(sess.read_plane(c), exp)


def test_fov_objects_and_features_match_batch(sess, dev):
    """Per-FOV tables == the batch kernels on the same planes and labels."""
    import torch
    from cpx.device import as_numpy, n_features
    C, H, W = 2, 300, 320
    planes = [sg.plane(800 + c, H, W, n_blobs=20) for c in range(C)]
    ill = [sg.illum(850 + c, H, W, np.float32) for c in range(C)]
    lab = sg.labels(61, H, W, n=25, rmin=4, rmax=30, skip_every=0)
    for c in range(C):
        sess.set_illum(c, ill[c])
    sess.submit(planes, C=C)
    ml = 64
    objs = sess.object_table(lab, box=60, max_objects=ml)
    feats = sess.features(lab, max_objects=ml)
    # batch path
    td = dev.torch_device
    raw = torch.from_numpy(np.stack(planes).view(np.int16)).to(td)
    illum = torch.from_numpy(np.stack(ill)).to(td)
    corr = torch.empty((C, H, W), dtype=torch.float32, device=td)
    stats = dev.empty_bytes(64 * C)
    dev.illum_correct(raw, illum, C, corr, stats)
    labt = torch.from_numpy(lab.astype(np.int32)).to(td)[None]
    lstats = dev.empty_bytes(64 * (ml + 1))
    ob = dev.empty_bytes(56 * ml)
    hdr = dev.empty_bytes(16)
    dev.objects(labt, ml, 60, lstats, ob, hdr)
    fb = torch.zeros((1, ml, n_features(C)), dtype=torch.float64, device=td)
    dev.features(labt, corr[None], C, ml, ob, hdr, fb)
    dev.sync()
    n = int(as_numpy(hdr, "hdr")[0]["n_objects"])
    assert len(objs) == n == len(feats)
    exp_o = as_numpy(ob, "object")[:n]
    for f in ("label", "area", "bbox", "yc", "xc", "kept", "cell_idx"):
        np.testing.assert_array_equal(objs[f], exp_o[f], err_msg=f)
    np.testing.assert_array_equal(feats, fb.cpu().numpy()[0, :n])


def test_fov_illum_shape_mismatch_uses_raw(sess):
    """An illum of another shape is ignored for that FOV (Illumination_QC_mult.py:148-153)."""
    H, W = 64, 80
    p = sg.plane(900, H, W, n_blobs=4)
    sess.set_illum(0, sg.illum(901, H + 8, W, np.float64))
    sess.submit([p], C=1)
    s1, p1, _ = sess.qc()
    sess.set_illum(0, None)
    sess.submit([p], C=1)
    s2, p2, _ = sess.qc()
    assert s1[0] == s2[0] and p1[0] == p2[0]
