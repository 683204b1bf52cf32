"""CPU: the oracle (CPU restatement) against golden vectors produced by the reference itself.

Goldens come from tools/make_golden.py, which imports the reference's Illumination_QC_mult.py,
MaxProjection.py and Cellpose_GPU_s3fs.py (scale_to_8bit) plus scikit-image 0.18.3.
"""
import json
import os

import numpy as np
import pytest

import cpx_oracle as orc
import synth_golden as sg


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name + ".npz"))


def _meta(golden_dir, name):
    with open(os.path.join(golden_dir, name + ".json")) as f:
        return json.load(f)


def _case_img(d, name, kind):
    raw = d[f"{name}_raw"]
    ill = d[f"{name}_illum"] if f"{name}_illum" in d.files else None
    return orc.illum_correct_qc(raw, ill)


def test_qc_small_cases(golden_dir):
    d = _load(golden_dir, "qc_cases")
    meta = _meta(golden_dir, "qc_cases")
    for name, m in meta.items():
        if name == "full":
            continue
        img = _case_img(d, name, m["kind"])
        res = orc.calculate_qc_metrics(img, "CH")
        s, p = res["ImageQuality_PowerLogLogSlope_CH"], res["ImageQuality_PercentMaximal_CH"]
        assert p == m["pct_max"], name  # exact: integer count / n
        if np.isnan(m["slope"]):
            assert np.isnan(s), name
        else:
            assert s == pytest.approx(m["slope"], rel=1e-9, abs=1e-12), name
        ps = orc.rps(img)[2]
        if len(np.atleast_1d(ps)) > 1:
            np.testing.assert_allclose(ps, d[f"{name}_powersum"], rtol=1e-9, atol=0, err_msg=name)


def test_qc_full_size_case(golden_dir):
    meta = _meta(golden_dir, "qc_cases")["full"]
    d = _load(golden_dir, "qc_cases")
    raw, ill = sg.full_case(meta["seed"], meta["H"], meta["W"], meta["C"], meta["n_blobs"])
    for c in range(meta["C"]):
        img = orc.illum_correct_qc(raw[c], ill[c])
        res = orc.calculate_qc_metrics(img, "X")
        exp = meta["channels"][c]
        assert res["ImageQuality_PercentMaximal_X"] == exp["pct_max"]
        assert res["ImageQuality_PowerLogLogSlope_X"] == pytest.approx(exp["slope"], rel=1e-10)
        np.testing.assert_allclose(orc.rps(img)[2], d[f"full_c{c}_powersum"], rtol=1e-9)


def test_max_projection_and_paths(golden_dir):
    d = _load(golden_dir, "maxproj")
    m = _meta(golden_dir, "maxproj")
    planes = [d[f"plane{z}"] for z in range(len(m["keys"]))]
    np.testing.assert_array_equal(orc.max_projection(planes), d["expected"])
    assert orc.modify_imagepath(m["keys"][0]) == m["out_key"]
    for src, dst in m["modify_imagepath"].items():
        assert orc.modify_imagepath(src) == dst
    with pytest.raises(ValueError):
        orc.max_projection([planes[0], planes[1][:10]])


def test_scale_to_8bit(golden_dir):
    d = _load(golden_dir, "scale8")
    k = 0
    while f"in{k}" in d.files:
        np.testing.assert_array_equal(orc.scale_to_8bit(d[f"in{k}"]), d[f"out{k}"])
        k += 1
    assert k >= 5


def test_object_table_matches_regionprops(golden_dir):
    d = _load(golden_dir, "objects_features")
    lab = d["objects_labels"]
    exp = d["objects_table"]
    tab = orc.object_table(lab, box=200)
    assert len(tab) == len(exp)
    for o, e in zip(tab, exp):
        assert o["label"] == int(e[0]) and o["area"] == int(e[1])
        assert tuple(o["bbox"]) == tuple(int(x) for x in e[2:6])
        assert o["centroid"] == (e[6], e[7])  # bit-exact float64 mean
        assert (o["yc"], o["xc"]) == (int(e[8]), int(e[9]))
    kept = [o for o in tab if o["kept"]]
    assert [o["cell_idx"] for o in kept] == list(range(len(kept)))
    assert 0 < len(kept) < len(tab)  # fixture has edge objects


def test_features_match_skimage(golden_dir):
    d = _load(golden_dir, "objects_features")
    got = orc.features(d["feat_labels"], d["feat_planes"])
    exp = d["feat_expected"]
    assert got.shape == exp.shape
    np.testing.assert_allclose(got, exp, rtol=1e-9, atol=1e-12)


def _boundary_case(golden_dir):
    d = np.load(os.path.join(golden_dir, "features_boundary.npz"))
    H, W, C = int(d["H"]), int(d["W"]), int(d["C"])
    lab = sg.boundary_objects(H, W)
    assert int(lab.astype(np.int64).sum()) == int(d["labels_sum"])  # same labels as the generator
    planes = np.stack([sg.plane(700 + c, H, W, n_blobs=40).astype(np.float32) /
                       sg.illum(750 + c, H, W, np.float32) for c in range(C)]).astype(np.float32)
    return lab, planes, d["expected"]


def test_features_boundary_objects_match_skimage(golden_dir):
    """Objects at the feature kernels' fast-path limits (tools/make_golden_bigobj.py)."""
    lab, planes, exp = _boundary_case(golden_dir)
    got = orc.features(lab, planes)
    assert got.shape == exp.shape
    np.testing.assert_allclose(got, exp, rtol=1e-9, atol=1e-12)


def test_synthetic_generator_is_deterministic():
    a = sg.plane(5, 33, 47)
    b = sg.plane(5, 33, 47)
    np.testing.assert_array_equal(a, b)
    assert a.dtype == np.uint16 and (a == 65535).any() or True
    lab = sg.labels(3, 64, 64, n=10)
    assert lab.max() > 0 and lab.dtype == np.int32


def test_expand_labels_matches_skimage(golden_dir):
    d = _load(golden_dir, "objects_features")
    lab = d["expand_labels_in"]
    for dist in (1, 5, 15):
        np.testing.assert_array_equal(orc.expand_labels(lab, dist), d[f"expand_labels_d{dist}"])
    cells, cyto = orc.secondary_objects(lab, 5)
    assert (cyto[lab > 0] == 0).all() and (cyto[(lab == 0)] == cells[lab == 0]).all()
