"""GPU: the GLCM work split of k_texture.hip against the oracle (skimage 0.18.3 greycomatrix /
greycoprops restated, cpx_oracle.features; rtol 1e-5 as every feature test).

k_tex_band counts an item's pairs in a band table (both values non-zero and |j - i| <= 31, plus
the (0, j) and (i, 0) rows) and lists the other pairs as outliers, up to 512 keys per angle; an
item whose list overflows is re-measured by the dense-table kernel k_tex_glcm.  The objects here
are built so that each path is taken, which the test checks on the host with the same
classification: smooth blobs (band only), blobs with a sharp intensity step inside (a few hundred
outlier pairs: the list), and uniform noise (thousands of outliers: the dense kernel).
"""
import numpy as np
import pytest
import scipy.ndimage as ndi

import cpx_oracle as orc

pytestmark = pytest.mark.gpu

OFFS = [(0, 3), (2, 2), (3, 0), (2, -2)]
BAND_D, OUT_CAP = 31, 512


def _outliers(q8):
    """Per angle: pairs with both values non-zero and |j - i| > BAND_D (k_tex_band's outliers)."""
    h, w = q8.shape
    out = []
    for dr, dc in OFFS:
        r1 = h - dr
        c0, c1 = (0, w - dc) if dc >= 0 else (-dc, w)
        a = q8[:r1, c0:c1].astype(int)
        b = q8[dr:dr + r1, c0 + dc:c1 + dc].astype(int)
        out.append(int(((a > 0) & (b > 0) & (np.abs(a - b) > BAND_D)).sum()))
    return out


def _scene(kind, H=300, W=320, seed=0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W]
    lab = np.zeros((H, W), np.int32)
    plane = np.full((H, W), 300.0)
    centres = [(60, 70), (70, 220), (200, 90), (210, 240)]
    for k, (cy, cx) in enumerate(centres):
        r2 = ((yy - cy) / 45.0) ** 2 + ((xx - cx + 0.3 * (yy - cy)) / 38.0) ** 2
        m = r2 <= 1.0
        lab[m] = k + 1
        plane += 5000.0 * np.exp(-2.0 * r2)
        if kind == "step":  # a sharp step across the object: a band of large |i - j| pairs
            plane += np.where(m & (xx > cx), 6000.0, 0.0)
    if kind == "noise":
        plane = np.where(lab > 0, rng.uniform(100.0, 20000.0, (H, W)), plane)
    plane += rng.normal(0.0, 15.0, (H, W))
    planes = np.stack([plane, plane[::-1, ::-1].copy()]).astype(np.float32)
    return lab, planes


@pytest.mark.parametrize("kind", ["smooth", "step", "noise"])
def test_glcm_paths_match_oracle(dev, kind):
    from test_gpu_parity import _feat_close, _features
    lab, planes = _scene(kind)
    outl = []
    for i, sl in enumerate(ndi.find_objects(lab)):
        for c in range(planes.shape[0]):
            outl.append(_outliers(orc.texture_input(planes[c], lab, sl, i + 1)))
    outl = np.array(outl)
    if kind == "smooth":
        assert outl.max() == 0
    elif kind == "step":
        assert outl.max() > 0 and outl.max() <= OUT_CAP, outl
    else:
        assert (outl.max(axis=1) > OUT_CAP).all(), outl
    got = _features(dev, lab, planes)
    _feat_close(got, orc.features(lab, planes))


def test_glcm_mixed_batch_paths_match_oracle(dev):
    """The three kinds in one label image (one launch: band items, list items and redo items
    interleaved in the queues), and a second call on the same context (the redo list and the
    outlier counters start from zero again)."""
    from test_gpu_parity import _feat_close, _features
    parts = [_scene(k, seed=i) for i, k in enumerate(("smooth", "step", "noise"))]
    lab = np.concatenate([p[0] + (p[0] > 0) * 4 * i for i, p in enumerate(parts)], axis=1).astype(np.int32)
    planes = np.concatenate([p[1] for p in parts], axis=2)
    exp = orc.features(lab, planes)
    for _ in range(2):
        _feat_close(_features(dev, lab, planes), exp)
