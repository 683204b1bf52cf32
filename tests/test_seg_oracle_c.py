"""CPU: the C restatement of the segmentation oracle's hot loops (oracle/seg_oracle_c.c) equals
the literal numpy loops of oracle/seg_oracle.py bit for bit, and the full-resolution
(resample=True) defaults are Cellpose's."""
import numpy as np
import pytest

import seg_oracle as so
import synth_golden as sg


def _yf(Ly, Lx, seed, noise=0.05):
    lab = sg.labels(seed, Ly, Lx, n=14, rmin=4, rmax=12, skip_every=0)
    mu = so.masks_to_flows(lab)
    rng = np.random.default_rng(seed)
    yf = np.zeros((3, Ly, Lx), np.float32)
    yf[0] = 5.0 * mu[0] + noise * rng.standard_normal((Ly, Lx))
    yf[1] = 5.0 * mu[1] + noise * rng.standard_normal((Ly, Lx))
    yf[2] = np.where(lab > 0, 3.0, -3.0) + 0.5 * rng.standard_normal((Ly, Lx))
    return yf, lab


def test_default_niter_is_cellpose_run_cp():
    assert so.default_niter("nuclei", 100.0) == 1176      # uint32(1 / 0.17 * 200)
    assert so.default_niter("cyto", 100.0) == 666         # uint32(1 / 0.3 * 200)
    assert so.default_niter("nuclei", 100.0, resample=False) == 200


@pytest.mark.skipif(so.clib() is None, reason="liboracle_seg.so not built")
@pytest.mark.parametrize("seed,niter", [(1, 60), (2, 137)])
def test_follow_flows_c_equals_numpy(seed, niter):
    yf, _ = _yf(90, 110, seed)
    cp = yf[2] > 0
    pn, nn = so.follow_flows(yf[:2], cp, niter, impl="numpy")
    pc, nc = so.follow_flows(yf[:2], cp, niter, impl="c")
    assert nn == nc and nn > 100
    np.testing.assert_array_equal(pn, pc)


@pytest.mark.skipif(so.clib() is None, reason="liboracle_seg.so not built")
def test_flow_error_c_equals_numpy():
    yf, lab = _yf(120, 100, 5, noise=0.4)
    lab[lab == 3] = 0  # an absent label (NaN error, as ndimage.mean of an empty label)
    en = so.flow_errors(lab, yf[:2], impl="numpy")
    ec = so.flow_errors(lab, yf[:2], impl="c")
    np.testing.assert_array_equal(np.isnan(en), np.isnan(ec))
    ok = ~np.isnan(en)
    # ndimage.mean's bincount sums run in raster order in both; equal to the last bit
    np.testing.assert_array_equal(en[ok], ec[ok])


def test_resample_changes_resolution_of_dynamics():
    yf, _ = _yf(60, 64, 9)
    H, W = 300, 320
    m_full = so.compute_masks(yf, H, W, niter=40, impl="numpy")
    m_net = so.compute_masks(yf, H, W, resample=False, impl="numpy")
    assert m_full.shape == m_net.shape == (H, W)
    assert m_full.max() >= 5 and m_net.max() >= 5


def test_upsample_is_cv2_linear_rule():
    # identity at equal size, exact edge clamping and half-pixel centres on a ramp
    x = np.arange(12, dtype=np.float32).reshape(3, 4)
    np.testing.assert_array_equal(so.resize_bilinear(x, 3, 4), x)
    up = so.resize_bilinear(np.array([[0.0, 4.0]], np.float32), 1, 4)
    np.testing.assert_array_equal(up, np.array([[0.0, 1.0, 3.0, 4.0]], np.float32))
