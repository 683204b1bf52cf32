"""Cellpose's order-dependent fill_holes_and_remove_small_masks for partly absorbed masks.

The reference loop (utils.fill_holes_and_remove_small_masks, reached through cell_model.eval at
/root/reference/Cellpose_GPU_s3fs.py:143; restated literally at oracle/seg_oracle.py:376-391)
walks the masks in label order; a mask lying PARTLY inside an earlier mask's filled holes keeps
the rest of its pixels when they still number >= min_size, is filled and takes the next label,
which renumbers every later mask.  libcpx's parallel fill reproduces the loop only when every
mask is untouched or wholly absorbed at its turn, so k_fill_final checks the absorbed masks and
routes a FOV with a partly absorbed one through k_fill_seq, the loop itself on the GPU
(CPX_SEG_OVF_FILL_PARTIAL, n_fill_partial).

The flows are built so that the dynamics produce chosen masks exactly: every pixel of mask k
carries dP = 5 (T_k - p) for a background target T_k in an empty row, so one Euler step lands it
on T_k (an exact fixed point: the field there is 0) and the histogram seeds one mask per target
(resample=False: dynamics at network resolution, the masks upsampled by nearest neighbour before
the fill, as Cellpose does).  Mask 1 is a one-pixel diamond ring (8-connected, so its inside is a
4-connected hole); mask 2 has pixels on both sides of the ring, touching diagonally across it.
"""
import numpy as np
import pytest

import seg_oracle as so

H = W = 700


def _geom():
    from cpx.segment import make_geom
    return make_geom(H, W)


def _shape(Ly, Lx, case):
    """Net-resolution label image (raster first-occurrence order = label order) and targets."""
    yy, xx = np.mgrid[0:Ly, 0:Lx]
    cy, cx, R = 40, 40, 14
    d = np.abs(yy - cy) + np.abs(xx - cx)
    wedge = (yy - cy >= 2) & (xx - cx >= 2)
    lab = np.zeros((Ly, Lx), np.int32)
    lab[d == R] = 1                                        # the ring (first: its top is row 26)
    if case in ("keep", "small"):
        inner = (d >= R - 4) & (d <= R - 1)
        outer = (d >= R + 1) & (d <= R + (5 if case == "keep" else 1))
        lab[wedge & (inner | outer)] = 2                   # partly inside the ring's hole
    elif case == "hole":
        inner = (d >= R - 4) & (d <= R - 1)
        ring2 = (np.abs(yy - 58) + np.abs(xx - 58) == 4)   # outside the big ring: a small ring
        lab[wedge & inner] = 2
        lab[ring2] = 2                                     # ... whose own hole the remainder fills
    lab[(yy - 95) ** 2 + (xx - 60) ** 2 <= 16] = 3         # a later mask: renumbered by the loop
    lab[(yy - 95) ** 2 + (xx - 90) ** 2 <= 16] = 4
    return lab


def _target(k, targets=None):
    if targets and k in targets:
        return targets[k]
    return 3, 12 + 22 * (k - 1)  # an empty row, targets 22 px apart (beyond the 13 x 13 expansion)


def _jump_yf(lab, targets=None):
    """yf [3, Ly, Lx] whose dynamics reproduce `lab` (module docstring); `targets` overrides the
    default target of some masks (a background pixel in a row without pixels of that mask)."""
    Ly, Lx = lab.shape
    yy, xx = np.mgrid[0:Ly, 0:Lx]
    yf = np.zeros((3, Ly, Lx), np.float32)
    yf[2] = -3.0
    for k in range(1, int(lab.max()) + 1):
        m = lab == k
        ty, tx = _target(k, targets)
        assert lab[ty, tx] == 0 and not (lab[ty] == k).any()
        yf[0][m] = 5.0 * (ty - yy[m])
        yf[1][m] = 5.0 * (tx - xx[m])
        yf[2][m] = 3.0
    return yf


def _oracle(yf, min_size):
    return so.compute_masks(yf, H, W, flow_threshold=0.0, min_size=min_size, resample=False)


CASES = [("keep", 15), ("small", 800), ("hole", 15)]


@pytest.mark.parametrize("case,min_size", CASES)
def test_construction_gives_the_partial_case(case, min_size):
    """CPU: the oracle's masks before the fill are the designed ones, and the reference loop keeps
    ("keep", "hole": renumbering the later masks) or clears ("small") the remainder."""
    g = _geom()
    lab = _shape(g.Ly, g.Lx, case)
    yf = _jump_yf(lab)
    cp = yf[2] > 0
    p, nmov = so.follow_flows(yf[:2], cp, so.default_niter(resample=False))
    m = so.get_masks(p, cp)
    # the dynamics give exactly `lab`, plus each (background) target pixel: get_masks labels
    # every pixel by the seed at its final position, and a non-cell pixel stays where it is
    exp = lab.copy()
    for k in range(1, int(lab.max()) + 1):
        exp[_target(k)] = k
    np.testing.assert_array_equal(m, exp)
    out = _oracle(yf, min_size)
    full = so.resize_nearest(exp, H, W)
    inside = (full == 1) | (out == 1)
    if case == "keep":
        # the remainder of mask 2 (outside the ring) stays and takes label 2; 3 and 4 follow
        assert out.max() == 4
        assert ((out == 2) == ((full == 2) & ~inside)).all()
        assert (out[full == 3] == 3).all() and (out[full == 4] == 4).all()
    elif case == "small":
        # the remainder is below min_size: cleared, no label used; 3 -> 2, 4 -> 3
        assert out.max() == 3
        assert not ((full == 2) & (out != 1) & (out != 0)).any()
        assert (out[full == 3] == 2).all() and (out[full == 4] == 3).all()
    else:
        # the remainder (the small ring) is kept and its own hole filled with its new label
        assert out.max() == 4
        hole2 = (out == 2) & (full == 0)
        assert hole2.sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("case,min_size", CASES)
def test_gpu_partial_fill_bit_exact_vs_oracle(dev, case, min_size):
    """GPU: the FOV with the partly absorbed mask is flagged (n_fill_partial 1), runs the
    sequential fill, and its labels equal the restatement's bit for bit; a clean FOV in the same
    batch keeps the parallel fill (no flag) and is bit-exact too."""
    from cpx.segment import SEG_OVF_FILL_PARTIAL
    from test_gpu_seg import _gpu_masks, _synthetic_yf
    g = _geom()
    yf_p = _jump_yf(_shape(g.Ly, g.Lx, case))
    yf_c, _ = _synthetic_yf(g.Ly, g.Lx, 3)
    yf = np.stack([yf_c, yf_p, yf_c])
    got, st = _gpu_masks(dev, yf, g, H, W, flow_threshold=0.0, min_size=min_size, resample=False)
    ref_p = _oracle(yf_p, min_size)
    ref_c = _oracle(yf_c, min_size)
    np.testing.assert_array_equal(got[1], ref_p)
    assert st[1]["overflow"] & SEG_OVF_FILL_PARTIAL and st[1]["n_fill_partial"] == 1, st[1]
    assert st[1]["n_final"] == ref_p.max()
    for b in (0, 2):
        np.testing.assert_array_equal(got[b], ref_c)
        assert st[b]["overflow"] == 0 and st[b]["n_fill_partial"] == 0
        assert st[b]["n_final"] == ref_c.max()


@pytest.mark.gpu
def test_gpu_wholly_absorbed_mask_keeps_parallel_fill(dev):
    """A mask wholly inside the ring's hole — its target pixel too: get_masks labels the target,
    which would otherwise leave a piece outside — is absorbed without the flag (the parallel fill
    is the reference loop there), bit-exact vs the restatement."""
    from test_gpu_seg import _gpu_masks
    g = _geom()
    lab = _shape(g.Ly, g.Lx, "none")
    yy, xx = np.mgrid[0:g.Ly, 0:g.Lx]
    lab[(np.abs(yy - 40) + np.abs(xx - 40) <= 6) & (yy > 36)] = 5   # wholly inside the hole
    _, inv = np.unique(lab, return_inverse=True)
    lab = inv.reshape(lab.shape).astype(np.int32)
    yf = _jump_yf(lab, targets={4: (30, 40)})  # the inner mask (label 4) -> a hole pixel
    got, st = _gpu_masks(dev, yf[None], g, H, W, flow_threshold=0.0, resample=False)
    ref = _oracle(yf, 15)
    np.testing.assert_array_equal(got[0], ref)
    assert st[0]["overflow"] == 0 and st[0]["n_fill_partial"] == 0
