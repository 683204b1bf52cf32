"""GPU: the register-resident flow-error screening (k_flowerr_reg.hip) on masks of every register
class and orientation, against the Cellpose restatement (oracle/seg_oracle.py).

fe_reg_class sends a mask to the one-column kernel (both sides <= 64, or one side <= 64 and the
other <= 80: stored transposed when its rows are the longer side), to the column-pair kernels
(columns <= 128 with rows <= 80 / 120) or leaves it to the LDS kernels (a fourth class, four
waves of column pairs for rows <= 160, measured slower than the LDS kernel it relieved and was
dropped; its 153 x 106 shapes stay here as LDS-path cases).  The masks here are sheared
ellipses drawn at network resolution with semi-axes chosen so that, at full resolution (x 100/17),
their bboxes land in each class in both orientations (about 40 x 60 / 60 x 40, 70 x 59, 100 x 70 /
70 x 100, 118 x 94, 153 x 106 / 106 x 153 and 141 x 141 px); each object's flows are scaled so that its flow error falls
on either side of the 0.4 threshold.  The labels must be bit-identical to the oracle's, i.e. every
mask's keep / remove decision equals the fp64 reference's.
"""
import numpy as np
import pytest

import seg_oracle as so
from cpx.segment import make_geom
from test_gpu_seg import _gpu_masks

pytestmark = pytest.mark.gpu

# (ry, rx) at network resolution -> full-resolution bbox ~ (2 ry, 2 rx) x 100 / 17
SHAPES = [(3, 5), (5, 3), (6, 5), (5, 6), (8, 6), (6, 8), (10, 8), (8, 10), (13, 9), (9, 13), (12, 12), (2, 2)]


def _labels(Ly, Lx, seed):
    rng = np.random.default_rng(seed)
    lab = np.zeros((Ly, Lx), np.int32)
    yy = np.arange(Ly)[:, None]
    xx = np.arange(Lx)[None, :]
    step = 30
    k = 0
    for cy in range(18, Ly - 17, step):
        for cx in range(18, Lx - 17, step):
            ry, rx = SHAPES[k % len(SHAPES)]
            shear = int(rng.integers(-2, 3))
            dy = yy - cy
            dx = xx - cx + (shear * dy) // 4
            inside = dy * dy * (rx * rx) + dx * dx * (ry * ry) <= (rx * rx) * (ry * ry)
            k += 1
            lab[inside] = k
    return lab


@pytest.mark.parametrize("seed", [11, 12])
def test_register_classes_decide_like_fp64(dev, seed):
    H = W = 1400
    g = make_geom(H, W)
    lab = _labels(g.Ly, g.Lx, seed)
    assert lab.max() >= 40
    mu = so.masks_to_flows(lab)
    rng = np.random.default_rng(seed)
    scale = np.ones(lab.max() + 1, np.float32)
    scale[1:] = rng.choice(np.float32([0.33, 0.37, 0.40, 0.6, 1.0]), lab.max())
    s = scale[lab]
    yf = np.zeros((3, g.Ly, g.Lx), np.float32)
    yf[0] = 5.0 * mu[0] * s + 0.02 * rng.standard_normal((g.Ly, g.Lx))
    yf[1] = 5.0 * mu[1] * s + 0.02 * rng.standard_normal((g.Ly, g.Lx))
    yf[2] = np.where(lab > 0, 3.0, -3.0)
    got, st = _gpu_masks(dev, yf[None], g, H, W)
    ref = so.compute_masks(yf, H, W)
    np.testing.assert_array_equal(got[0], ref)
    # the masks before the filter reached every register class in both orientations, and the
    # filter removed some (the oracle without the filter: flow_threshold 0)
    pre = so.compute_masks(yf, H, W, flow_threshold=0.0)
    bh, bw = [], []
    for v in range(1, pre.max() + 1):
        ys, xs = np.nonzero(pre == v)
        bh.append(ys.max() - ys.min() + 1)
        bw.append(xs.max() - xs.min() + 1)
    bh, bw = np.array(bh), np.array(bw)
    mn, mx = np.minimum(bh, bw), np.maximum(bh, bw)
    c1 = (mx <= 64) | ((mn <= 64) & (mx <= 80))
    c2 = ~c1 & (mx <= 128) & (mn <= 80)
    c3 = ~c1 & ~c2 & (mx <= 128) & (mn <= 120)
    c4 = ~c1 & ~c2 & ~c3 & (mx <= 160) & (mn <= 128)  # LDS kernels (elongated large masks)
    print("masks per class (1, 2, 3, 4, LDS):", int(c1.sum()), int(c2.sum()), int(c3.sum()), int(c4.sum()),
          int((~c1 & ~c2 & ~c3 & ~c4).sum()), "removed:", int(st[0]["n_bad_flow"]))
    assert c1[bh > bw].any() and c1[bh < bw].any()
    assert c2[bh > bw].any() and c2[bh < bw].any()
    assert c3.any() and c4[bh > bw].any() and c4[bh < bw].any()
    assert st[0]["n_bad_flow"] >= 2 and ref.max() < pre.max()
