"""CPU restatement of the Cellpose (<= v3, U-Net) evaluation path used by the reference —
TEST INFRASTRUCTURE ONLY ("parity unpinned" against real Cellpose).

The reference calls ``models.CellposeModel(model_type='nuclei').eval(image_hwc, diameter=100)``
(Cellpose_GPU_s3fs.py:28,108,143) with every other argument at its default.  Cellpose is a
third-party dependency absent from /root/reference and from this image, with no pinned version
(requirements.txt:1-12) and no weights on disk, so its behaviour cannot be pinned here.  This
module restates the Cellpose 2.x/3.x algorithm (transforms.normalize99 / resize_image /
pad_image_ND / make_tiles / average_tiles, dynamics.follow_flows / get_masks /
remove_bad_flow_masks / masks_to_flows, utils.fill_holes_and_remove_small_masks) with every
numeric choice spelled out, and it is the oracle that the HIP segmentation post-processing in
libcpx must match bit-exactly on identical network outputs.  Choices:
  * channels=None with C > 2 -> the first nchan=2 channels are used;
  * normalize99 per channel: exact order statistics, fp64 linear interpolation (numpy's lerp
    formula), x' = fp32(((double)x - p1) / (p99 - p1));
  * rescale = diam_mean / diameter (nuclei 17 / 100); resize = cv2.resize INTER_LINEAR
    (scale = 1 / (dst / src), half-pixel centres, clamped edges), fp32, no FMA;
  * resample=True (CellposeModel.eval's default): the averaged network output is resized back
    to H x W before the dynamics, so follow_flows / get_masks / the flow-error filter /
    fill-holes all run at full resolution; niter = uint32(1 / rescale * 200) (1176 for the
    reference's nuclei model at diameter 100; `_run_cp`).  resample=False (dynamics at network
    resolution, masks nearest-resized) is kept as a named option;
  * follow_flows uses the CPU map_coordinates step (numba: fp64 expression, fp32 storage);
  * get_masks keeps Cellpose's seed order (the `for s in seeds: s = s[isort]` no-op leaves seeds
    in row-major order) and renumbers labels by first occurrence (fastremap.renumber);
  * flow-error filter (threshold 0.4) with the 2.x CPU masks_to_flows heat diffusion (median
    centre, niter = 2*(ptp x + ptp y), no log), fp64.
The literal numpy loops of follow_flows and masks_to_flows take minutes per 2080^2 FOV at
niter 1176; oracle/seg_oracle_c.c repeats them statement by statement in C (liboracle_seg.so,
built by oracle/Makefile) and is used when present (`impl="auto"`); tests/test_seg_oracle_c.py
checks the two implementations against each other.
"""
from __future__ import annotations

import math

import numpy as np
from scipy import ndimage as ndi

NET_CHANNELS = 2
DIAM_MEAN = {"nuclei": 17.0, "cyto": 30.0, "cyto2": 30.0, "cyto3": 30.0}
BSIZE = 224
TILE_OVERLAP = 0.1
NITER_NET = 200          # resample=False keeps Cellpose 2.x's fixed 200 steps at network size
CELLPROB_THRESHOLD = 0.0
FLOW_THRESHOLD = 0.4
MIN_SIZE = 15
RPAD = 20


# ---------------------------------------------------------------------------------------------
# normalisation / resize / tiling
# ---------------------------------------------------------------------------------------------

def _lerp(a: float, b: float, t: float) -> float:
    """numpy's _lerp (lib/function_base.py) in fp64."""
    d = b - a
    return b - d * (1.0 - t) if t >= 0.5 else a + d * t


def percentile(x: np.ndarray, q: float) -> float:
    """Exact order statistics of the fp32 values, linear interpolation at (n-1)*q/100 (fp64)."""
    v = np.sort(x.ravel().astype(np.float32))
    n = v.size
    vi = (n - 1) * (q / 100.0)
    lo = int(math.floor(vi))
    hi = min(lo + 1, n - 1)
    return _lerp(float(v[lo]), float(v[hi]), vi - lo)


def normalize99(x32: np.ndarray):
    """transforms.normalize99(img, lower=1, upper=99) restated; returns (xn, p1, p99)."""
    p1, p99 = percentile(x32, 1.0), percentile(x32, 99.0)
    den = p99 - p1
    if den == 0.0:
        den = 1.0
    xn = ((x32.astype(np.float64) - p1) / den).astype(np.float32)
    return xn, p1, p99


def net_size(H: int, W: int, model: str = "nuclei", diameter: float = 100.0):
    rescale = DIAM_MEAN[model] / diameter
    return int(H * rescale), int(W * rescale)


def default_niter(model: str = "nuclei", diameter: float = 100.0, resample: bool = True) -> int:
    """CellposeModel._run_cp: niter = 1 / rescale * 200, cast by follow_flows to uint32."""
    if not resample:
        return NITER_NET
    rescale = DIAM_MEAN[model] / diameter
    return int(np.uint32(1 / rescale * 200))


_CLIB = None


def clib():
    """liboracle_seg.so (oracle/seg_oracle_c.c) or None when it has not been built."""
    global _CLIB
    if _CLIB is None:
        import ctypes as ct
        import os
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "liboracle_seg.so")
        if not os.path.exists(path):
            _CLIB = False
        else:
            lib = ct.CDLL(path)
            P = ct.c_void_p
            lib.follow_flows_c.argtypes = [P, ct.c_int, ct.c_int, ct.c_int64, ct.c_int, P, P]
            lib.follow_flows_c.restype = None
            lib.flow_error_c.argtypes = [P, P, ct.c_int, ct.c_int, ct.c_int, P]
            lib.flow_error_c.restype = None
            _CLIB = lib
    return _CLIB or None


def _axis_coeffs(n_src: int, n_dst: int):
    scale = 1.0 / (n_dst / n_src)  # cv2.resize: scale_x = 1. / inv_scale_x, inv = dst / src
    i0 = np.zeros(n_dst, np.int64)
    w = np.zeros(n_dst, np.float32)
    for d in range(n_dst):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(math.floor(f))
        f = np.float32(f - np.float32(s))
        if s < 0:
            s, f = 0, np.float32(0.0)
        if s >= n_src - 1:
            s, f = n_src - 1, np.float32(0.0)
        i0[d], w[d] = s, f
    return i0, np.minimum(i0 + 1, n_src - 1), w


def resize_bilinear(img32: np.ndarray, Ly: int, Lx: int) -> np.ndarray:
    """cv2.resize INTER_LINEAR (half-pixel centres, clamped edges), fp32 arithmetic, row pass
    h = a*(1-wx) + b*wx then column pass h0*(1-wy) + h1*wy."""
    H, W = img32.shape
    y0, y1, wy = _axis_coeffs(H, Ly)
    x0, x1, wx = _axis_coeffs(W, Lx)
    one = np.float32(1.0)
    a = img32.astype(np.float32)
    r0 = a[y0][:, x0] * (one - wx) + a[y0][:, x1] * wx
    r1 = a[y1][:, x0] * (one - wx) + a[y1][:, x1] * wx
    return (r0 * (one - wy)[:, None] + r1 * wy[:, None]).astype(np.float32)


def pad_amounts(L: int, div: int = 16, extra: int = 1):
    """transforms.pad_image_ND: pad to a multiple of div plus extra*div//2 each side."""
    Lpad = int(div * np.ceil(L / div) - L)
    return extra * div // 2 + Lpad // 2, extra * div // 2 + Lpad - Lpad // 2


def tile_starts(Lp: int, bsize: int = BSIZE, overlap: float = TILE_OVERLAP):
    """transforms.make_tiles (augment=False) tile origins along one axis."""
    overlap = min(0.5, max(0.05, overlap))
    b = min(bsize, Lp)
    n = 1 if Lp <= bsize else int(np.ceil((1.0 + 2 * overlap) * Lp / bsize))
    return np.linspace(0, Lp - b, n).astype(int), b


def taper_mask(ly: int = BSIZE, lx: int | None = None, sig: float = 7.5) -> np.ndarray:
    """transforms._taper_mask(ly, lx, sig): built at bsize = max(224, ly, lx) (fp64 formula),
    centre-cropped to ly x lx, stored fp32."""
    lx = ly if lx is None else lx
    bsize = max(224, max(ly, lx))
    xm = np.arange(bsize)
    xm = np.abs(xm - xm.mean())
    m = 1 / (1 + np.exp((xm - (bsize / 2 - 20)) / sig))
    m = m * m[:, np.newaxis]
    m = m[bsize // 2 - ly // 2: bsize // 2 + ly // 2 + ly % 2, bsize // 2 - lx // 2: bsize // 2 + lx // 2 + lx % 2]
    return m.astype(np.float32)


class TileGeom:
    def __init__(self, Ly: int, Lx: int):
        self.Ly, self.Lx = Ly, Lx
        self.py0, py1 = pad_amounts(Ly)
        self.px0, px1 = pad_amounts(Lx)
        self.Lyp, self.Lxp = Ly + self.py0 + py1, Lx + self.px0 + px1
        self.ys, self.by = tile_starts(self.Lyp)
        self.xs, self.bx = tile_starts(self.Lxp)
        self.tiles = [(int(y), int(x)) for y in self.ys for x in self.xs]


def make_net_input(planes32: np.ndarray, Ly: int, Lx: int) -> tuple[np.ndarray, TileGeom]:
    """planes32 [C,H,W] -> tiles [n_tiles, 2, by, bx] fp32 (normalised, resized, padded)."""
    g = TileGeom(Ly, Lx)
    img = np.zeros((NET_CHANNELS, g.Lyp, g.Lxp), np.float32)
    for c in range(NET_CHANNELS):
        xn, _, _ = normalize99(planes32[c])
        img[c, g.py0:g.py0 + Ly, g.px0:g.px0 + Lx] = resize_bilinear(xn, Ly, Lx)
    tiles = np.stack([img[:, y:y + g.by, x:x + g.bx] for (y, x) in g.tiles])
    return tiles, g


def average_tiles(y: np.ndarray, g: TileGeom) -> np.ndarray:
    """transforms.average_tiles in fp32, tile order; returns yf [3, Ly, Lx] (pad cropped)."""
    mask = taper_mask(g.by, g.bx)
    acc = np.zeros((y.shape[1], g.Lyp, g.Lxp), np.float32)
    nav = np.zeros((g.Lyp, g.Lxp), np.float32)
    for t, (ys, xs) in enumerate(g.tiles):
        acc[:, ys:ys + g.by, xs:xs + g.bx] += y[t].astype(np.float32) * mask
        nav[ys:ys + g.by, xs:xs + g.bx] += mask
    yf = acc / nav
    return yf[:, g.py0:g.py0 + g.Ly, g.px0:g.px0 + g.Lx].astype(np.float32)


# ---------------------------------------------------------------------------------------------
# dynamics
# ---------------------------------------------------------------------------------------------

def follow_flows(dP: np.ndarray, cp_mask: np.ndarray, niter: int, impl: str = "auto"):
    """dynamics.follow_flows(dP * cp_mask / 5., niter, interp=True) with the CPU map_coordinates
    step (numba: fp64 expression, fp32 storage); returns p [2,Ly,Lx] fp32 and n_moving.
    impl: "numpy" (the literal loop below), "c" (seg_oracle_c.c, same statements) or "auto"."""
    Ly, Lx = dP.shape[1:]
    dPs = (dP * cp_mask / np.float32(5.0)).astype(np.float32)
    p = np.array(np.meshgrid(np.arange(Ly), np.arange(Lx), indexing="ij")).astype(np.float32)
    inds = np.array(np.nonzero(np.abs(dPs[0]) > 1e-3)).T
    if inds.shape[0] < 5:
        return p, int(inds.shape[0])
    py = p[0][inds[:, 0], inds[:, 1]].copy()
    px = p[1][inds[:, 0], inds[:, 1]].copy()
    lib = clib() if impl in ("auto", "c") else None
    if impl == "c" and lib is None:
        raise RuntimeError("liboracle_seg.so not built (make -C oracle)")
    if lib is not None:
        import ctypes as ct
        dpc = np.ascontiguousarray(dPs)
        lib.follow_flows_c(dpc.ctypes.data_as(ct.c_void_p), Ly, Lx, py.size, int(niter),
                           py.ctypes.data_as(ct.c_void_p), px.ctypes.data_as(ct.c_void_p))
    else:
        I = dPs.astype(np.float64)
        for _ in range(niter):
            yf = py.astype(np.int32)
            xf = px.astype(np.int32)
            y = (py - yf).astype(np.float32).astype(np.float64)
            x = (px - xf).astype(np.float32).astype(np.float64)
            y0 = np.minimum(Ly - 1, np.maximum(0, yf))
            x0 = np.minimum(Lx - 1, np.maximum(0, xf))
            y1 = np.minimum(Ly - 1, y0 + 1)
            x1 = np.minimum(Lx - 1, x0 + 1)
            d = []
            for c in range(2):
                v = (I[c, y0, x0] * (1 - y) * (1 - x) + I[c, y0, x1] * (1 - y) * x +
                     I[c, y1, x0] * y * (1 - x) + I[c, y1, x1] * y * x)
                d.append(v.astype(np.float32))
            py = np.minimum(np.float32(Ly - 1), np.maximum(np.float32(0), (py + d[0]).astype(np.float32)))
            px = np.minimum(np.float32(Lx - 1), np.maximum(np.float32(0), (px + d[1]).astype(np.float32)))
    p[0][inds[:, 0], inds[:, 1]] = py
    p[1][inds[:, 0], inds[:, 1]] = px
    return p, int(inds.shape[0])


def get_masks(p: np.ndarray, iscell: np.ndarray, rpad: int = RPAD) -> np.ndarray:
    """dynamics.get_masks restated (2-D)."""
    shape0 = p.shape[1:]
    p = p.copy()
    inds = np.meshgrid(np.arange(shape0[0]), np.arange(shape0[1]), indexing="ij")
    for i in range(2):
        p[i, ~iscell] = inds[i][~iscell]
    pflows = [p[i].flatten().astype("int32") for i in range(2)]
    shape = (shape0[0] + 2 * rpad, shape0[1] + 2 * rpad)
    h = np.zeros(shape, np.int64)
    np.add.at(h, (pflows[0] + rpad, pflows[1] + rpad), 1)
    hmax = h.copy()
    for i in range(2):
        hmax = ndi.maximum_filter1d(hmax, 5, axis=i)
    seeds = np.nonzero(np.logical_and(h - hmax > -1e-6, h > 10))  # row-major (isort is a no-op)
    M = np.zeros(shape, np.uint32)
    good = h > 2
    for k, (sy, sx) in enumerate(zip(*seeds)):
        # the expansion never leaves the 13 x 13 window (pix within +-6 after 5 dilations that
        # are clipped to it), so it is computed on the window alone; seeds sit >= 20 px inside
        y0, y1, x0, x1 = sy - 6, sy + 7, sx - 6, sx + 7
        cur = np.zeros((13, 13), bool)
        cur[6, 6] = True
        for _ in range(5):
            dil = ndi.binary_dilation(cur, structure=np.ones((3, 3), bool))
            cur = dil & good[y0:y1, x0:x1]
        M[y0:y1, x0:x1][cur] = k + 1
    M0 = M[pflows[0] + rpad, pflows[1] + rpad]
    # remove big masks (> 40% of the image)
    uniq, counts = np.unique(M0, return_counts=True)
    big = np.prod(shape0) * 0.4
    bigc = uniq[counts > big]
    if len(bigc) > 0 and (len(bigc) > 1 or bigc[0] != 0):
        M0[np.isin(M0, bigc)] = 0
    # fastremap.renumber: first-occurrence order, 0 preserved
    flat = M0.ravel()
    nz = flat[flat > 0]
    _, first = np.unique(nz, return_index=True)
    order = np.unique(nz)[np.argsort(first)]
    remap = np.zeros(int(flat.max()) + 1 if flat.size else 1, np.int64)
    remap[order] = np.arange(1, len(order) + 1)
    return remap[M0].reshape(shape0).astype(np.int32)


def masks_to_flows(masks: np.ndarray) -> np.ndarray:
    """dynamics.masks_to_flows_cpu (2.x heat diffusion from the pixel nearest the median)."""
    Ly, Lx = masks.shape
    mu = np.zeros((2, Ly, Lx), np.float64)
    for i, si in enumerate(ndi.find_objects(masks)):
        if si is None:
            continue
        sr, sc = si
        ly, lx = sr.stop - sr.start + 2, sc.stop - sc.start + 2
        y, x = np.nonzero(masks[sr, sc] == (i + 1))
        y = y.astype(np.int64) + 1
        x = x.astype(np.int64) + 1
        ymed, xmed = np.median(y), np.median(x)
        imin = np.argmin((x - xmed) ** 2 + (y - ymed) ** 2)
        xm, ym = int(x[imin]), int(y[imin])
        niter = 2 * int(np.ptp(x) + np.ptp(y))
        T = np.zeros(ly * lx, np.float64)
        for _ in range(niter):
            T[ym * lx + xm] += 1
            T[y * lx + x] = 1 / 9. * (T[y * lx + x] + T[(y - 1) * lx + x] + T[(y + 1) * lx + x] +
                                      T[y * lx + x - 1] + T[y * lx + x + 1] +
                                      T[(y - 1) * lx + x - 1] + T[(y - 1) * lx + x + 1] +
                                      T[(y + 1) * lx + x - 1] + T[(y + 1) * lx + x + 1])
        dy = T[(y + 1) * lx + x] - T[(y - 1) * lx + x]
        dx = T[y * lx + x + 1] - T[y * lx + x - 1]
        mu[:, sr.start + y - 1, sc.start + x - 1] = np.stack((dy, dx))
    mu /= (1e-20 + (mu ** 2).sum(axis=0) ** 0.5)
    return mu


def flow_errors(masks: np.ndarray, dP: np.ndarray, impl: str = "auto") -> np.ndarray:
    """metrics.flow_error: per label 1..max, mean over its pixels of (mu - dP/5)^2 summed over
    the two flow components (masks_to_flows of the masks vs the network flows)."""
    n = int(masks.max())
    lib = clib() if impl in ("auto", "c") else None
    if impl == "c" and lib is None:
        raise RuntimeError("liboracle_seg.so not built (make -C oracle)")
    if lib is not None:
        import ctypes as ct
        m = np.ascontiguousarray(masks, dtype=np.int32)
        d = np.ascontiguousarray(dP, dtype=np.float32)
        err = np.zeros(n, np.float64)
        with np.errstate(all="ignore"):
            lib.flow_error_c(m.ctypes.data_as(ct.c_void_p), d.ctypes.data_as(ct.c_void_p),
                             m.shape[0], m.shape[1], n, err.ctypes.data_as(ct.c_void_p))
        return err
    mu = masks_to_flows(masks)
    err = np.zeros(n)
    idx = np.arange(1, n + 1)
    for i in range(2):
        with np.errstate(all="ignore"):
            err += ndi.mean((mu[i] - dP[i].astype(np.float32) / np.float32(5.0)) ** 2, masks, index=idx)
    return err


def remove_bad_flow_masks(masks: np.ndarray, dP: np.ndarray, threshold: float = FLOW_THRESHOLD,
                          impl: str = "auto"):
    """dynamics.remove_bad_flow_masks / metrics.flow_error restated."""
    n = int(masks.max())
    if n == 0:
        return masks
    err = flow_errors(masks, dP, impl)
    bad = 1 + np.nonzero(err > threshold)[0]
    out = masks.copy()
    out[np.isin(out, bad)] = 0
    return out


def resize_nearest(masks: np.ndarray, H: int, W: int) -> np.ndarray:
    """cv2.resize(..., INTER_NEAREST): src = min(floor(dst * (1/(dst_n/src_n))), src_n - 1)."""
    Ly, Lx = masks.shape
    ify = 1.0 / (H / Ly)
    ifx = 1.0 / (W / Lx)
    ys = np.minimum(np.floor(np.arange(H) * ify).astype(np.int64), Ly - 1)
    xs = np.minimum(np.floor(np.arange(W) * ifx).astype(np.int64), Lx - 1)
    return masks[ys][:, xs]


def fill_holes_and_remove_small_masks(masks: np.ndarray, min_size: int = MIN_SIZE) -> np.ndarray:
    """utils.fill_holes_and_remove_small_masks (2-D), literal loop."""
    masks = masks.copy()
    j = 0
    for i, slc in enumerate(ndi.find_objects(masks)):
        if slc is None:
            continue
        msk = masks[slc] == (i + 1)
        npix = msk.sum()
        if min_size > 0 and npix < min_size:
            masks[slc][msk] = 0
        elif npix > 0:
            msk = ndi.binary_fill_holes(msk)
            masks[slc][msk] = j + 1
            j += 1
    return masks


def upsample_flows(yf: np.ndarray, H: int, W: int) -> np.ndarray:
    """CellposeModel._run_cp with resample=True: transforms.resize_image(yf, H, W) of the
    averaged network output (cv2 INTER_LINEAR per channel)."""
    return np.stack([resize_bilinear(yf[c], H, W) for c in range(yf.shape[0])])


def compute_masks(yf: np.ndarray, H: int, W: int, niter: int | None = None,
                  flow_threshold: float = FLOW_THRESHOLD, min_size: int = MIN_SIZE,
                  resample: bool = True, model: str = "nuclei", diameter: float = 100.0,
                  impl: str = "auto") -> np.ndarray:
    """masks of one FOV from the averaged network output yf [3, Ly, Lx] (dy, dx, cellprob).
    resample=True (the reference call's default): flows resized to H x W, then
    dynamics.compute_masks at full resolution with niter = default_niter(model, diameter).
    resample=False: compute_masks at network resolution (niter 200) with resize=(H, W)."""
    if niter is None:
        niter = default_niter(model, diameter, resample)
    if resample:
        yf = upsample_flows(yf, H, W)
    dP, cellprob = yf[:2], yf[2]
    cp_mask = cellprob > CELLPROB_THRESHOLD
    if not np.any(cp_mask):
        return np.zeros((H, W), np.int32)
    p, nmov = follow_flows(dP, cp_mask, niter, impl)
    if nmov < 5:
        return np.zeros((H, W), np.int32)
    m = get_masks(p, cp_mask)
    if m.max() > 0 and flow_threshold > 0:
        m = remove_bad_flow_masks(m, dP, flow_threshold, impl)
    if not resample:
        m = resize_nearest(m, H, W)
    return fill_holes_and_remove_small_masks(m, min_size).astype(np.int32)
