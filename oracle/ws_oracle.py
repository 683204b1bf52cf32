"""TEST INFRASTRUCTURE (oracle) — Cells by marker watershed, never imported by the product.

SURVEY.md §8(a8): Cells are grown from the Nuclei by a marker watershed (skimage 0.18.3
`segmentation.watershed`, skimage/segmentation/_watershed.py:94); Cytoplasm = Cells minus
Nuclei with the same ObjectNumber (consumers: Pycyto_pertime.py:46-49, Normalize_CP_ami.py:47-52).
The CellProfiler pipeline that does this in the reference is not in the repo, so the stated
inputs are:

  markers   = Nuclei labels
  mask      = expand_labels(Nuclei, distance) > 0        (the footprint within `distance` px)
  elevation = inverted illumination-corrected cell channel (AGP), truncated to 16 bits, with the
              pixel's raster index as a tie-break:
                q(p)   = 65535 if not (corr < 65535) else max(0, trunc(corr))
                key(p) = (65535 - q(p)) * 2**23 + (y * W + x)        (exact in float64, H*W <= 2**23)
  Cells     = watershed(key, markers, mask=mask)          (connectivity 1)

Distinct keys make the flooding order a total order (no heap tie can matter), which is what lets
the GPU compute the same labels in parallel: `watershed_minimax` restates the result in that
form (minimax flood level by relaxation + label pointers) and is checked equal to the
sequential heap flood (`watershed`, C in ws_oracle_c.c, pure Python for small cases), which
tests/golden/watershed_cases.npz pins to skimage 0.18.3 itself.
"""
from __future__ import annotations

import ctypes as ct
import heapq

import numpy as np

KEY_SHIFT = 23
MAX_PIXELS = 1 << KEY_SHIFT


def quantise(corr: np.ndarray) -> np.ndarray:
    """q(p): float32 corrected intensity -> uint16 (NaN / >= 65535 -> 65535, <= 0 -> 0, trunc)."""
    c = np.asarray(corr, np.float32)
    q = np.where(c > 0, c, np.float32(0)).astype(np.float64)
    q = np.where(np.isnan(c) | (c >= 65535), 65535.0, np.floor(q))
    return q.astype(np.uint16)


def elevation_key(corr: np.ndarray) -> np.ndarray:
    """uint64 key per pixel (see module docstring)."""
    H, W = corr.shape
    if H * W > MAX_PIXELS:
        raise ValueError("watershed elevation: H*W must be <= 2**23")
    q = quantise(corr).astype(np.uint64)
    idx = np.arange(H * W, dtype=np.uint64).reshape(H, W)
    return ((np.uint64(65535) - q) << np.uint64(KEY_SHIFT)) | idx


def _clib():
    import seg_oracle
    lib = seg_oracle.clib()
    if lib is None:
        return None
    if not getattr(lib, "_ws_ready", False):
        lib.watershed_c.argtypes = [ct.c_void_p] * 3 + [ct.c_int, ct.c_int, ct.c_void_p]
        lib.watershed_c.restype = ct.c_int
        lib._ws_ready = True
    return lib


def watershed(image: np.ndarray, markers: np.ndarray, mask: np.ndarray | None = None,
              impl: str = "auto") -> np.ndarray:
    """skimage.segmentation.watershed(image, markers, connectivity=1, mask=mask), 2-D."""
    H, W = image.shape
    img = np.ascontiguousarray(image, np.float64)
    mk = np.ascontiguousarray(markers, np.int32)
    ms = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    lib = _clib() if impl in ("auto", "c") else None
    if impl == "c" and lib is None:
        raise RuntimeError("liboracle_seg.so not built (make -C oracle)")
    if lib is not None:
        out = np.zeros((H, W), np.int32)
        rc = lib.watershed_c(img.ctypes.data, mk.ctypes.data, None if ms is None else ms.ctypes.data,
                             H, W, out.ctypes.data)
        if rc:
            raise MemoryError("watershed_c")
        return out
    return _watershed_py(img, mk, ms)


def _watershed_py(img, mk, ms):
    """Literal pure-Python form of the Cython flood (small cases)."""
    H, W = img.shape
    Hp, Wp = H + 2, W + 2
    image = np.zeros((Hp, Wp)); image[1:-1, 1:-1] = img
    mask = np.zeros((Hp, Wp), bool); mask[1:-1, 1:-1] = True if ms is None else ms != 0
    out = np.zeros((Hp, Wp), np.int32); out[1:-1, 1:-1] = mk * mask[1:-1, 1:-1]
    image, mask, out = image.ravel(), mask.ravel(), out.ravel()
    nb = (-Wp, -1, 1, Wp)
    heap = [(image[i], 0, int(i)) for i in np.flatnonzero(out)]
    heapq.heapify(heap)
    age = 1
    while heap:
        _, _, i = heapq.heappop(heap)
        for o in nb:
            q = i + o
            if not mask[q] or out[q]:
                continue
            age += 1
            out[q] = out[i]
            heapq.heappush(heap, (image[q], age, q))
    return out.reshape(Hp, Wp)[1:-1, 1:-1].copy()


def watershed_minimax(key: np.ndarray, markers: np.ndarray, mask: np.ndarray, return_info=False):
    """The same labels in the parallel form the GPU computes (distinct keys required):

    1. flood level  B(p) = min over 4-paths marker -> p inside the mask of max key on the path
       (markers: B = key), by relaxation  B(p) = max(key(p), min_n B(n))  to the fixed point;
    2. a non-marker pixel is labelled by the first of its neighbours the flood pops, i.e. the one
       with the smallest B; so with parent(p) = the pixel whose key is B(p) (its "pass") when
       B(p) > key(p), else the neighbour with the smallest B (< key(p)), every chain ends at a
       marker and label(p) = label(that marker).
    Pixels the flood never reaches (B infinite) stay 0."""
    H, W = key.shape
    INF = np.uint64(0xFFFFFFFFFFFFFFFF)
    m = mask.astype(bool)
    mk = markers.astype(np.int32) * m
    free = m & (mk == 0)
    B = np.where(mk > 0, key, INF).astype(np.uint64)
    sweeps = 0
    while True:
        old = B.copy()
        for axis, rev in ((1, False), (1, True), (0, False), (0, True)):
            n = B.shape[axis]
            rng = range(n - 2, -1, -1) if rev else range(1, n)
            for i in rng:
                j = i + 1 if rev else i - 1
                if axis == 1:
                    cur, prv, k, f = B[:, i], B[:, j], key[:, i], free[:, i]
                else:
                    cur, prv, k, f = B[i], B[j], key[i], free[i]
                nv = np.maximum(k, np.minimum(cur, prv))
                cur[f] = nv[f]
            sweeps += 1
        if np.array_equal(old, B):
            break
    # label pointers
    flat = B.ravel()
    pad = np.full((H + 2, W + 2), INF, np.uint64)
    pad[1:-1, 1:-1] = B
    nbs = np.stack([pad[:-2, 1:-1], pad[1:-1, :-2], pad[1:-1, 2:], pad[2:, 1:-1]])  # up, left, right, down
    arg = nbs.argmin(0)
    offs = np.array([-W, -1, 1, W])
    idx = np.arange(H * W).reshape(H, W)
    parent = np.where(B > key, (B & np.uint64(MAX_PIXELS - 1)).astype(np.int64), idx + offs[arg])
    reach = free & (B != INF)
    lab = np.where(mk > 0, mk, 0).ravel().astype(np.int32)
    par = np.where(reach, parent, -1).ravel()
    done = (mk > 0).ravel() | ~reach.ravel()
    rounds = 0
    while not done.all():  # pointer jumping
        todo = ~done
        p = par[todo]
        lab_t = lab[p]
        fin = done[p]
        sel = np.flatnonzero(todo)
        lab[sel[fin]] = lab_t[fin]
        done[sel[fin]] = True
        par[sel[~fin]] = par[p[~fin]]
        rounds += 1
    out = lab.reshape(H, W) * (reach | (mk > 0))
    if return_info:
        return out, {"sweep_rounds": sweeps // 4, "jump_rounds": rounds, "B": B}
    return out


def cells_watershed(nuclei: np.ndarray, corr_cell: np.ndarray, distance: int, impl: str = "auto"):
    """(Cells, Cytoplasm) of one FOV: the stated watershed (module docstring)."""
    import cpx_oracle
    foot = cpx_oracle.expand_labels(nuclei, distance) > 0
    key = elevation_key(corr_cell)
    cells = watershed(key.astype(np.float64), nuclei, foot, impl=impl).astype(nuclei.dtype)
    cyto = np.where(nuclei == 0, cells, 0).astype(cells.dtype)
    return cells, cyto
