"""Deterministic, integer-only synthetic inputs for the golden fixtures — TEST INFRASTRUCTURE.

Every value is produced with uint64/int64 arithmetic (splitmix64 hashing, integer blob
profiles) plus IEEE-exact divisions, so the same (seed, shape) yields bit-identical arrays under
numpy 1.26 (the survey container's python3.9 that generated tests/golden/) and numpy 2.x (this
image).  That lets full-size 2080x2080 golden cases be stored as a seed plus expected outputs.
"""
from __future__ import annotations

import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.asarray(x, dtype=np.uint64) + _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _stream(seed: int, n: int, salt: int) -> np.ndarray:
    base = np.uint64((seed * 1000003 + salt * 7919) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        return splitmix64(np.arange(n, dtype=np.uint64) + base * np.uint64(0x100000001))


def plane(seed: int, H: int, W: int, n_blobs: int = 40, saturate: bool = True,
          halo: bool = False) -> np.ndarray:
    """uint16 plane: noisy background ~300, integer paraboloid 'nuclei', rare 65535 pixels."""
    h = _stream(seed, H * W, 1).reshape(H, W)
    img = (280 + (h % np.uint64(41)).astype(np.int64)).astype(np.int64)
    p = _stream(seed, n_blobs * 5, 2).reshape(n_blobs, 5)
    yy = np.arange(H, dtype=np.int64)[:, None]
    xx = np.arange(W, dtype=np.int64)[None, :]
    rmax = max(4, min(H, W) // 12)
    for k in range(n_blobs):
        cy = int(p[k, 0] % np.uint64(H))
        cx = int(p[k, 1] % np.uint64(W))
        ry = 3 + int(p[k, 2] % np.uint64(rmax))
        rx = 3 + int(p[k, 3] % np.uint64(rmax))
        if halo:
            ry, rx = 2 * ry + 2, 2 * rx + 2
        peak = 1000 + int(p[k, 4] % np.uint64(19000))
        y0, y1 = max(0, cy - ry), min(H, cy + ry + 1)
        x0, x1 = max(0, cx - rx), min(W, cx + rx + 1)
        dy = yy[y0:y1] - cy
        dx = xx[:, x0:x1] - cx
        R2 = ry * ry * rx * rx
        d2 = dy * dy * (rx * rx) + dx * dx * (ry * ry)
        img[y0:y1, x0:x1] += peak * np.maximum(0, R2 - d2) // R2
    if saturate:
        img[(h % np.uint64(9973)) == 0] = 65535
    return np.clip(img, 0, 65535).astype(np.uint16)


def illum(seed: int, H: int, W: int, dtype=np.float32) -> np.ndarray:
    """Smooth flat-field in ~[0.7, 1.3]: float(rational of integers), IEEE-exact."""
    q = _stream(seed, 4, 3)
    cy = int(q[0] % np.uint64(H))
    cx = int(q[1] % np.uint64(W))
    yy = np.arange(H, dtype=np.int64)[:, None] - cy
    xx = np.arange(W, dtype=np.int64)[None, :] - cx
    num = 1300 * H * H * W * W - 600 * (yy * yy * W * W + xx * xx * H * H) // 2
    den = 1000 * H * H * W * W
    val = num.astype(np.float64) / float(den)
    return np.maximum(val, 0.7).astype(dtype)


def labels(seed: int, H: int, W: int, n: int = 30, skip_every: int = 7,
           rmin: int = 4, rmax: int | None = None) -> np.ndarray:
    """int32 label image of filled ellipses (integer test); later labels overwrite earlier
    ones (touching/overlapping objects); label values skip every `skip_every`-th (gaps);
    some objects hit the image border."""
    lab = np.zeros((H, W), dtype=np.int32)
    p = _stream(seed, n * 6, 4).reshape(n, 6)
    rmax = rmax or max(rmin + 1, min(H, W) // 8)
    yy = np.arange(H, dtype=np.int64)[:, None]
    xx = np.arange(W, dtype=np.int64)[None, :]
    value = 0
    for k in range(n):
        value += 1
        if skip_every and value % skip_every == 0:
            value += 1
        cy = int(p[k, 0] % np.uint64(H))
        cx = int(p[k, 1] % np.uint64(W))
        ry = rmin + int(p[k, 2] % np.uint64(rmax - rmin))
        rx = rmin + int(p[k, 3] % np.uint64(rmax - rmin))
        shear = int(p[k, 4] % np.uint64(5)) - 2  # skews the ellipse -> generic orientation
        dy = yy - cy
        dx = xx - cx + (shear * dy) // 4
        inside = dy * dy * (rx * rx) + dx * dx * (ry * ry) <= (rx * rx) * (ry * ry)
        lab[inside] = value
    return lab


def boundary_objects(H: int = 2200, W: int = 720) -> np.ndarray:
    """int32 labels whose objects straddle the feature kernels' fast-path limits (integer test,
    sheared shapes): a texture bbox just under and just over 65535 px, a 2100 x 30 slanted strip
    (bbox <= 65535 px but > 4096 membership-mask words: shape and texture fallbacks), a 400 x 400
    blob (both fallbacks), and small / mid objects around them."""
    lab = np.zeros((H, W), dtype=np.int32)
    yy = np.arange(H, dtype=np.int64)[:, None]
    xx = np.arange(W, dtype=np.int64)[None, :]

    def ellipse(value, cy, cx, ry, rx, shear):
        dy = yy - cy
        dx = xx - cx + (shear * dy) // 8
        inside = dy * dy * (rx * rx) + dx * dx * (ry * ry) <= (rx * rx) * (ry * ry)
        lab[inside] = value

    ellipse(1, 140, 150, 127, 120, 1)     # bbox 255 x 256 = 65280 px: LDS texture path
    ellipse(2, 450, 160, 129, 128, 1)     # bbox 259 x 274 > 65535 px: texture fallback
    ellipse(3, 900, 560, 200, 150, 2)     # bbox 401 x 351: shape + texture fallbacks
    # slanted strip, rows 60 .. 2159, 6 px of slant, 24-25 px wide
    y0, y1 = 60, 2160
    dy = yy - y0
    left = 640 + (dy * 6) // (y1 - y0)
    strip = (yy >= y0) & (yy < y1) & (xx >= left) & (xx < left + 24 + (dy % 7 == 0))
    lab[strip] = 4                        # bbox 2100 x 31: (2104) x 2 words > 4096: fallbacks
    small = labels(12345, H, W - 120, n=30, rmin=4, rmax=40, skip_every=0)
    small_vals = np.where(small > 0, small + 10, 0)
    sub = lab[:, : W - 120]
    sub[(sub == 0) & (small_vals > 0)] = small_vals[(sub == 0) & (small_vals > 0)]
    return lab


def full_case(seed: int, H: int = 2080, W: int = 2080, C: int = 5, n_blobs: int = 300):
    """The full-size FOV used by the golden QC fixture: C planes + C flat-fields."""
    raw = np.stack([plane(seed * 10 + c, H, W, n_blobs=n_blobs, halo=(c > 0)) for c in range(C)])
    ill = np.stack([illum(seed * 10 + c, H, W) for c in range(C)])
    return raw, ill
