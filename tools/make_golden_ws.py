"""Golden fixtures for the Cells marker watershed (tests/golden/watershed_cases.npz) — test tooling.

Runs scikit-image 0.18.3 itself (the survey container's python3.9):

    /opt/conda/bin/python3.9 tools/make_golden_ws.py

Inputs are generated here with seeded numpy (synthetic nuclei as labelled ellipses, some
touching; a cell channel of Gaussian halos + Poisson noise, float32, with a flat region to force
16-bit ties), then skimage.segmentation.expand_labels gives the footprint and
skimage.segmentation.watershed(key, nuclei, mask=footprint) the expected Cells, with the stated
elevation key (oracle/ws_oracle.py docstring).  Two generic cases (random distinct float64
images, random markers, with and without a mask) pin the flood itself.  Only inputs and outputs
are written.
"""
import os

import numpy as np
from skimage.segmentation import expand_labels, watershed

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "tests", "golden", "watershed_cases.npz")


def key_of(corr):
    c = corr.astype(np.float32)
    q = np.where(c > 0, c, np.float32(0)).astype(np.float64)
    q = np.where(np.isnan(c) | (c >= 65535), 65535.0, np.floor(q)).astype(np.uint64)
    H, W = c.shape
    idx = np.arange(H * W, dtype=np.uint64).reshape(H, W)
    return ((np.uint64(65535) - q) << np.uint64(23)) | idx


def synth_cells(H, W, n, seed, flat=False):
    rng = np.random.default_rng(seed)
    yy, xx = np.indices((H, W))
    nuc = np.zeros((H, W), np.int32)
    lam = np.full((H, W), 300.0)
    for i in range(n):
        cy, cx = rng.uniform(0, H), rng.uniform(0, W)
        ry, rx = rng.uniform(5, 22), rng.uniform(5, 22)
        th = rng.uniform(0, np.pi)
        dy, dx = yy - cy, xx - cx
        u = (dy * np.cos(th) + dx * np.sin(th)) / ry
        v = (-dy * np.sin(th) + dx * np.cos(th)) / rx
        inside = u * u + v * v <= 1.0
        nuc[inside & (nuc == 0)] = i + 1           # later nuclei never overwrite (touching, not overlapping)
        s = 2.5 * max(ry, rx)
        lam += rng.uniform(500, 4000) * np.exp(-(dy * dy + dx * dx) / (2 * s * s))
    corr = (rng.poisson(lam) / rng.uniform(0.7, 1.3)).astype(np.float32)
    if flat:
        corr[H // 3: H // 2, :] = np.float32(1234.5)  # 16-bit ties: the raster index decides
        corr[5, 5] = np.float32(np.nan)
        corr[6, 6] = np.float32(np.inf)
        corr[7, 7] = np.float32(-3.0)
        corr[8, 8] = np.float32(70000.0)
    # relabel in raster first-occurrence order with gaps, as a label image would come
    return nuc, corr


def main():
    out = {}
    rng = np.random.default_rng(7)
    # generic flood: distinct float64 values
    for name, mask_on in (("generic_nomask", False), ("generic_mask", True)):
        H, W = 40, 50
        img = rng.permutation(H * W).astype(np.float64).reshape(H, W) * 0.37 - 100.0
        mk = np.zeros((H, W), np.int32)
        pts = rng.choice(H * W, 7, replace=False)
        mk.ravel()[pts] = rng.permutation(np.arange(1, 8)) * 3
        mask = (rng.random((H, W)) < 0.8) if mask_on else None
        res = watershed(img, mk, mask=mask)
        out[f"{name}_image"] = img
        out[f"{name}_markers"] = mk
        out[f"{name}_mask"] = np.ones((H, W), bool) if mask is None else mask
        out[f"{name}_has_mask"] = np.array(mask_on)
        out[f"{name}_out"] = res.astype(np.int32)
    # stated Cells watershed
    for name, (H, W, n, seed, flat) in {"cells_small": (200, 240, 40, 1, False),
                                        "cells_ties": (256, 256, 60, 2, True),
                                        "cells_512": (512, 512, 300, 3, False),
                                        "cells_768": (768, 768, 500, 4, True)}.items():
        nuc, corr = synth_cells(H, W, n, seed, flat)
        foot = expand_labels(nuc, 15) > 0
        cells = watershed(key_of(corr).astype(np.float64), nuc, mask=foot)
        out[f"{name}_nuclei"] = nuc
        out[f"{name}_corr"] = corr
        out[f"{name}_cells"] = cells.astype(np.int32)
    out["names_generic"] = np.array(["generic_nomask", "generic_mask"])
    out["names_cells"] = np.array(["cells_small", "cells_ties", "cells_512", "cells_768"])
    out["distance"] = np.array(15)
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT))


if __name__ == "__main__":
    main()
