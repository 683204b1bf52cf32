"""CPU restatement (test infrastructure only) of the reference's image re-binning:
Image_re-binning.py:12-22 `process_image_in_memory` = PIL `Image.resize(target, LANCZOS)` on the
16-bit TIFF plane (mode "I;16"), Pillow >= 9.1 (the script uses `Image.Resampling`; pinned here
against Pillow 12.2.0 outputs of the reference function, tests/golden/rebin_cases.npz).

Pillow's separable resampler (libImaging/Resample.c), restated:
  * per axis, precompute_coeffs: scale = in/out, filterscale = max(scale, 1), support =
    3 * filterscale; for output x: center = (x + 0.5) * scale, xmin = max(0, int(center -
    support + 0.5)), xmax = min(in, int(center + support + 0.5)); weights
    w_i = lanczos3((i + xmin - center + 0.5) / filterscale), normalised by their sum (fp64);
    lanczos3(t) = sinc(t) sinc(t/3) on [-3, 3), sinc(t) = sin(pi t)/(pi t);
  * horizontal pass first, over the source rows the vertical pass needs, into a 16-bit image
    of the same mode, then the vertical pass;
  * each output: fp64 ss = sum_i pixel_i * w_i in index order (no FMA), ROUND_UP(ss) =
    int(ss + 0.5) for ss >= 0 else int(ss - 0.5), stored as two bytes low = CLIP8(v % 256)
    (C remainder), high = CLIP8(v >> 8) — values above 65535 keep their low byte.
"""
from __future__ import annotations

import math

import numpy as np


def lanczos3(x: float) -> float:
    def sinc(t):
        if t == 0.0:
            return 1.0
        t = t * math.pi
        return math.sin(t) / t
    if -3.0 <= x < 3.0:
        return sinc(x) * sinc(x / 3.0)
    return 0.0


def precompute_coeffs(in_size: int, out_size: int):
    """Returns (xmin[out], xmax[out] (count), k[out][ksize]) as Pillow computes them."""
    scale = float(in_size) / out_size
    filterscale = max(scale, 1.0)
    support = 3.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.float64)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        ww = 0.0
        w = []
        for x in range(xmax):
            v = lanczos3((x + xmin - center + 0.5) * ss)
            w.append(v)
            ww += v
        for x in range(xmax):
            kk[xx, x] = w[x] / ww if ww != 0.0 else w[x]
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _round_store16(ss: np.ndarray) -> np.ndarray:
    v = np.where(ss >= 0.0, np.trunc(ss + 0.5), np.trunc(ss - 0.5)).astype(np.int64)
    lo = np.fmod(v, 256)                     # C remainder (sign of the dividend)
    hi = v >> 8                              # arithmetic shift
    lo = np.clip(lo, 0, 255)
    hi = np.clip(hi, 0, 255)
    return (lo + (hi << 8)).astype(np.uint16)


def _pass(src: np.ndarray, bounds, kk, axis: int) -> np.ndarray:
    """One resample pass along `axis` (1 = horizontal over columns, 0 = vertical)."""
    a = src.astype(np.float64)
    if axis == 0:
        a = a.T
    out_n = bounds.shape[0]
    ss = np.zeros((a.shape[0], out_n), np.float64)
    for xx in range(out_n):
        xmin, cnt = bounds[xx]
        acc = np.zeros(a.shape[0], np.float64)
        for x in range(cnt):  # index order, separate multiply and add
            acc = acc + a[:, xmin + x] * kk[xx, x]
        ss[:, xx] = acc
    out = _round_store16(ss)
    return out.T if axis == 0 else out


def resize_lanczos_u16(img: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """PIL Image.fromarray(img uint16).resize((out_w, out_h), LANCZOS) restated."""
    H, W = img.shape
    bh, kh = precompute_coeffs(W, out_w)
    bv, kv = precompute_coeffs(H, out_h)
    need_h = out_w != W
    need_v = out_h != H
    cur = img.astype(np.uint16)
    if need_h:
        y0 = int(bv[0, 0])
        y1 = int(bv[-1, 0] + bv[-1, 1])
        cur = _pass(cur[y0:y1] if need_v else cur, bh, kh, axis=1)
        if need_v:
            bv = bv.copy()
            bv[:, 0] -= y0
    if need_v:
        cur = _pass(cur, bv, kv, axis=0)
    return cur
