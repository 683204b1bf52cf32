"""CPU restatement (test infrastructure only) of the reference's embedding preprocessing:
Cellpose_GPU_s3fs.py:177-187 — per kept crop and channel scale_to_8bit -> PIL L -> RGB, then
transformers' TimmWrapperImageProcessor for "timm/tf_efficientnetv2_l.in21k" = timm's eval
transform of the pretrained config (input 384, crop_pct 1.0, bicubic, mean = std = 0.5):
PIL Image.resize(384, BICUBIC) -> CenterCrop(384) (identity for square crops) -> ToTensor
(x / 255, fp32) -> Normalize ((x - 0.5) / 0.5, fp32); the fp16 autocast of the model casts the
result to fp16.  timm is absent here, so the transform chain is restated from its source (parity
of the chain unpinned); the resize itself is pinned against Pillow in tests/test_embed.py.

Pillow's 8-bit resampler (libImaging/Resample.c, 8 bits per channel):
  * precompute_coeffs per axis (fp64): scale = in/out, filterscale = max(scale, 1),
    support = 2 * filterscale (bicubic, a = -0.5); for output x: center = (x + 0.5) * scale,
    xmin = max(0, int(center - support + 0.5)), xmax = min(in, int(center + support + 0.5));
    w_i = bicubic((i + xmin - center + 0.5) / filterscale) normalised by their sum;
  * normalize_coeffs_8bpc: k_i = int(w_i * 2^22 + 0.5) (w >= 0) or int(w_i * 2^22 - 0.5);
  * each output: ss = 2^21 + sum_i pixel_i * k_i (int32), value = clamp(ss >> 22, 0, 255);
  * horizontal pass first (into an 8-bit image), then the vertical pass.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def bicubic(x: float) -> float:
    a = -0.5
    if x < 0.0:
        x = -x
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def precompute_coeffs_8bpc(in_size: int, out_size: int):
    """(xmin[out], count[out], k[out][ksize] int32) as Pillow's 8-bit path uses them."""
    scale = float(in_size) / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    xmins = np.zeros(out_size, np.int64)
    counts = np.zeros(out_size, np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
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
        w = [bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        for x in range(xmax):
            v = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        xmins[xx], counts[xx] = xmin, xmax
    return xmins, counts, kk


def _pass(img: np.ndarray, xmins, counts, kk, axis: int) -> np.ndarray:
    a = np.moveaxis(img.astype(np.int64), axis, -1)
    out = np.empty(a.shape[:-1] + (len(xmins),), np.int64)
    for xx in range(len(xmins)):
        s = np.full(a.shape[:-1], 1 << (PRECISION_BITS - 1), np.int64)
        for k in range(counts[xx]):
            s += a[..., xmins[xx] + k] * kk[xx, k]
        out[..., xx] = np.clip(s >> PRECISION_BITS, 0, 255)
    return np.moveaxis(out, -1, axis).astype(np.uint8)


def resize_bicubic_u8(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """PIL Image.fromarray(img).resize((out_w, out_h), BICUBIC) for an 8-bit plane."""
    H, W = img.shape
    x = img
    if out_w != W:
        x = _pass(x, *precompute_coeffs_8bpc(W, out_w), axis=1)
    if out_h != H:
        x = _pass(x, *precompute_coeffs_8bpc(H, out_h), axis=0)
    return x


def pixel_values(img8: np.ndarray, size: int = 384, mean: float = 0.5, std: float = 0.5) -> np.ndarray:
    """[3, size, size] float32 model input of one 8-bit crop channel (R = G = B)."""
    r = resize_bicubic_u8(img8, size, size).astype(np.float32)
    x = (r / np.float32(255.0) - np.float32(mean)) / np.float32(std)
    return np.stack([x, x, x]).astype(np.float32)
