"""Synthetic cell-painting plates generated directly in HBM (bench / smoke inputs).

Spec: uint16 planes with a Poisson(300) background, ~250-400 nuclei per FOV as
Gaussian blobs (sigma 10-35 px, peak 1k-20k) in channel 0, cytoplasm halos (2-3x the nuclear
radius) in the other channels, ~0.01 % of pixels clamped to 65535; flat-fields are smooth
quadratic surfaces in [0.7, 1.3] (fp32).  Blobs are rendered per sigma class in the Fourier
domain (impulses x analytic Gaussian transfer function), so a 2080^2 x 5 FOV costs a few FFTs.
"""
from __future__ import annotations

import math

import numpy as np
import torch

SIGMAS = (10.0, 16.0, 24.0, 34.0)  # nucleus sigma classes (px)
HALO = 2.5                         # cytoplasm sigma / nucleus sigma


def _gauss_tf(H, W, sigma, device):
    fy = torch.fft.fftfreq(H, device=device, dtype=torch.float32)[:, None]
    fx = torch.fft.rfftfreq(W, device=device, dtype=torch.float32)[None, :]
    # unit-peak Gaussian: transfer function of exp(-r^2 / (2 s^2)) is 2 pi s^2 exp(-2 pi^2 s^2 f^2)
    return (2 * math.pi * sigma * sigma) * torch.exp(-2 * math.pi ** 2 * sigma * sigma * (fx * fx + fy * fy))


def synth_fovs(B: int, C: int, H: int, W: int, device, seed: int = 0,
               nuclei=(250, 400), return_params: bool = False):
    """Returns int16 [B*C, H, W] holding uint16 bit patterns (plane p = channel p % C), and with
    return_params the per-FOV nucleus list (y, x, sigma) for ground truth."""
    g = torch.Generator(device=device).manual_seed(seed)
    out = torch.empty((B * C, H, W), dtype=torch.int16, device=device)
    tfs = [_gauss_tf(H, W, s, device) for s in SIGMAS]
    tfh = [_gauss_tf(H, W, s * HALO, device) for s in SIGMAS]
    params = []
    for b in range(B):
        n = int(torch.randint(nuclei[0], nuclei[1] + 1, (1,), generator=g, device=device).item())
        ys = torch.randint(0, H, (n,), generator=g, device=device)
        xs = torch.randint(0, W, (n,), generator=g, device=device)
        cls = torch.randint(0, len(SIGMAS), (n,), generator=g, device=device)
        peak = 1000.0 + 19000.0 * torch.rand((n,), generator=g, device=device)
        chan_gain = 0.2 + 0.8 * torch.rand((C, n), generator=g, device=device)
        if return_params:
            params.append((ys, xs, torch.tensor(SIGMAS, device=device)[cls], peak))
        for c in range(C):
            spec = None
            for k in range(len(SIGMAS)):
                sel = cls == k
                imp = torch.zeros((H, W), dtype=torch.float32, device=device)
                amp = peak[sel] if c == 0 else 0.15 * peak[sel] * chan_gain[c, sel]
                imp.index_put_((ys[sel], xs[sel]), amp, accumulate=True)
                f = torch.fft.rfft2(imp) * (tfs[k] if c == 0 else tfh[k])
                spec = f if spec is None else spec + f
            img = torch.fft.irfft2(spec, s=(H, W))
            if c > 0:  # some nuclear signal bleeds into the other channels
                img = img * 1.0
            lam = torch.clamp(img, min=0.0) + 300.0
            img = torch.poisson(lam, generator=g)
            sat = torch.rand((H, W), generator=g, device=device) < 1e-4
            img = torch.where(sat, torch.full_like(img, 65535.0), img)
            v = torch.clamp(img, 0, 65535).to(torch.int32)
            out[b * C + c] = torch.where(v > 32767, v - 65536, v).to(torch.int16)
    return (out, params) if return_params else out


def synth_illum(C: int, H: int, W: int, seed: int = 0) -> np.ndarray:
    """Smooth quadratic flat-fields in [0.7, 1.3] (fp32, host)."""
    rng = np.random.default_rng(seed)
    yy = np.linspace(-1, 1, H)[:, None]
    xx = np.linspace(-1, 1, W)[None, :]
    out = np.zeros((C, H, W), np.float32)
    for c in range(C):
        cy, cx = rng.uniform(-0.3, 0.3, 2)
        r2 = (yy - cy) ** 2 + (xx - cx) ** 2
        out[c] = np.clip(1.3 - 0.3 * r2, 0.7, 1.3).astype(np.float32)
    return out


def to_uint16(planes_i16: torch.Tensor) -> np.ndarray:
    return planes_i16.cpu().numpy().view(np.uint16)


def synth_zstack(B: int, C: int, Z: int, H: int, W: int, device, seed: int = 0) -> torch.Tensor:
    """Z-stack variant (SURVEY.md 8(d), configs[4]): int16 [B*C, Z, H, W] uint16 bit patterns.
    Plane z is the in-focus FOV (synth_fovs) blurred by a Gaussian of sigma 2|z - Z//2| plus
    Poisson(20) read noise, so the per-pixel argmax over z varies across the plane."""
    focus = synth_fovs(B, C, H, W, device, seed=seed)
    g = torch.Generator(device=device).manual_seed(seed + 7)
    out = torch.empty((B * C, Z, H, W), dtype=torch.int16, device=device)
    for p in range(B * C):
        img = focus[p].to(torch.int32)
        img = torch.where(img < 0, img + 65536, img).to(torch.float32)
        spec = torch.fft.rfft2(img)
        for z in range(Z):
            s = 2.0 * abs(z - Z // 2)
            if s > 0:
                tf = _gauss_tf(H, W, s, device) / (2 * math.pi * s * s)  # unit-gain blur
                plane = torch.fft.irfft2(spec * tf, s=(H, W))
            else:
                plane = img
            plane = plane + torch.poisson(torch.full_like(plane, 20.0), generator=g)
            v = torch.clamp(plane, 0, 65535).to(torch.int32)
            out[p, z] = torch.where(v > 32767, v - 65536, v).to(torch.int16)
    return out
