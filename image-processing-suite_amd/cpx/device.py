"""Device context: the Python face of libcpx on one GPU.

PyTorch-ROCm is used here only as plumbing — device allocations, the HIP stream (torch's
current stream is handed to libcpx so every kernel is ordered with torch work) and host<->device
copies.  All per-FOV arithmetic runs in the hand-written HIP kernels of libcpx.
"""
from __future__ import annotations

import atexit
import ctypes as ct
import os

import torch

from . import _lib
from ._lib import check

_STATS_BYTES = 64
_QC_BYTES = 24
_LSTAT_BYTES = 64
_OBJ_BYTES = 56
_HDR_BYTES = 16

OBJ_DTYPE = None  # numpy structured dtype, built lazily


def _np_dtypes():
    import numpy as np
    global OBJ_DTYPE
    if OBJ_DTYPE is None:
        OBJ_DTYPE = {
            "stats": np.dtype([("max_q", "f8"), ("min_q", "f8"), ("sum_q", "f8"), ("pct_max", "f8"),
                               ("count_max", "i8"), ("n", "i8"), ("has_nan", "i4"), ("has_inf", "i4"),
                               ("_pad", "i8")]),
            "qc": np.dtype([("slope", "f8"), ("pct_max", "f8"), ("n_valid", "i4"), ("n_rings", "i4")]),
            "object": np.dtype([("label", "i4"), ("area", "i4"), ("bbox", "i4", (4,)),
                                ("centroid_r", "f8"), ("centroid_c", "f8"), ("yc", "i4"), ("xc", "i4"),
                                ("kept", "i4"), ("cell_idx", "i4")]),
            "hdr": np.dtype([("n_objects", "i4"), ("n_kept", "i4"), ("max_label", "i4"),
                             ("overflow", "i4")]),
        }
        assert OBJ_DTYPE["stats"].itemsize == _STATS_BYTES
        assert OBJ_DTYPE["qc"].itemsize == _QC_BYTES
        assert OBJ_DTYPE["object"].itemsize == _OBJ_BYTES
        assert OBJ_DTYPE["hdr"].itemsize == _HDR_BYTES
    return OBJ_DTYPE


def _ptr(t: torch.Tensor | None):
    if t is None:
        return None
    assert t.is_cuda and t.is_contiguous(), "libcpx needs contiguous device tensors"
    return ct.c_void_p(t.data_ptr())


def _illum_dtype(illum: torch.Tensor | None) -> int:
    if illum is None:
        return _lib.CPX_DTYPE_NONE
    if illum.dtype == torch.float32:
        return _lib.CPX_DTYPE_F32
    if illum.dtype == torch.float64:
        return _lib.CPX_DTYPE_F64
    raise TypeError(f"illumination function dtype {illum.dtype} unsupported (float32/float64)")


class Device:
    """One libcpx context bound to one GPU and to torch's current stream on it."""

    def __init__(self, device: int = 0):
        if not torch.cuda.is_available():
            raise _lib.CpxNativeMissing("no HIP device visible: the product path has no CPU fallback")
        self.lib = _lib.load()
        self.index = device
        self.torch_device = torch.device("cuda", device)
        torch.cuda.set_device(self.torch_device)
        h = ct.c_void_p()
        check(self.lib.cpx_init(device, ct.byref(h)), "cpx_init")
        self.h = h
        self._bind_stream()

    def _bind_stream(self):
        s = torch.cuda.current_stream(self.torch_device).cuda_stream
        check(self.lib.cpx_set_stream(self.h, ct.c_void_p(s)), "cpx_set_stream")

    def close(self):
        if getattr(self, "h", None):
            self.lib.cpx_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        check(self.lib.cpx_sync(self.h), "cpx_sync")

    def reserve(self, max_planes: int, H: int, W: int, max_fovs: int = 0, max_label: int = 0):
        check(self.lib.cpx_reserve(self.h, max_planes, H, W, max_fovs, max_label), "cpx_reserve")

    # ---- raw buffers -----------------------------------------------------------------------
    def empty_bytes(self, nbytes: int) -> torch.Tensor:
        return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=self.torch_device)

    # ---- a1 + a4 ---------------------------------------------------------------------------
    def illum_correct(self, raw: torch.Tensor, illum: torch.Tensor | None, C: int,
                      corr: torch.Tensor | None, stats: torch.Tensor):
        """raw: uint16 [n_planes, H, W] (int16 view ok); illum: [C,H,W] f32/f64 or None."""
        n, H, W = raw.shape[-3], raw.shape[-2], raw.shape[-1]
        self._bind_stream()
        check(self.lib.cpx_illum_correct(self.h, _ptr(raw), _ptr(illum), _illum_dtype(illum), C, n, H, W,
                                         _ptr(corr), _ptr(stats)), "cpx_illum_correct")

    # ---- a2 + a3 ---------------------------------------------------------------------------
    def qc_rps(self, raw: torch.Tensor, illum: torch.Tensor | None, C: int, stats: torch.Tensor,
               qc: torch.Tensor, powersum: torch.Tensor | None = None):
        n, H, W = raw.shape[-3], raw.shape[-2], raw.shape[-1]
        self._bind_stream()
        check(self.lib.cpx_qc_rps(self.h, _ptr(raw), _ptr(illum), _illum_dtype(illum), C, n, H, W,
                                  _ptr(stats), _ptr(powersum), _ptr(qc)), "cpx_qc_rps")

    # ---- a5 ------------------------------------------------------------------------------
    def zmax(self, src: torch.Tensor, out: torch.Tensor):
        """src: uint16 [G, Z, ...] ; out: uint16 [G, ...]."""
        G, Z = src.shape[0], src.shape[1]
        N = src[0, 0].numel()
        self._bind_stream()
        check(self.lib.cpx_zmax_u16(self.h, _ptr(src), G, Z, N, _ptr(out)), "cpx_zmax_u16")

    # ---- 8(f) rank 4: re-binning ------------------------------------------------------------
    def rebin(self, src: torch.Tensor, out_h: int, out_w: int, out: torch.Tensor):
        """src: uint16 bits (int16) [G, H, W] ; out: [G, out_h, out_w] (PIL LANCZOS resize)."""
        G, H, W = src.shape
        assert src.is_contiguous() and out.is_contiguous() and tuple(out.shape) == (G, out_h, out_w)
        self._bind_stream()
        check(self.lib.cpx_rebin_u16(self.h, _ptr(src), G, H, W, out_h, out_w, _ptr(out)), "cpx_rebin_u16")

    # ---- 8(f) rank 1: per-time profiles ------------------------------------------------------
    def group_kahan(self, values: torch.Tensor, order: torch.Tensor, offs: torch.Tensor,
                    sumx: torch.Tensor, comp: torch.Tensor, nobs: torch.Tensor,
                    row_scale: torch.Tensor | None = None, col_scaled: torch.Tensor | None = None):
        """values fp64 [n, ld] (first K = sumx.shape[1] columns); order/offs int32; state [G, K];
        optional fp64 row_scale [n] applied to the columns where uint8 col_scaled [K] != 0."""
        n, ld = values.shape
        G, K = sumx.shape
        assert values.dtype == torch.float64 and values.is_contiguous() and K <= ld
        assert order.dtype == torch.int32 and offs.dtype == torch.int32 and offs.numel() == G + 1
        assert comp.shape == sumx.shape and nobs.shape == sumx.shape and nobs.dtype == torch.int64
        self._bind_stream()
        if row_scale is not None:
            assert row_scale.dtype == torch.float64 and row_scale.numel() == n
            assert col_scaled is not None and col_scaled.dtype == torch.uint8 and col_scaled.numel() == K
        check(self.lib.cpx_group_kahan_accumulate(self.h, _ptr(values), n, K, ld, _ptr(order),
                                                  _ptr(offs), G, _ptr(row_scale), _ptr(col_scaled),
                                                  _ptr(sumx), _ptr(comp), _ptr(nobs)),
              "cpx_group_kahan_accumulate")

    def group_median(self, values: torch.Tensor, order: torch.Tensor, offs: torch.Tensor,
                     max_group_rows: int, out: torch.Tensor, row_scale: torch.Tensor | None = None,
                     col_scaled: torch.Tensor | None = None):
        n, ld = values.shape
        G, K = out.shape
        assert values.dtype == torch.float64 and values.is_contiguous() and K <= ld
        self._bind_stream()
        check(self.lib.cpx_group_median(self.h, _ptr(values), n, K, ld, _ptr(order), _ptr(offs), G,
                                        int(max_group_rows), _ptr(row_scale), _ptr(col_scaled), _ptr(out)),
              "cpx_group_median")

    def group_finalize(self, sumx: torch.Tensor, nobs: torch.Tensor, out: torch.Tensor):
        G, K = sumx.shape
        assert out.shape == sumx.shape and out.dtype == torch.float64
        self._bind_stream()
        check(self.lib.cpx_group_mean_finalize(self.h, _ptr(sumx), _ptr(nobs), G, K, _ptr(out)),
              "cpx_group_mean_finalize")

    def nancorr(self, colmajor: torch.Tensor, out: torch.Tensor):
        """colmajor fp64 [K, N] (one row per feature) -> out [K, K]."""
        K, N = colmajor.shape
        assert colmajor.is_contiguous() and out.shape == (K, K)
        self._bind_stream()
        check(self.lib.cpx_nancorr(self.h, _ptr(colmajor), N, K, _ptr(out)), "cpx_nancorr")

    def robust_mad(self, colmajor: torch.Tensor, fit_rows: torch.Tensor, scale: float,
                   med: torch.Tensor, mad: torch.Tensor):
        K, N = colmajor.shape
        assert colmajor.is_contiguous() and fit_rows.dtype == torch.int32
        self._bind_stream()
        check(self.lib.cpx_robust_mad(self.h, _ptr(colmajor), N, K, _ptr(fit_rows), fit_rows.numel(),
                                      float(scale), _ptr(med), _ptr(mad)), "cpx_robust_mad")

    def mad_transform(self, colmajor: torch.Tensor, med, mad, eps: float, out,
                      double_sigmoid: bool = False, alpha: float = 1.0):
        K, N = colmajor.shape
        assert colmajor.is_contiguous() and out.shape == colmajor.shape
        self._bind_stream()
        check(self.lib.cpx_mad_transform(self.h, _ptr(colmajor), N, K, _ptr(med), _ptr(mad), float(eps),
                                         int(bool(double_sigmoid)), float(alpha), _ptr(out)),
              "cpx_mad_transform")

    def column_stats(self, colmajor: torch.Tensor, stats: torch.Tensor):
        """stats: uint8 [K * 48] (cpx_column_stat[K])."""
        K, N = colmajor.shape
        assert colmajor.is_contiguous() and stats.numel() >= 48 * K
        self._bind_stream()
        check(self.lib.cpx_column_stats(self.h, _ptr(colmajor), N, K, _ptr(stats)), "cpx_column_stats")

    def cosine_groups(self, x: torch.Tensor, offs: torch.Tensor, pair_offs: torch.Tensor,
                      norms: torch.Tensor, out: torch.Tensor):
        N, F = x.shape
        G = offs.numel() - 1
        assert x.is_contiguous() and offs.dtype == torch.int32 and pair_offs.dtype == torch.int64
        self._bind_stream()
        check(self.lib.cpx_cosine_groups(self.h, _ptr(x), N, F, _ptr(offs), _ptr(pair_offs), G,
                                         out.numel(), _ptr(norms), _ptr(out)), "cpx_cosine_groups")

    # ---- a7 ------------------------------------------------------------------------------
    def objects(self, labels: torch.Tensor, max_label: int, box: int, lstats: torch.Tensor,
                objects: torch.Tensor, hdr: torch.Tensor):
        B, H, W = labels.shape
        self._bind_stream()
        check(self.lib.cpx_objects(self.h, _ptr(labels), B, H, W, max_label, box, _ptr(lstats),
                                   _ptr(objects), _ptr(hdr)), "cpx_objects")

    def crops(self, labels, corr, C, max_label, objects, hdr, box, max_crops, crops, crops8=None):
        B, H, W = labels.shape
        self._bind_stream()
        check(self.lib.cpx_crops(self.h, _ptr(labels), _ptr(corr), B, C, H, W, max_label, _ptr(objects),
                                 _ptr(hdr), box, max_crops, _ptr(crops), _ptr(crops8)), "cpx_crops")

    # ---- a8 ------------------------------------------------------------------------------
    def features(self, labels, corr, C, max_label, objects, hdr, feats):
        B, H, W = labels.shape
        self._bind_stream()
        check(self.lib.cpx_features(self.h, _ptr(labels), _ptr(corr), B, C, H, W, max_label,
                                    _ptr(objects), _ptr(hdr), _ptr(feats)), "cpx_features")

    def features_pair(self, cells, cyto, corr, C, max_label, cells_tab, cyto_tab):
        """cpx_features of Cells and Cytoplasm in one call; *_tab = (objects, hdr, feats)."""
        B, H, W = cells.shape
        self._bind_stream()
        check(self.lib.cpx_features_pair(self.h, _ptr(cells), _ptr(cyto), _ptr(corr), B, C, H, W, max_label,
                                         *(_ptr(t) for t in cells_tab), *(_ptr(t) for t in cyto_tab)),
              "cpx_features_pair")


# Pipeline streams with their own CUs (round 5): two pipelines whose streams each hold a CU mask
# of one contiguous half of the GPU's CUs (hipExtStreamCreateWithCUMask) ran the bench 0.8-0.9 %
# faster than two unrestricted streams, four of four same-box pairs (`gpurun_out/r05as`,
# `r05at`: 457.0 -> 461.1 FOV/s): the two batches' kernels stop evicting each other from the
# CUs' LDS and L2 while the stage exclusivity (pipeline.STAGE_EXCLUSIVE) still keeps their CPnets
# apart; interleaved CUs measured no better than none, dropping the exclusivity 2 % worse,
# three pipelines in thirds 18 % worse.  Callers choose with `split` (bench.py --cu-split).


class _MaskedStreams:
    """Owner of the CU-masked pipeline streams: created once per (device, n, split) by libcpx
    (cpx_stream_create_cu_mask — the HIP runtime libcpx and torch share, never a second copy of
    libamdhip64), handed out as torch ExternalStreams, and destroyed at interpreter exit after
    their work has drained (each holds a hardware queue; round 5 created a fresh pair per call
    from ctypes and never released them)."""
    _cache: dict = {}

    @classmethod
    def get(cls, td: torch.device, n: int, split: str) -> list:
        key = (td.index, n, split)
        if key not in cls._cache:
            if not cls._cache:
                atexit.register(cls.release_all)
            lib = _lib.load()
            n_cu = torch.cuda.get_device_properties(td).multi_processor_count
            handles = []
            try:
                for p in range(n):
                    words = (ct.c_uint32 * ((n_cu + 31) // 32))()
                    for i in range(n_cu):
                        if (i % n == p) if split == "interleave" else (i * n // n_cu == p):
                            words[i // 32] |= 1 << (i % 32)
                    h = ct.c_void_p()
                    check(lib.cpx_stream_create_cu_mask(td.index, words, len(words), ct.byref(h)),
                          "cpx_stream_create_cu_mask")
                    handles.append(h.value)
            except Exception:
                for h in handles:
                    lib.cpx_stream_destroy(ct.c_void_p(h))
                raise
            cls._cache[key] = (handles, [torch.cuda.ExternalStream(h, device=td) for h in handles])
        return list(cls._cache[key][1])

    @classmethod
    def release_all(cls):
        lib = _lib._lib
        for handles, _ in cls._cache.values():
            for h in handles:
                if lib is not None:
                    lib.cpx_stream_destroy(ct.c_void_p(h))
        cls._cache.clear()


def pipeline_streams(device, n: int, split: str | None = None) -> list:
    """HIP streams for n pipelines on `device`: with split "halves" (the default for n == 2) each
    stream is restricted to a contiguous 1/n of the CUs, "interleave" to every n-th CU, "none"
    plain torch streams.  The masked streams are shared per (device, n, split) for the process
    and released at exit (_MaskedStreams)."""
    td = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
    if td.index is None:
        td = torch.device("cuda", torch.cuda.current_device())
    split = split or "auto"
    if split == "auto":
        split = "halves" if n == 2 else "none"
    if split == "none" or n < 2:
        return [torch.cuda.Stream(device=td) for _ in range(n)]
    if split not in ("halves", "interleave"):
        raise ValueError(f"pipeline_streams: split {split!r}")
    return _MaskedStreams.get(td, n, split)


def n_features(C: int) -> int:
    return _lib.N_SHAPE + C * _lib.FEATURES_PER_CHANNEL


def as_numpy(t: torch.Tensor, kind: str):
    """View a raw byte tensor (device or host) as a numpy structured array of `kind`."""
    import numpy as np
    dt = _np_dtypes()[kind]
    b = t.detach().cpu().numpy().view(np.uint8)
    return b[: (b.size // dt.itemsize) * dt.itemsize].view(dt)
