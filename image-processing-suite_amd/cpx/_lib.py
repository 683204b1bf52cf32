"""ctypes binding of libcpx.so — the C ABI declared in include/cpx.h.

This module is the only place that knows the native signatures.  It never falls back to a
Python implementation: if the shared library is missing or fails to load, every product entry
point raises :class:`CpxNativeMissing` (the CPU restatement under ``oracle/`` is test
infrastructure only and is never imported from the product package).
"""
from __future__ import annotations

import ctypes as ct
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CPX_LIB", os.path.join(_HERE, "libcpx.so"))

CPX_OK = 0
CPX_DTYPE_NONE, CPX_DTYPE_F32, CPX_DTYPE_F64, CPX_DTYPE_IMAGE_F64 = 0, 1, 2, 3
CPX_QC_OK, CPX_QC_FLAT, CPX_QC_NAN = 0, 1, 2

# feature layout constants (mirror include/cpx.h)
N_SHAPE = 15
N_INT = 5
N_TEX_PROPS = 6
N_ANGLES = 4
N_TEX = N_TEX_PROPS * N_ANGLES
FEATURES_PER_CHANNEL = N_INT + N_TEX
TEX_DISTANCE = 3


class CpxError(RuntimeError):
    """A libcpx entry point returned a non-zero status."""


class CpxNativeMissing(CpxError):
    """libcpx.so could not be loaded (the product path has no CPU fallback)."""


class PlaneStats(ct.Structure):
    _fields_ = [("max_q", ct.c_double), ("min_q", ct.c_double), ("sum_q", ct.c_double),
                ("pct_max", ct.c_double), ("count_max", ct.c_int64), ("n", ct.c_int64),
                ("has_nan", ct.c_int32), ("has_inf", ct.c_int32), ("_pad", ct.c_int64)]


class QcResult(ct.Structure):
    _fields_ = [("slope", ct.c_double), ("pct_max", ct.c_double), ("n_valid", ct.c_int32),
                ("n_rings", ct.c_int32)]


class LabelStats(ct.Structure):
    _fields_ = [("area", ct.c_int64), ("sum_r", ct.c_int64), ("sum_c", ct.c_int64),
                ("sum_rr", ct.c_int64), ("sum_cc", ct.c_int64), ("sum_rc", ct.c_int64),
                ("rmin", ct.c_int32), ("rmax", ct.c_int32), ("cmin", ct.c_int32),
                ("cmax", ct.c_int32)]


class Object(ct.Structure):
    _fields_ = [("label", ct.c_int32), ("area", ct.c_int32), ("bbox", ct.c_int32 * 4),
                ("centroid_r", ct.c_double), ("centroid_c", ct.c_double), ("yc", ct.c_int32),
                ("xc", ct.c_int32), ("kept", ct.c_int32), ("cell_idx", ct.c_int32)]


class FovObjects(ct.Structure):
    _fields_ = [("n_objects", ct.c_int32), ("n_kept", ct.c_int32), ("max_label", ct.c_int32),
                ("overflow", ct.c_int32)]


class ColumnStat(ct.Structure):
    _fields_ = [("na_count", ct.c_int64), ("nunique", ct.c_int64), ("top_count", ct.c_int64),
                ("second_count", ct.c_int64), ("max", ct.c_double), ("min", ct.c_double)]


SIZES = {"cpx_column_stat": 48, "cpx_plane_stats": 64, "cpx_qc_result": 24, "cpx_label_stats": 64, "cpx_object": 56,
         "cpx_fov_objects": 16}

_P = ct.c_void_p
_I = ct.c_int
_I64 = ct.c_int64

# name -> (restype, argtypes); every symbol declared in include/cpx.h
SIGNATURES = {
    "cpx_abi_version": (_I, []),
    "cpx_init": (_I, [_I, ct.POINTER(_P)]),
    "cpx_destroy": (None, [_P]),
    "cpx_last_error": (ct.c_char_p, []),
    "cpx_set_stream": (_I, [_P, _P]),
    "cpx_sync": (_I, [_P]),
    "cpx_stream_create_cu_mask": (_I, [_I, _P, _I, _P]),
    "cpx_stream_destroy": (_I, [_P]),
    "cpx_reserve": (_I, [_P, _I, _I, _I, _I, _I]),
    "cpx_illum_correct": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "cpx_qc_rps": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "cpx_zmax_u16": (_I, [_P, _P, _I, _I, _I64, _P]),
    "cpx_rebin_u16": (_I, [_P, _P, _I, _I, _I, _I, _I, _P]),
    "cpx_group_kahan_accumulate": (_I, [_P, _P, _I, _I, ct.c_longlong, _P, _P, _I, _P, _P, _P, _P, _P]),
    "cpx_group_mean_finalize": (_I, [_P, _P, _P, _I, _I, _P]),
    "cpx_group_median": (_I, [_P, _P, _I, _I, ct.c_longlong, _P, _P, _I, _I, _P, _P, _P]),
    "cpx_nancorr": (_I, [_P, _P, _I, _I, _P]),
    "cpx_robust_mad": (_I, [_P, _P, _I, _I, _P, _I, ct.c_double, _P, _P]),
    "cpx_mad_transform": (_I, [_P, _P, _I, _I, _P, _P, ct.c_double, _I, ct.c_double, _P]),
    "cpx_column_stats": (_I, [_P, _P, _I, _I, _P]),
    "cpx_cosine_groups": (_I, [_P, _P, _I, _I, _P, _P, _I, ct.c_longlong, _P, _P]),
    "cpx_objects": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "cpx_crops": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _I, _I, _P, _P]),
    "cpx_features": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "cpx_features_pair": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "cpx_csv_format": (_I64, [_I64, _I64, _I, _P, _P, _P, _P, _I64]),
    "cpx_debug_glcm_timing": (_I, [_P, _I]),
    "cpx_debug_glcm_ms": (_I, [_P, ct.POINTER(ct.c_double), ct.POINTER(_I)]),
    "cpx_debug_seg_timing": (_I, [_P, _I]),
    "cpx_debug_seg_stats": (_I, [_P, ct.POINTER(ct.c_double), ct.POINTER(ct.c_double), ct.POINTER(ct.c_double),
                                 ct.POINTER(_I)]),
    "cpx_expand_labels": (_I, [_P, _P, _I, _I, _I, _I, _P, _P]),
    "cpx_watershed_cells": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _I]),
    "cpx_seg_percentiles": (_I, [_P, _P, _I, _I, _I, _I, _I, _P]),
    "cpx_seg_tiles": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _I, _P]),
    "cpx_seg_average": (_I, [_P, _P, _I, _I, _I, _P, _P, _P]),
    "cpx_embed_preprocess": (_I, [_P, _P, _P, _I, _I, _I, ct.c_float, ct.c_float, _P]),
    "cpx_effnet_stem": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P]),
    "cpx_effnet_conv": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _I, _P, _P, _P]),
    "cpx_effnet_dw": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
    "cpx_effnet_dw_blocks": (_I, [_I, _I, _I]),
    "cpx_effnet_se": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
    "cpx_effnet_pool": (_I, [_P, _P, _I, _I, _I, _P]),
    "cpx_seg_masks": (_I, [_P, _P, _I, _P, _I, _I, _I, ct.c_double, _I, _I, _I, _P, _P]),
    "cpx_cpnet_epilogue": (_I, [_P, _P, _P, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _I]),
    "cpx_cpnet_pool": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "cpx_cpnet_conv_cfg": (_I, [_I, _I, _P, _P]),
    "cpx_set_illum": (_I, [_P, _I, _P, _I, _I, _I]),
    "cpx_fov_submit": (_I, [_P, ct.c_int64, _P, _I, _I, _I, _I]),
    "cpx_fov_qc": (_I, [_P, _P, _P, _P]),
    "cpx_fov_planes": (_I, [_P, _P, _P]),
    "cpx_fov_read_plane": (_I, [_P, _I, _P]),
    "cpx_fov_segment_post": (_I, [_P, _P, _I, _P, _P, _I, ct.c_double, _I, _I, _I, _P, _P]),
    "cpx_fov_object_table": (_I, [_P, _P, _I, _I, _P, _P]),
    "cpx_fov_features": (_I, [_P, _P, _I, _P, _P]),
    "cpx_fov_wait": (_I, [_P]),
    "cpx_cpnet_conv3x3": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _I, _P, _P, _P, _I, _P, _P, _I]),
    "cpx_cpnet_conv3x3_head": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _I, _P, _P, _P, _I, _P,
                                    _P, _P, _I, _P]),
    "cpx_cpnet_stem": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "cpx_cpnet_x3_cfg": (_I, [_I, _I, _I, _I, _P]),
    "cpx_cpnet_x3_conv": (_I, [_P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _I, _P, _I, _P, _P, _I,
                               _P, _P, _I, _P, _P, _I, _P, _P]),
    "cpx_cpnet_x3_conv_proj": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _P, _P, _I, _P, _P, _P, _I, _P, _P, _I,
                                    _P, _P, _I, _P]),
    "cpx_cpnet_x3_conv_pool": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "cpx_cpnet_x3_mask_overflow": (_I, [_P, _P, _I, _I, _I, _I, _P]),
    "cpx_cpnet_x3_stem": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "cpx_cpnet_x3_pool": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "cpx_cpnet_x3_style": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _I, _P]),
}

_lib = None
_lock = threading.Lock()


def load(path: str | None = None):
    """Load libcpx.so once and attach the signatures; raises CpxNativeMissing on failure."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or LIB_PATH
        # libcpx must bind to the SAME HIP runtime as torch: torch ships its own
        # libamdhip64.so (SONAME libamdhip64.so.7); loading torch first makes libcpx's
        # NEEDED libamdhip64.so.7 resolve to that already-loaded copy (one runtime, one set of
        # streams).  Loading libcpx first would pull /opt/rocm's copy and a second HSA runtime.
        try:
            import torch  # noqa: F401
        except ImportError:  # pure-C consumers: /opt/rocm runtime is used
            pass
        if not os.path.exists(p):
            raise CpxNativeMissing(
                f"libcpx.so not found at {p}; build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        try:
            lib = ct.CDLL(p)
        except OSError as e:  # pragma: no cover - depends on the runtime
            raise CpxNativeMissing(f"failed to load {p}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def exported_symbols() -> list[str]:
    return list(SIGNATURES)


def check(status: int, what: str) -> None:
    if status != CPX_OK:
        msg = _lib.cpx_last_error().decode(errors="replace") if _lib is not None else ""
        raise CpxError(f"{what} failed with status {status}: {msg}")
