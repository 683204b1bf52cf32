"""Per-FOV session over the C ABI's drop-in boundary (include/cpx.h, "per-FOV drop-in boundary").

One session = one libcpx context on one GPU, driven one FOV at a time like the reference's
per-site workers (Illumination_QC_mult.process_site, MaxProjection.max_projection, the
Cellpose_GPU_s3fs consumer).  Host numpy planes go in, host numpy tables come out; the session
owns all device memory.  This is the path a non-torch caller binds; the
batched `cpx.pipeline` path is the throughput path used by bench.py.
"""
from __future__ import annotations

import ctypes as ct
import threading

import numpy as np

from . import _lib
from ._lib import check
from .device import n_features


class FovSession:
    def __init__(self, device: int = 0):
        import torch  # device memory for label images and the stream/runtime binding
        if not torch.cuda.is_available():
            raise _lib.CpxNativeMissing("no HIP device visible: the product path has no CPU fallback")
        self.torch = torch
        self.lib = _lib.load()
        self.td = torch.device("cuda", device)
        torch.cuda.set_device(self.td)
        h = ct.c_void_p()
        check(self.lib.cpx_init(device, ct.byref(h)), "cpx_init")
        self.h = h
        check(self.lib.cpx_set_stream(self.h, ct.c_void_p(torch.cuda.current_stream(self.td).cuda_stream)),
              "cpx_set_stream")
        self.lock = threading.Lock()  # a context is single-threaded
        self._illum_ids = {}
        self.C = self.H = self.W = 0

    # -- illumination cache ----------------------------------------------------------------------
    def set_illum(self, ch: int, illum: np.ndarray | None):
        """Upload channel `ch`'s flat-field (float32/float64 [H][W]) or clear it (None).
        Re-uploads are skipped when the same array object is passed again."""
        key = None if illum is None else (id(illum), illum.shape, illum.dtype.str)
        if self._illum_ids.get(ch, "unset") == key:
            return
        if illum is None:
            check(self.lib.cpx_set_illum(self.h, ch, None, _lib.CPX_DTYPE_NONE, 0, 0), "cpx_set_illum")
        else:
            a = np.ascontiguousarray(illum)
            if a.dtype == np.float32:
                dt = _lib.CPX_DTYPE_F32
            elif a.dtype == np.float64:
                dt = _lib.CPX_DTYPE_F64
            else:
                a = a.astype(np.float64)
                dt = _lib.CPX_DTYPE_F64
            check(self.lib.cpx_set_illum(self.h, ch, a.ctypes.data_as(ct.c_void_p), dt, a.shape[0], a.shape[1]),
                  "cpx_set_illum")
        self._illum_ids[ch] = key

    # -- one FOV ---------------------------------------------------------------------------------
    def submit(self, planes, C: int, Z: int = 1, site_id: int = 0):
        """planes: C*Z uint16 [H][W] arrays in plane-major order (planes[z*C + c])."""
        assert len(planes) == C * Z
        arrs = [np.ascontiguousarray(p, dtype=np.uint16) for p in planes]
        H, W = arrs[0].shape
        for a in arrs:
            if a.shape != (H, W):
                raise ValueError(f"Image shape mismatch in group: {[x.shape for x in arrs]}")
        ptrs = (ct.c_void_p * len(arrs))(*[a.ctypes.data_as(ct.c_void_p) for a in arrs])
        self._keep = arrs  # valid until the next synchronising call
        check(self.lib.cpx_fov_submit(self.h, int(site_id), ptrs, C, Z, H, W), "cpx_fov_submit")
        self.C, self.H, self.W = C, H, W

    def qc(self):
        """(slope[C], pct_max[C], status[C]) of the submitted FOV."""
        C = self.C
        slope = np.empty(C, np.float64)
        pct = np.empty(C, np.float64)
        st = np.empty(C, np.int32)
        check(self.lib.cpx_fov_qc(self.h, slope.ctypes.data_as(ct.c_void_p), pct.ctypes.data_as(ct.c_void_p),
                                  st.ctypes.data_as(ct.c_void_p)), "cpx_fov_qc")
        return slope, pct, st

    def read_plane(self, ch: int) -> np.ndarray:
        out = np.empty((self.H, self.W), np.uint16)
        check(self.lib.cpx_fov_read_plane(self.h, ch, out.ctypes.data_as(ct.c_void_p)), "cpx_fov_read_plane")
        return out

    def corrected(self):
        """Torch view of the corrected float32 planes [C][H][W] (device, until the next submit)."""
        p = ct.c_void_p()
        check(self.lib.cpx_fov_planes(self.h, ct.byref(p), None), "cpx_fov_planes")
        return self.torch.as_tensor(_DevPtr(p.value, (self.C, self.H, self.W), "<f4"), device=self.td)

    def object_table(self, labels, box: int = 200, max_objects: int = 4096):
        lab = self._labels(labels)
        out = (ct.c_ubyte * (56 * max_objects))()
        n = ct.c_int()
        check(self.lib.cpx_fov_object_table(self.h, ct.c_void_p(lab.data_ptr()), box, max_objects,
                                            out, ct.byref(n)), "cpx_fov_object_table")
        arr = np.frombuffer(bytes(out)[: 56 * n.value], dtype=np.uint8)
        return as_numpy_bytes(arr, "object")

    def features(self, labels, max_objects: int = 4096) -> np.ndarray:
        lab = self._labels(labels)
        F = n_features(self.C)
        out = np.empty((max_objects, F), np.float64)
        n = ct.c_int()
        check(self.lib.cpx_fov_features(self.h, ct.c_void_p(lab.data_ptr()), max_objects,
                                        out.ctypes.data_as(ct.c_void_p), ct.byref(n)), "cpx_fov_features")
        return out[: n.value].copy()

    def _labels(self, labels):
        t = self.torch
        if isinstance(labels, np.ndarray):
            assert labels.shape == (self.H, self.W)
            return t.from_numpy(np.ascontiguousarray(labels, dtype=np.int32)).to(self.td)
        assert labels.is_cuda and labels.dtype == t.int32 and labels.is_contiguous()
        return labels

    def wait(self):
        check(self.lib.cpx_fov_wait(self.h), "cpx_fov_wait")

    def close(self):
        if getattr(self, "h", None):
            self.lib.cpx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _DevPtr:
    """__cuda_array_interface__ view of a device buffer owned by the session."""

    def __init__(self, ptr, shape, typestr):
        self.__cuda_array_interface__ = {"shape": shape, "typestr": typestr, "data": (ptr, False),
                                         "version": 3, "strides": None}


def as_numpy_bytes(arr: np.ndarray, kind: str) -> np.ndarray:
    from .device import _np_dtypes
    return arr.view(_np_dtypes()[kind])
