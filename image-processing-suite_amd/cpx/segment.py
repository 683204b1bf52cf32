"""Segmentation host logic — the MI355X replacement for ``cell_model.eval(image_4ch, diameter=100)``
(Cellpose_GPU_s3fs.py:108,143), Cellpose <= v3 semantics as pinned in DESIGN.md §Segmentation.

Pipeline per batch of FOVs (all device-resident, one HIP stream):
  libcpx cpx_seg_percentiles -> cpx_seg_tiles (bf16 NHWC) -> CPnet forward (native MFMA
  convolutions, HIP-graph captured) -> cpx_seg_average -> cpx_seg_masks -> int32 labels [B,H,W].
Every other eval() argument is at Cellpose's default: resample=True (the averaged flows are
resized to H x W and the dynamics run at full resolution) with niter = uint32(1 / rescale * 200)
(_run_cp; 1176 for the nuclei model at diameter 100).  resample=False is a named option.
"""
from __future__ import annotations

import ctypes as ct
import math
import warnings

import numpy as np
import torch

from . import _lib
from ._lib import check
from .cpnet import build_cpnet
from .cpnet_fused import FusedCPnet
from .cpnet_x3 import FusedCPnetX3
from .device import Device, _ptr

DIAM_MEAN = {"nuclei": 17.0, "cyto": 30.0, "cyto2": 30.0, "cyto3": 30.0}
_capture_streams: dict = {}  # device index -> CPnet warm-up / graph-capture stream

CELLPOSE_MODEL = "nuclei"  # Cellpose_GPU_s3fs.py:28
DIAMETER = 100.0           # Cellpose_GPU_s3fs.py:143
BSIZE = 224
TILE_OVERLAP = 0.1
RESAMPLE = True           # CellposeModel.eval default (the reference passes only diameter)
NITER_NET = 200           # Cellpose 2.x's steps when the dynamics run at network size


def default_niter(model: str = CELLPOSE_MODEL, diameter: float = DIAMETER, resample: bool = RESAMPLE) -> int:
    """CellposeModel._run_cp: niter = 1 / rescale * 200 (rescale = diam_mean / diameter), cast
    to uint32 by dynamics.follow_flows."""
    if not resample:
        return NITER_NET
    rescale = DIAM_MEAN[model] / diameter
    return int(np.uint32(1 / rescale * 200))
FLOW_THRESHOLD = 0.4
MIN_SIZE = 15
NET_CHANNELS = 2


class SegGeom(ct.Structure):
    _fields_ = [("Ly", ct.c_int32), ("Lx", ct.c_int32), ("py0", ct.c_int32), ("px0", ct.c_int32),
                ("Lyp", ct.c_int32), ("Lxp", ct.c_int32), ("by", ct.c_int32), ("bx", ct.c_int32),
                ("ny", ct.c_int32), ("nx", ct.c_int32), ("ys", ct.c_int32 * 16), ("xs", ct.c_int32 * 16)]

    @property
    def n_tiles(self):
        return self.ny * self.nx


SEG_STATS_DTYPE = np.dtype([("n_moving", "i4"), ("n_seeds", "i4"), ("n_masks", "i4"),
                            ("n_bad_flow", "i4"), ("n_final", "i4"), ("overflow", "i4"), ("cells_status", "i4"), ("n_seeds_found", "i4"),
                            ("n_fill_partial", "i4"), ("_reserved", "i4", (3,))])
SEG_STATS_BYTES = 48
assert SEG_STATS_DTYPE.itemsize == SEG_STATS_BYTES
SEG_OVF_FILL_PARTIAL = 2  # cpx.h CPX_SEG_OVF_FILL_PARTIAL: a partly absorbed mask; the FOV took the sequential fill
SEG_OVF_SEEDS = 1        # cpx.h CPX_SEG_OVF_SEEDS: more seeds than max_objects (re-run with more)
SEG_ERR_INTERNAL = 8     # cpx.h CPX_SEG_ERR_INTERNAL: a flow-error work loop hit its claim bound


def _pad_amounts(L: int, div: int = 16, extra: int = 1):
    """transforms.pad_image_ND padding (multiple of div, plus extra*div//2 on each side)."""
    Lpad = int(div * math.ceil(L / div) - L)
    return extra * div // 2 + Lpad // 2, extra * div // 2 + Lpad - Lpad // 2


def _tile_starts(Lp: int, bsize: int = BSIZE, overlap: float = TILE_OVERLAP):
    """transforms.make_tiles (augment=False) origins along one axis."""
    overlap = min(0.5, max(0.05, overlap))
    b = min(bsize, Lp)
    n = 1 if Lp <= bsize else int(math.ceil((1.0 + 2 * overlap) * Lp / bsize))
    return np.linspace(0, Lp - b, n).astype(int), b


def make_geom(H: int, W: int, model: str = CELLPOSE_MODEL, diameter: float = DIAMETER) -> SegGeom:
    rescale = DIAM_MEAN[model] / diameter
    Ly, Lx = int(H * rescale), int(W * rescale)
    g = SegGeom()
    g.Ly, g.Lx = Ly, Lx
    py0, py1 = _pad_amounts(Ly)
    px0, px1 = _pad_amounts(Lx)
    g.py0, g.px0 = py0, px0
    g.Lyp, g.Lxp = Ly + py0 + py1, Lx + px0 + px1
    ys, g.by = _tile_starts(g.Lyp)
    xs, g.bx = _tile_starts(g.Lxp)
    if len(ys) > 16 or len(xs) > 16:
        raise ValueError("too many tiles per axis")
    g.ny, g.nx = len(ys), len(xs)
    for i, v in enumerate(ys):
        g.ys[i] = int(v)
    for i, v in enumerate(xs):
        g.xs[i] = int(v)
    return g


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


class Segmenter:
    """Batched segmentation on one device.  `segment(corr)` takes device fp32 planes
    [B, C, H, W] and returns device int32 labels [B, H, W]."""

    def __init__(self, dev: Device, H: int, W: int, batch: int, model: str = CELLPOSE_MODEL,
                 diameter: float = DIAMETER, weights: str | None = None, seed: int = 0,
                 use_graph: bool = True, max_objects: int = 4096, net_dtype=torch.bfloat16,
                 fused: bool = True, resample: bool = RESAMPLE,
                 niter: int | None = None, flow_threshold: float = FLOW_THRESHOLD, min_size: int = MIN_SIZE,
                 precision: str | None = None):
        self.dev = dev
        self.H, self.W, self.B = H, W, batch
        self.geom = make_geom(H, W, model, diameter)
        g = self.geom
        td = dev.torch_device
        self.max_objects = max_objects
        self.resample = bool(resample)
        self.niter = default_niter(model, diameter, self.resample) if niter is None else int(niter)
        self.flow_threshold, self.min_size = flow_threshold, min_size
        # precision: "f16x3" (default: native split-fp16 MFMA kernels at the fp32 network's
        # accuracy, cpx.cpnet_x3), "bf16" (native bf16 MFMA kernels, cpx.cpnet_fused) or "fp32"
        # (the eager PyTorch module); net_dtype / fused select the latter two for older callers
        if precision is None:
            precision = "bf16" if net_dtype == torch.bfloat16 and fused else ("fp32" if net_dtype == torch.float32 else "bf16")
        if precision not in ("f16x3", "bf16", "fp32"):
            raise ValueError(f"Segmenter precision {precision!r}")
        self.precision = precision
        net_dtype = torch.bfloat16 if precision == "bf16" else torch.float32
        self.net_dtype = net_dtype
        self.net = build_cpnet(seed=seed, model=model, state_dict_path=weights)
        self.layout = {"bf16": 1, "fp32": 0, "f16x3": 2}[precision]
        self.fnet = None
        if precision == "f16x3":
            # the native kernels hold their own split, packed weights: the module stays on the
            # host (it is never run in this mode)
            self.fnet = FusedCPnetX3(self.net, dev)
        else:
            self.net = self.net.to(td)
            if precision == "bf16" and fused:
                self.fnet = FusedCPnet(self.net, dev)
            self.net = self.net.to(memory_format=torch.channels_last, dtype=net_dtype)
        nt = batch * g.n_tiles
        if self.layout == 2:
            self.tiles = torch.empty((nt, g.by, g.bx, NET_CHANNELS), dtype=torch.float32, device=td)
            self.tiles_nchw = self.tiles
        elif self.layout == 1:
            self.tiles = torch.empty((nt, g.by, g.bx, NET_CHANNELS), dtype=torch.bfloat16, device=td)
            self.tiles_nchw = self.tiles.permute(0, 3, 1, 2)  # channels_last view
        else:
            self.tiles = torch.empty((nt, NET_CHANNELS, g.by, g.bx), dtype=torch.float32, device=td)
            self.tiles_nchw = self.tiles
        self.pct = torch.empty((batch, NET_CHANNELS, 2), dtype=torch.float64, device=td)
        self.taper = torch.from_numpy(taper_mask(g.by, g.bx)).to(td)
        self.yf = torch.empty((batch, 3, g.Ly, g.Lx), dtype=torch.float32, device=td)
        self.stats = torch.zeros(batch * SEG_STATS_BYTES, dtype=torch.uint8, device=td)
        self.net_out = None
        self.graph = None
        self.use_graph = use_graph
        self._lib = dev.lib

    # -- network -----------------------------------------------------------------------------
    def _forward(self):
        if self.layout == 2:
            return self.fnet(self.tiles)
        if self.fnet is not None:
            return self.fnet(self.tiles_nchw)
        with torch.no_grad():
            y = self.net(self.tiles_nchw)
        return y

    def _run_net(self):
        if not self.use_graph:
            self.net_out = self._forward().contiguous(memory_format=torch.channels_last) \
                if self.layout == 1 else self._forward().contiguous()
            return
        if self.graph is not None:
            self.graph.replay()
            return
        if self.graph is None:
            # warm-up / capture on the caller's stream when it is a side stream (a pipeline's
            # own), else on one shared stream per device: each extra stream holds one of the
            # process's few hardware queues (see FovPipeline._copy_streams)
            td = self.dev.torch_device
            s = torch.cuda.current_stream(td)
            if s == torch.cuda.default_stream(td):
                if td.index not in _capture_streams:
                    _capture_streams[td.index] = torch.cuda.Stream(td)
                s = _capture_streams[td.index]
            s.wait_stream(torch.cuda.current_stream(td))
            with torch.cuda.stream(s):
                for _ in range(2):
                    self._forward()
            torch.cuda.current_stream(td).wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, stream=s):
                out = self._forward()
                out = out.contiguous(memory_format=torch.channels_last) if self.layout == 1 else out.contiguous()
            self.net_out = out
        self.graph.replay()

    def cpnet_overflow(self) -> torch.Tensor | None:
        """Device int32 [B * n_tiles]: per network tile, non-zero once a split-fp16 activation of that
        tile left the fp16 range (f16x3); cleared by every forward."""
        return self.fnet.ovf if self.layout == 2 else None

    # -- pipeline ----------------------------------------------------------------------------
    def prepare(self, corr: torch.Tensor):
        """percentiles + tiles (libcpx)."""
        B, C, H, W = corr.shape
        assert B == self.B and H == self.H and W == self.W and C >= NET_CHANNELS
        self.dev._bind_stream()
        lib = self._lib
        check(lib.cpx_seg_percentiles(self.dev.h, _ptr(corr), B, C, H, W, NET_CHANNELS, _ptr(self.pct)),
              "cpx_seg_percentiles")
        check(lib.cpx_seg_tiles(self.dev.h, _ptr(corr), B, C, H, W, NET_CHANNELS, _ptr(self.pct),
                                ct.c_void_p(ct.addressof(self.geom)), self.layout, _ptr(self.tiles)), "cpx_seg_tiles")

    def postprocess(self, labels: torch.Tensor):
        """tile average + dynamics + masks (libcpx)."""
        self.dev._bind_stream()
        lib = self._lib
        out = self.net_out
        check(lib.cpx_seg_average(self.dev.h, ct.c_void_p(out.data_ptr()), self.layout, self.B, 3,
                                  ct.c_void_p(ct.addressof(self.geom)), _ptr(self.taper), _ptr(self.yf)), "cpx_seg_average")
        check(lib.cpx_seg_masks(self.dev.h, _ptr(self.yf), self.B, ct.c_void_p(ct.addressof(self.geom)), self.H, self.W,
                                self.niter, float(self.flow_threshold), self.min_size, self.max_objects,
                                int(self.resample), _ptr(labels), _ptr(self.stats)), "cpx_seg_masks")

    def segment(self, corr: torch.Tensor, labels: torch.Tensor | None = None) -> torch.Tensor:
        """The whole segmentation of a batch (the direct API; FovPipeline runs the stages itself and
        re-runs a FOV whose seeds overflowed).  Waits for the batch and warns when a FOV found more
        seeds than max_objects: its labels are then truncated (SEG_OVF_SEEDS)."""
        if labels is None:
            labels = torch.empty((self.B, self.H, self.W), dtype=torch.int32, device=self.dev.torch_device)
        self.prepare(corr)
        self._run_net()
        self.postprocess(labels)
        ovf = self.seg_stats()["overflow"].ravel()[: self.B]
        bad = np.flatnonzero(ovf & SEG_OVF_SEEDS)
        if bad.size:
            warnings.warn(f"Segmenter.segment: FOV(s) {bad.tolist()} found more seeds than max_objects="
                          f"{self.max_objects}; their labels are truncated (raise max_objects, or run "
                          f"them through FovPipeline, which re-runs such FOVs)", RuntimeWarning, stacklevel=2)
        return labels

    def seg_stats(self) -> np.ndarray:
        return self.stats.cpu().numpy().view(SEG_STATS_DTYPE)
