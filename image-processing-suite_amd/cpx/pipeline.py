"""Per-FOV hot path on one GPU: flat-field + QC -> segmentation -> object tables -> features.

This is the MI355X replacement of the per-FOV work split across the reference's workers:
  Illumination_QC_mult.process_site        (Illumination_QC_mult.py:131-162)  -> stage A
  Cellpose_GPU_s3fs producer/consumer      (Cellpose_GPU_s3fs.py:47-232)      -> stages A, B, C
  CellProfiler measurement step            (Feature_extraction_opt.py:164-167) -> stage D
for a batch of B FOVs that are already resident in HBM (uint16 planes [B*C, H, W]):
  A  libcpx cpx_illum_correct (fp32 corrected planes + PercentMaximal) + cpx_qc_rps (slope)
  B  Segmenter (libcpx normalise/tiles -> CPnet bf16 -> libcpx tile average/dynamics/masks)
  C  libcpx cpx_expand_labels (Cells, Cytoplasm) + cpx_objects for Nuclei / Cells / Cytoplasm
  D  libcpx cpx_features for the three object sets (+ optional a7 crops)
Everything is enqueued on one HIP stream; `fetch()` is the only synchronisation.
"""
from __future__ import annotations

import dataclasses

import numpy as np
import torch

from . import _lib
from .device import Device, as_numpy, n_features
from .segment import CELLPOSE_MODEL, DIAMETER, Segmenter

OBJECT_SETS = ("Nuclei", "Cells", "Cytoplasm")


@dataclasses.dataclass
class PipelineConfig:
    H: int = 2080
    W: int = 2080
    C: int = 5
    batch: int = 8
    channels: tuple = ("DNA", "ER", "RNA", "AGP", "Mito")
    model: str = CELLPOSE_MODEL
    diameter: float = DIAMETER
    cell_expand: int = 15            # Cells = expand_labels(Nuclei, cell_expand)
    max_objects: int = 2048          # per FOV and object set
    box: int = 200                   # Cellpose_GPU_s3fs.py:30 BOX_SIZE
    weights: str | None = None       # local CPnet state_dict; None = seeded random init
    seed: int = 0
    use_graph: bool = True
    crops: bool = False              # a7 crops for the embedding consumer (off in the bench)


@dataclasses.dataclass
class FovResults:
    qc: np.ndarray                   # structured [B*C] (slope, pct_max, ...)
    hdr: dict                        # set -> structured [B] (n_objects, n_kept, ...)
    objects: dict                    # set -> list of structured arrays (per FOV)
    feats: dict                      # set -> list of float64 [n_objects, F]
    seg_stats: np.ndarray


class FovPipeline:
    def __init__(self, dev: Device, cfg: PipelineConfig, illum: np.ndarray | None):
        self.dev, self.cfg = dev, cfg
        B, C, H, W = cfg.batch, cfg.C, cfg.H, cfg.W
        td = dev.torch_device
        self.raw = torch.empty((B * C, H, W), dtype=torch.int16, device=td)  # uint16 bits
        self.illum = None if illum is None else torch.from_numpy(np.ascontiguousarray(illum)).to(td)
        self.corr = torch.empty((B, C, H, W), dtype=torch.float32, device=td)
        self.stats = dev.empty_bytes(64 * B * C)
        self.qc = dev.empty_bytes(24 * B * C)
        ML = cfg.max_objects
        self.labels = {s: torch.empty((B, H, W), dtype=torch.int32, device=td) for s in OBJECT_SETS}
        self.lstats = dev.empty_bytes(64 * B * (ML + 1))
        self.objects = {s: dev.empty_bytes(56 * B * ML) for s in OBJECT_SETS}
        self.hdr = {s: dev.empty_bytes(16 * B) for s in OBJECT_SETS}
        self.F = n_features(C)
        self.feats = {s: torch.zeros((B, ML, self.F), dtype=torch.float64, device=td) for s in OBJECT_SETS}
        self.seg = Segmenter(dev, H, W, B, model=cfg.model, diameter=cfg.diameter, weights=cfg.weights,
                             seed=cfg.seed, use_graph=cfg.use_graph, max_objects=ML)
        self.crops = None
        if cfg.crops:
            self.crops = torch.zeros((B, ML, cfg.box, cfg.box, C), dtype=torch.float32, device=td)
            self.crops8 = torch.zeros((B, ML, C, cfg.box, cfg.box), dtype=torch.uint8, device=td)
        dev.reserve(B * C, H, W, B, ML)

    # ---- stages ---------------------------------------------------------------------------
    def stage_illum_qc(self):
        C = self.cfg.C
        self.dev.illum_correct(self.raw, self.illum, C, self.corr, self.stats)
        self.dev.qc_rps(self.raw, self.illum, C, self.stats, self.qc)

    def stage_segment(self):
        self.seg.segment(self.corr, self.labels["Nuclei"])

    def stage_objects(self):
        from ._lib import check
        from .device import _ptr
        cfg = self.cfg
        B, H, W = cfg.batch, cfg.H, cfg.W
        check(self.dev.lib.cpx_expand_labels(self.dev.h, _ptr(self.labels["Nuclei"]), B, H, W,
                                             cfg.cell_expand, _ptr(self.labels["Cells"]),
                                             _ptr(self.labels["Cytoplasm"])), "cpx_expand_labels")
        for s in OBJECT_SETS:
            self.dev.objects(self.labels[s], cfg.max_objects, cfg.box, self.lstats, self.objects[s], self.hdr[s])
            self.dev.features(self.labels[s], self.corr, cfg.C, cfg.max_objects, self.objects[s],
                              self.hdr[s], self.feats[s])
        if self.crops is not None:
            self.dev.objects(self.labels["Nuclei"], cfg.max_objects, cfg.box, self.lstats,
                             self.objects["Nuclei"], self.hdr["Nuclei"])
            self.dev.crops(self.labels["Nuclei"], self.corr, cfg.C, cfg.max_objects, self.objects["Nuclei"],
                           self.hdr["Nuclei"], cfg.box, cfg.max_objects, self.crops, self.crops8)

    def run(self, raw: torch.Tensor | None = None):
        """Enqueue the whole hot path for a batch of uint16 planes [B*C, H, W] already in HBM
        (default: self.raw, filled by the host loader)."""
        if raw is not None:
            assert raw.shape == self.raw.shape and raw.dtype == torch.int16 and raw.is_contiguous()
            self.raw = raw
        self.stage_illum_qc()
        self.stage_segment()
        self.stage_objects()

    def fetch(self) -> FovResults:
        """Synchronise and copy the per-FOV results to the host (only the valid object rows)."""
        B = self.cfg.batch
        hdrs = {s: as_numpy(self.hdr[s], "hdr") for s in OBJECT_SETS}  # syncs
        qc = as_numpy(self.qc, "qc")
        objs, feats = {}, {}
        for s in OBJECT_SETS:
            n = hdrs[s]["n_objects"].astype(int)
            nmax = int(n.max()) if B else 0
            f = self.feats[s][:, :max(nmax, 1)].cpu().numpy()
            o = as_numpy(self.objects[s], "object").reshape(B, self.cfg.max_objects)[:, :max(nmax, 1)]
            feats[s] = [f[b, : n[b]] for b in range(B)]
            objs[s] = [o[b, : n[b]] for b in range(B)]
        return FovResults(qc=qc, hdr=hdrs, objects=objs, feats=feats, seg_stats=self.seg.seg_stats())
