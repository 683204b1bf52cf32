"""Per-FOV hot path on one GPU: flat-field + QC -> segmentation -> object tables -> features.

This is the MI355X replacement of the per-FOV work split across the reference's workers:
  Illumination_QC_mult.process_site        (Illumination_QC_mult.py:131-162)  -> stage A
  Cellpose_GPU_s3fs producer/consumer      (Cellpose_GPU_s3fs.py:47-232)      -> stages A, B, C
  CellProfiler measurement step            (Feature_extraction_opt.py:164-167) -> stage D
for a batch of B FOVs that are already resident in HBM (uint16 planes [B*C, H, W]):
  A  libcpx cpx_illum_correct (fp32 corrected planes + PercentMaximal) + cpx_qc_rps (slope)
  B  Segmenter (libcpx normalise/tiles -> CPnet bf16 -> libcpx tile average/dynamics/masks)
  C  libcpx cpx_watershed_cells (Cells by marker watershed from the Nuclei, Cytoplasm; or
     cpx_expand_labels with cells="expand") + cpx_objects for Nuclei / Cells / Cytoplasm
  D  libcpx cpx_features for the three object sets (+ optional a7 crops)
Everything is enqueued on one HIP stream.  Results (QC, object tables, features) live in
`slots` alternating buffer sets: `run()` writes slot i % slots and records an event, and
`fetch(slot)` copies that slot to pinned host memory on a separate copy stream after waiting
for the event only — so the host can fetch step i while the GPU already runs step i + 1.
"""
from __future__ import annotations

import dataclasses
import logging
import os

import numpy as np
import torch

from . import _lib
from .device import Device, as_numpy, n_features
from .segment import CELLPOSE_MODEL, DIAMETER, Segmenter

OBJECT_SETS = ("Nuclei", "Cells", "Cytoplasm")
# stages that never overlap themselves across the batches in flight on one GPU (FovPipeline._stage):
# the CPnet and the feature stage, each contending with its own copy for HBM / MFMA and LDS,
# overlap better with the other batch's different stages — 439.5 -> 446.4 FOV/s (three interleaved
# pairs of 60-step benches, `gpurun_out/r05t`); tests/test_gpu_streams.py runs both settings
STAGE_EXCLUSIVE = ("cpnet", "features")
# Cells + Cytoplasm features in one libcpx call (tests/test_gpu_features_pair.py checks it against
# one call per set, bit for bit)
PAIR_FEATURES = True
log = logging.getLogger("cpx.pipeline")


@dataclasses.dataclass
class PipelineConfig:
    H: int = 2080
    W: int = 2080
    C: int = 5
    batch: int = 8
    channels: tuple = ("DNA", "ER", "RNA", "AGP", "Mito")
    model: str = CELLPOSE_MODEL
    diameter: float = DIAMETER
    resample: bool = True            # CellposeModel.eval default: dynamics at full resolution
    cpnet_precision: str = "f16x3"   # "f16x3": native split-fp16 MFMA kernels at the fp32
                                     # network's accuracy (the reference's precision: masks and
                                     # IDs identical to the fp32 CPU network);
                                     # "bf16": native bf16 MFMA kernels (faster, boundary pixels
                                     # and IDs differ); "fp32": the eager PyTorch module
    cells: str = "watershed"         # "watershed": marker watershed of the inverted cell channel
                                     # inside the expand_labels(Nuclei, cell_expand) footprint
                                     # (DESIGN.md §7); "expand": Cells = that footprint's labels
    cell_expand: int = 15            # footprint distance (px)
    cell_channel: int | None = None  # watershed elevation channel; None: "AGP" when present
                                     # among the first C channel names, else the last channel
    ws_rounds: tuple = (24, 16)      # watershed relax tile rounds / label pointer-jump rounds
                                     # enqueued per batch (bench plates: <= 9 / ~8; idle ~6 us)
    max_objects: int = 2048          # per FOV and object set
    box: int = 200                   # Cellpose_GPU_s3fs.py:30 BOX_SIZE
    weights: str | None = None       # local CPnet state_dict; None = seeded random init
    seed: int = 0
    use_graph: bool = True
    crops: bool = False              # a7 crops for the embedding consumer (off in the bench)
    crops_f32: bool = True           # also keep the float crops (the embedder needs only crops8)
    slots: int = 2                   # result buffer sets (fetch of step i overlaps step i + 1)

    def ws_channel(self) -> int:
        """The watershed elevation channel (cell_channel, or "AGP" / the last channel)."""
        if self.cell_channel is not None:
            return self.cell_channel
        names = list(self.channels)[: self.C]
        return names.index("AGP") if "AGP" in names else self.C - 1


@dataclasses.dataclass
class FovResults:
    qc: np.ndarray                   # structured [B*C] (slope, pct_max, ...)
    hdr: dict                        # set -> structured [B] (n_objects, n_kept, ...)
    objects: dict                    # set -> list of structured arrays (per FOV)
    feats: dict                      # set -> list of float64 [n_objects, F]
    seg_stats: np.ndarray
    failed: np.ndarray | None = None  # [B] bool: the FOV's Cells watershed did not converge even
                                      # after the re-runs with more rounds; its object tables are
                                      # emptied (the reference's per-site 'empty' result,
                                      # Cellpose_GPU_s3fs.py:225-232)
    recovered: np.ndarray | None = None  # [B] int: 0, or how the FOV was re-run on its own
                                         # (RECOVER_FP32: a split-fp16 activation overflowed, so its
                                         # CPnet ran in fp32; RECOVER_WS: its watershed needed more
                                         # rounds; RECOVER_CAPACITY: it has more seeds / objects
                                         # than max_objects, so it ran with larger tables; bits
                                         # combine; RECOVER_FILL_SEQ: not a re-run — a mask lay
                                         # partly inside an earlier mask's holes, so libcpx ran
                                         # Cellpose's sequential fill loop for this FOV)
    crops8: dict | None = None           # FOV -> device uint8 [1][ML'][C][box][box]: the a7 crops
                                         # of a re-run FOV (cfg.crops), replacing its batch slot


RECOVER_FP32 = 1
RECOVER_WS = 2
RECOVER_CAPACITY = 4
RECOVER_FILL_SEQ = 8
WS_RETRIES = 4   # at most this many re-runs of a FOV whose watershed did not converge, with 2x,
                 # 4x, 8x, 16x the configured rounds
REC_CACHE = 4    # single-FOV recovery pipelines kept per process (shared by every pipeline)


def _sync_after(stream):
    """Wait for the work enqueued on `stream` so far (not for what other threads of the host
    loop enqueue on it later, e.g. the next batch's upload)."""
    ev = torch.cuda.Event()
    ev.record(stream)
    ev.synchronize()


class FovPipeline:
    _copy_streams: dict = {}
    _upload_streams: dict = {}
    _rec_cache: dict = {}  # (device, precision, max_objects, crops, config) -> single-FOV pipeline

    def __init__(self, dev: Device, cfg: PipelineConfig, illum, recovery: bool = True):
        self.dev, self.cfg = dev, cfg
        B, C, H, W = cfg.batch, cfg.C, cfg.H, cfg.W
        td = dev.torch_device
        # the host loader's staging planes (uint16 bits): one buffer per result slot, so a step's
        # planes stay intact until its fetch() (which may re-run single FOVs from them); self.raw
        # is always the buffer the next run() reads
        self._raw_bufs = [torch.empty((B * C, H, W), dtype=torch.int16, device=td)]
        self.raw = self._raw_bufs[0]
        if illum is None or isinstance(illum, torch.Tensor):
            self.illum = None if illum is None else illum.to(td)
        else:
            self.illum = torch.from_numpy(np.ascontiguousarray(illum)).to(td)
        self._recovery = recovery  # False for the single-FOV pipelines that do the re-runs
        self.ws_rounds = tuple(cfg.ws_rounds)  # per run (a recovery re-run raises them)
        self.corr = torch.empty((B, C, H, W), dtype=torch.float32, device=td)
        self.stats = dev.empty_bytes(64 * B * C)
        ML = cfg.max_objects
        self.labels = {s: torch.empty((B, H, W), dtype=torch.int32, device=td) for s in OBJECT_SETS}
        self.lstats = dev.empty_bytes(64 * B * (ML + 1))
        self.F = n_features(C)
        self.seg = Segmenter(dev, H, W, B, model=cfg.model, diameter=cfg.diameter, weights=cfg.weights,
                             seed=cfg.seed, use_graph=cfg.use_graph and cfg.cpnet_precision != "fp32",
                             max_objects=ML, resample=cfg.resample, precision=cfg.cpnet_precision)
        # result slots (device) and their pinned host mirrors
        self._slots = []
        for _ in range(max(1, cfg.slots)):
            self._slots.append({
                "qc": dev.empty_bytes(24 * B * C),
                "hdr": {s: dev.empty_bytes(16 * B) for s in OBJECT_SETS},
                "objects": {s: dev.empty_bytes(56 * B * ML) for s in OBJECT_SETS},
                "feats": {s: torch.zeros((B, ML, self.F), dtype=torch.float64, device=td) for s in OBJECT_SETS},
                "seg_stats": torch.empty_like(self.seg.stats),
                "cpnet_ovf": torch.zeros(max(1, B * self.seg.geom.n_tiles), dtype=torch.int32, device=td),
                "raw": None, "event": None})
        self._host = {
            "qc": torch.empty(24 * B * C, dtype=torch.uint8, pin_memory=True),
            "hdr": {s: torch.empty(16 * B, dtype=torch.uint8, pin_memory=True) for s in OBJECT_SETS},
            "objects": {s: torch.empty(56 * B * ML, dtype=torch.uint8, pin_memory=True) for s in OBJECT_SETS},
            "feats": {s: torch.empty(B * ML * self.F, dtype=torch.float64, pin_memory=True) for s in OBJECT_SETS},
            "seg_stats": torch.empty(self.seg.stats.shape, dtype=self.seg.stats.dtype, pin_memory=True),
            "cpnet_ovf": torch.zeros(max(1, B * self.seg.geom.n_tiles), dtype=torch.int32, pin_memory=True)}
        # one result-copy stream per device, shared by its pipelines: a process has only
        # GPU_MAX_HW_QUEUES (4) hardware queues, and streams beyond that share one, which
        # serialises two pipelines' kernels behind each other
        key = torch.device(td).index
        if key not in FovPipeline._copy_streams:
            FovPipeline._copy_streams[key] = torch.cuda.Stream(device=td)
        self._copy_stream = FovPipeline._copy_streams[key]
        self._step = 0
        self._use_slot(0)
        self.crops = None
        if cfg.crops:
            self.crops = (torch.zeros((B, ML, cfg.box, cfg.box, C), dtype=torch.float32, device=td)
                          if cfg.crops_f32 else None)
            self.crops8 = torch.zeros((B, ML, C, cfg.box, cfg.box), dtype=torch.uint8, device=td)
        dev.reserve(B * C, H, W, B, ML)

    @staticmethod
    def upload_stream(device: torch.device) -> torch.cuda.Stream:
        """One host-to-device upload stream per device (cpx.plate's staging uploads), so a result
        fetch never queues behind an upload.  With the two pipeline streams, the result-copy
        stream and the default stream the plate process holds five streams: cpx.plate raises
        GPU_MAX_HW_QUEUES to 8 so that no two of them share a hardware queue."""
        key = torch.device(device).index
        if key not in FovPipeline._upload_streams:
            FovPipeline._upload_streams[key] = torch.cuda.Stream(device=device)
        return FovPipeline._upload_streams[key]

    def _use_slot(self, k: int):
        sl = self._slots[k]
        self.cur = k
        self.qc, self.hdr, self.objects, self.feats = sl["qc"], sl["hdr"], sl["objects"], sl["feats"]

    # ---- stages ---------------------------------------------------------------------------
    # A stage in STAGE_EXCLUSIVE (of illum_qc, cpnet, seg_post, cells, features) of one pipeline
    # waits on the device for the same stage of the pipeline enqueued before it (one shared event
    # per device and stage), so two batches in flight never run that stage at once and overlap
    # only across different stages
    _excl: dict = {}

    def _stage(self, name, fn):
        if name not in STAGE_EXCLUSIVE:
            return fn()
        key = (self.dev.index, name)
        stream = torch.cuda.current_stream(self.dev.torch_device)
        ev = FovPipeline._excl.get(key)
        if ev is not None:
            stream.wait_event(ev)
        out = fn()
        ev = torch.cuda.Event()
        ev.record(stream)
        FovPipeline._excl[key] = ev
        return out

    def stage_illum_qc(self):
        C = self.cfg.C

        def run():
            self.dev.illum_correct(self.raw, self.illum, C, self.corr, self.stats)
            self.dev.qc_rps(self.raw, self.illum, C, self.stats, self.qc)
        self._stage("illum_qc", run)

    def stage_segment(self):
        self.seg.prepare(self.corr)
        self._stage("cpnet", self.seg._run_net)
        self._stage("seg_post", lambda: self.seg.postprocess(self.labels["Nuclei"]))

    def stage_objects(self):
        self._stage("cells", self.stage_cells)
        self._stage("features", self.stage_features)

    def stage_cells(self):
        """Cells (marker watershed or expand_labels) and Cytoplasm from the Nuclei labels."""
        from ._lib import check
        from .device import _ptr
        cfg = self.cfg
        B, H, W = cfg.batch, cfg.H, cfg.W
        if cfg.cells == "watershed":
            ch = cfg.ws_channel()
            st = self.seg.stats  # cpx_seg_stats [B] (48 bytes): cells_status is int32 field 6 of 12
            check(self.dev.lib.cpx_watershed_cells(
                self.dev.h, _ptr(self.labels["Nuclei"]), _ptr(self.corr), B, cfg.C, ch,
                H, W, cfg.cell_expand, self.ws_rounds[0], self.ws_rounds[1], _ptr(self.labels["Cells"]),
                _ptr(self.labels["Cytoplasm"]), st.data_ptr() + 6 * 4, 12),
                "cpx_watershed_cells")
        elif cfg.cells == "expand":
            check(self.dev.lib.cpx_expand_labels(self.dev.h, _ptr(self.labels["Nuclei"]), B, H, W,
                                                 cfg.cell_expand, _ptr(self.labels["Cells"]),
                                                 _ptr(self.labels["Cytoplasm"])), "cpx_expand_labels")
        else:
            raise ValueError(f"PipelineConfig.cells: {cfg.cells!r}")

    def stage_features(self):
        """Object tables and shape / intensity / texture features of the three object sets (Cells
        and Cytoplasm measured together: cpx_features_pair stages a Cytoplasm object from its
        cell's reads of the channels when the two share the bbox)."""
        cfg = self.cfg
        for s in OBJECT_SETS:
            self.dev.objects(self.labels[s], cfg.max_objects, cfg.box, self.lstats, self.objects[s], self.hdr[s])
        self.dev.features(self.labels["Nuclei"], self.corr, cfg.C, cfg.max_objects, self.objects["Nuclei"],
                          self.hdr["Nuclei"], self.feats["Nuclei"])
        if PAIR_FEATURES:
            self.dev.features_pair(self.labels["Cells"], self.labels["Cytoplasm"], self.corr, cfg.C, cfg.max_objects,
                                   (self.objects["Cells"], self.hdr["Cells"], self.feats["Cells"]),
                                   (self.objects["Cytoplasm"], self.hdr["Cytoplasm"], self.feats["Cytoplasm"]))
        else:
            for s in ("Cells", "Cytoplasm"):
                self.dev.features(self.labels[s], self.corr, cfg.C, cfg.max_objects, self.objects[s],
                                  self.hdr[s], self.feats[s])
        if self.cfg.crops:
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
        k = self._step % len(self._slots)
        self._step += 1
        sl = self._slots[k]
        stream = torch.cuda.current_stream(self.dev.torch_device)
        # (a slot's previous fetch() returned only after its copies completed)
        self._use_slot(k)
        sl["raw"] = self.raw
        self.stage_illum_qc()
        self.stage_segment()
        self.stage_objects()
        sl["seg_stats"].copy_(self.seg.stats)
        ovf = self.seg.cpnet_overflow()
        if ovf is not None:
            sl["cpnet_ovf"].copy_(ovf)
        sl["event"] = torch.cuda.Event()
        sl["event"].record(stream)
        if raw is None:  # the loader fills the next slot's own staging buffer
            nk = self._step % len(self._slots)
            while len(self._raw_bufs) <= nk:
                self._raw_bufs.append(torch.empty_like(self._raw_bufs[0]))
            self.raw = self._raw_bufs[nk]
        return k

    def fetch(self, slot: int | None = None) -> FovResults:
        """Copy one slot's results to the host (default: the last run) and return them.  Waits
        only for that slot's step (its recorded event), with the copies on the device's copy stream, so a
        step enqueued after it keeps the GPU busy meanwhile."""
        from .segment import SEG_ERR_INTERNAL, SEG_OVF_FILL_PARTIAL, SEG_OVF_SEEDS, SEG_STATS_DTYPE
        k = self.cur if slot is None else slot
        sl, hb = self._slots[k], self._host
        B, ML, F = self.cfg.batch, self.cfg.max_objects, self.F
        cs = self._copy_stream
        cs.wait_event(sl["event"])
        with torch.cuda.stream(cs):
            hb["qc"].copy_(sl["qc"], non_blocking=True)
            hb["seg_stats"].copy_(sl["seg_stats"], non_blocking=True)
            hb["cpnet_ovf"].copy_(sl["cpnet_ovf"], non_blocking=True)
            for s in OBJECT_SETS:
                hb["hdr"][s].copy_(sl["hdr"][s], non_blocking=True)
        _sync_after(cs)
        hdrs = {s: as_numpy(hb["hdr"][s], "hdr").copy() for s in OBJECT_SETS}
        qc = as_numpy(hb["qc"], "qc").copy()
        seg_stats = hb["seg_stats"].numpy().view(SEG_STATS_DTYPE).copy()
        sovf = seg_stats["overflow"].ravel()[:B]
        if (sovf & SEG_ERR_INTERNAL).any():
            raise RuntimeError("cpx_seg_masks: a flow-error work loop reached its claim bound "
                               "(CPX_SEG_ERR_INTERNAL): the batch's masks are invalid")
        # only each FOV's own rows cross PCIe: the rows are gathered on the device into one
        # contiguous block per table (one D2H each) instead of copying [:, :max n] of every FOV
        # (~30 % padding rows: each FOV has its own object count)
        n_bs = {s: np.minimum(hdrs[s]["n_objects"].astype(np.int64), ML) for s in OBJECT_SETS}
        keep = []  # device index tensors and their pinned sources, alive until the copies end
        with torch.cuda.stream(cs):
            for s in OBJECT_SETS:
                n_b = n_bs[s]
                tot = int(n_b.sum())
                if tot == 0:
                    continue
                rows = np.concatenate([b * ML + np.arange(n_b[b], dtype=np.int64) for b in range(B)])
                src = torch.from_numpy(rows).pin_memory()
                idx = src.to(self.dev.torch_device, non_blocking=True)
                fg = sl["feats"][s].view(B * ML, F).index_select(0, idx)
                og = sl["objects"][s].view(B * ML, 56).index_select(0, idx)
                hb["feats"][s][:tot * F].view(tot, F).copy_(fg, non_blocking=True)
                hb["objects"][s][:tot * 56].view(tot, 56).copy_(og, non_blocking=True)
                keep.append((src, idx, fg, og))
        _sync_after(cs)
        del keep
        objs, feats = {}, {}
        for s in OBJECT_SETS:
            n_b = n_bs[s]
            tot = int(n_b.sum())
            off = np.concatenate([[0], np.cumsum(n_b)])
            f = hb["feats"][s][:tot * F].view(tot, F).numpy()
            o = as_numpy(hb["objects"][s][:max(tot, 1) * 56], "object")[:tot]
            feats[s] = [f[off[b]:off[b + 1]].copy() for b in range(B)]
            objs[s] = [o[off[b]:off[b + 1]].copy() for b in range(B)]
        nt = self.seg.geom.n_tiles
        ovf = hb["cpnet_ovf"][:B * nt].numpy().reshape(B, nt).any(axis=1)
        failed = np.zeros(B, dtype=bool)
        if self.cfg.cells == "watershed":
            failed = seg_stats["cells_status"].ravel()[:B] < 0
        # capacity: a FOV with more seeds than max_objects (its masks were truncated), or a label
        # table that dropped labels above max_objects, needs larger tables (reference: no limit,
        # Cellpose_GPU_s3fs.py:143-170); masks <= seeds, so n_seeds_found tables are enough
        need = np.where(sovf & SEG_OVF_SEEDS, seg_stats["n_seeds_found"].ravel()[:B], 0)
        for s in OBJECT_SETS:
            need = np.maximum(need, np.where(hdrs[s]["overflow"] != 0, hdrs[s]["max_label"], 0))
        # a FOV with a partly absorbed mask already took the sequential fill on the GPU
        # (k_fill_seq, cpx.h CPX_SEG_OVF_FILL_PARTIAL): its labels are the reference loop's
        recovered = np.where(sovf & SEG_OVF_FILL_PARTIAL, RECOVER_FILL_SEQ, 0).astype(np.int32)
        res = FovResults(qc=qc, hdr=hdrs, objects=objs, feats=feats, seg_stats=seg_stats, failed=failed,
                         recovered=recovered)
        if self._recovery and (ovf.any() or failed.any() or (need > ML).any()):
            self._recover(sl["raw"], res, ovf, failed, need)
        elif (need > ML).any():
            raise RuntimeError(f"FOV(s) {np.nonzero(need > ML)[0].tolist()} need {int(need.max())} object "
                               f"slots, max_objects is {ML} (recovery disabled)")
        if res.failed.any():
            # per-site failure, not a failed batch: those FOVs get no object rows, every other
            # FOV of the batch is kept (the reference logs a site's error and moves on)
            log.error("cpx_watershed_cells: no convergence within %s rounds for FOV(s) %s of the batch; "
                      "recorded as empty sites", self.cfg.ws_rounds, np.nonzero(res.failed)[0].tolist())
            for s in OBJECT_SETS:
                for b in np.nonzero(res.failed)[0]:
                    res.objects[s][b] = res.objects[s][b][:0]
                    res.feats[s][b] = res.feats[s][b][:0]
                    res.hdr[s][b]["n_objects"] = 0
                    res.hdr[s][b]["n_kept"] = 0
        return res

    # ---- per-FOV recovery (Cellpose_GPU_s3fs.py:142-147: a site that fails is retried, not
    # dropped) ----------------------------------------------------------------------------------
    def _recovery_pipe(self, precision: str, max_objects: int) -> "FovPipeline":
        """A single-FOV pipeline for re-runs, shared by every pipeline of the process (one per
        (device, precision, max_objects, ...), at most REC_CACHE kept: the oldest is dropped)."""
        cfg = dataclasses.replace(self.cfg, batch=1, cpnet_precision=precision, max_objects=max_objects,
                                  slots=1, crops_f32=False)
        key = (self.dev.index, repr(cfg))
        cache = FovPipeline._rec_cache
        if key in cache:
            cache[key] = cache.pop(key)  # most recently used last
        else:
            while len(cache) >= REC_CACHE:
                cache.pop(next(iter(cache)))
            cache[key] = FovPipeline(Device(self.dev.index), cfg, self.illum, recovery=False)
        return cache[key]

    def _recover(self, raw: torch.Tensor, res: FovResults, ovf: np.ndarray, failed: np.ndarray,
                 need: np.ndarray):
        """Re-run single FOVs of a fetched step from its planes (`raw`, kept per slot) and splice
        their results into `res`: a FOV whose split-fp16 CPnet overflowed runs its CPnet in fp32
        (the reference's own arithmetic; the split format holds |a| < 65504 only); a FOV with more
        seeds or labels than max_objects runs with tables of the next power of two that holds
        them; a FOV whose Cells watershed did not converge runs again with twice the rounds, at
        most WS_RETRIES times.  The re-runs are synchronous on the device's copy stream (after the
        step's event): the host thread that called fetch() waits for them (about one single-FOV
        pipeline each), and so do result copies of the other pipelines queued behind them; the
        other pipelines' kernels keep running on their own streams."""
        C, ML = self.cfg.C, self.cfg.max_objects
        with torch.cuda.stream(self._copy_stream):
            for b in np.nonzero(ovf | failed | (need > ML))[0]:
                precision = "fp32" if ovf[b] else self.cfg.cpnet_precision
                flag = RECOVER_FP32 if ovf[b] else 0
                ml = ML
                if need[b] > ML:
                    ml = max(2 * ML, 1 << int(need[b] - 1).bit_length())
                    flag |= RECOVER_CAPACITY
                # a FOV re-run only for its watershed starts at twice the rounds; every re-run
                # that still does not converge doubles them again, up to 2^WS_RETRIES x
                rounds, doublings = tuple(self.cfg.ws_rounds), 0
                if failed[b] and flag == 0:
                    rounds, flag, doublings = (2 * rounds[0], 2 * rounds[1]), RECOVER_WS, 1
                while True:
                    rp = self._recovery_pipe(precision, ml)
                    rp.ws_rounds = rounds
                    rp.illum = self.illum  # the cached pipeline may have been built for another flat-field
                    rp.raw.copy_(raw[b * C:(b + 1) * C])
                    r1 = rp.fetch(rp.run())
                    if not r1.failed[0] or doublings >= WS_RETRIES:
                        break
                    rounds, flag, doublings = (2 * rounds[0], 2 * rounds[1]), flag | RECOVER_WS, doublings + 1
                log.warning("FOV %d of the batch re-run on its own (%s; watershed rounds %s): %s", b,
                            ", ".join(w for f, w in ((RECOVER_FP32, "CPnet fp32 after a split-fp16 overflow"),
                                                     (RECOVER_CAPACITY, f"max_objects {ml}"),
                                                     (RECOVER_WS, "more watershed rounds")) if flag & f) or "rerun",
                            rounds, "converged" if not r1.failed[0] else "watershed still not converged")
                for s in OBJECT_SETS:
                    res.hdr[s][b] = r1.hdr[s][0]
                    res.objects[s][b] = r1.objects[s][0]
                    res.feats[s][b] = r1.feats[s][0]
                res.seg_stats[b] = r1.seg_stats[0]
                res.failed[b] = bool(r1.failed[0])
                res.recovered[b] = flag | (RECOVER_FILL_SEQ if r1.recovered[0] & RECOVER_FILL_SEQ else 0)
                if self.cfg.crops:
                    if res.crops8 is None:
                        res.crops8 = {}
                    res.crops8[int(b)] = rp.crops8.clone()
