"""CPU restatement of the whole per-FOV hot path — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

Used by tests and by bench.py's cpu_baseline leg (never by the product).  One FOV:
  flat-field + QC (cpx_oracle: the reference's Illumination_QC_mult arithmetic)
  -> segmentation (CPnet forward in PyTorch on the CPU, fp32, same seeded weights as the GPU run,
     then seg_oracle: tile average, dynamics, masks)
  -> Cells / Cytoplasm (ws_oracle.cells_watershed: the stated marker watershed, heap flood in C;
     cells="expand": cpx_oracle.secondary_objects)
  -> features for Nuclei / Cells / Cytoplasm (cpx_oracle.features, skimage 0.18.3 definitions).
"""
from __future__ import annotations

import time

import numpy as np

import cpx_oracle as orc
import seg_oracle as so


def run_fov(raw: np.ndarray, illum: np.ndarray, net, cell_expand: int = 15, model: str = "nuclei",
            diameter: float = 100.0, timings: dict | None = None, cells: str = "watershed",
            cell_channel: int = 3, flows: np.ndarray | None = None):
    """raw uint16 [C,H,W], illum fp32 [C,H,W]; net = CPU CPnet (torch).  Returns dict of outputs.
    flows: tile-averaged network output [3,H',W'] to use instead of running `net` (the CSV parity
    test feeds the GPU's own flows, so everything after the network is compared bit for bit)."""
    import torch
    t = time.perf_counter()
    C, H, W = raw.shape
    qc = []
    corr = np.empty((C, H, W), np.float32)
    for c in range(C):
        img = orc.illum_correct_qc(raw[c], illum[c])
        qc.append(orc.calculate_qc_metrics(img, str(c)))
        corr[c] = orc.illum_correct_producer(raw[c], illum[c])
    t1 = time.perf_counter()
    if flows is None:
        Ly, Lx = so.net_size(H, W, model, diameter)
        tiles, g = so.make_net_input(corr, Ly, Lx)
        with torch.no_grad():
            y = net(torch.from_numpy(tiles)).numpy()
        yf = so.average_tiles(y, g)
    else:
        yf = flows
    nuclei = so.compute_masks(yf, H, W)
    t2 = time.perf_counter()
    if cells == "watershed":
        import ws_oracle
        cells, cyto = ws_oracle.cells_watershed(nuclei, corr[cell_channel], cell_expand)
    else:
        cells, cyto = orc.secondary_objects(nuclei, cell_expand)
    feats = {"Nuclei": orc.features(nuclei, corr), "Cells": orc.features(cells, corr),
             "Cytoplasm": orc.features(cyto, corr)}
    t3 = time.perf_counter()
    if timings is not None:
        timings.update(illum_qc=t1 - t, segment=t2 - t1, objects_features=t3 - t2, total=t3 - t)
    return dict(qc=qc, nuclei=nuclei, cells=cells, cyto=cyto, feats=feats, corr=corr, flows=yf)
