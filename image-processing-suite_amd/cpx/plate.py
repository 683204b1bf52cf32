"""Plate/time measurement run on one GPU: LoadData CSV + TIFF planes -> the four CSV tables.

Replaces the CellProfiler job that Feature_extraction_opt.py:159-177 launches per (plate, time)
(LoadData CSV in, per-object tables synced to `<base>/<plate>/<time>/`), with the GPU pipeline
of cpx.pipeline: flat-field + QC -> Cellpose-restated segmentation -> Cells/Cytoplasm -> object
tables -> features, in batches of FOVs resident in HBM.  Host threads decode the next batch's
TIFFs while the GPU works on the current one.

  python -m cpx.plate --load-data load_data_P01_24_illum.csv --data-path IMAGES \\
      --illum-path ILLUM --channels DNA ER RNA AGP Mito --out RESULTS [--batch 8]

Channel files come from FileName_<ch> (relative to --data-path); flat-fields from
<ch>_illum.npy or Illum<ch>.npy (as the QC tool); plate and time from Metadata_Plate /
Metadata_Timepoint unless given.  Multi-GPU: run one process per GPU on a well shard
(cpx.shard.shard) and concatenate the tables (rows are keyed by ImageNumber).
"""
from __future__ import annotations

import argparse
import concurrent.futures
import logging
import os

import numpy as np

log = logging.getLogger("cpx.plate")


def parse_args(argv=None):
    ap = argparse.ArgumentParser(prog="python -m cpx.plate", description="GPU per-object measurement of one plate/time")
    ap.add_argument("--load-data", required=True)
    ap.add_argument("--data-path", required=True)
    ap.add_argument("--illum-path", default=None)
    ap.add_argument("--channels", nargs="+", required=True)
    ap.add_argument("--out", required=True, help="base folder; tables go to <out>/<plate>/<time>/")
    ap.add_argument("--plate", default=None)
    ap.add_argument("--time", default=None)
    ap.add_argument("--batch", type=int, default=8, help="FOVs per GPU batch")
    ap.add_argument("--threads", type=int, default=16, help="TIFF decode threads")
    ap.add_argument("--weights", default=None, help="CPnet state_dict (default: packaged synthetic-trained weights)")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--pipes", type=int, default=2,
                    help="pipelines (libcpx context + HIP stream) on the GPU: batches in flight")
    ap.add_argument("--csv-image-key", default=None,
                    help="folder with an Image.csv whose ImageQC_* flags exclude FOVs (Cellpose_GPU_s3fs.py:252-255)")
    return ap.parse_args(argv)


def qc_filter(load_data, image_df):
    """Cellpose_GPU_s3fs.py:252-255: keep the LoadData rows whose ImageQC_* flags sum below 1
    (boolean indexing aligned on the row index, as the reference)."""
    not_failing = image_df.filter(like="ImageQC_").sum(axis=1) < 1
    return load_data[not_failing].copy()


def _illum(illum_path, channels, H, W):
    from .qc import load_illum
    found = load_illum(illum_path, channels)
    if all(a is None for a in found):
        return None
    planes = []
    for ch, a in zip(channels, found):
        if a is None or a.shape != (H, W):
            if a is not None:
                log.warning("flat-field for %s has shape %s, planes are %s: not applied", ch, a.shape, (H, W))
            planes.append(np.ones((H, W), np.float32))
        else:
            planes.append(a.astype(np.float32))
    return np.stack(planes)


def run(argv=None):
    import pandas as pd
    import torch
    from . import tiffio
    from .csvout import PlateTables
    from .device import Device
    from .pipeline import OBJECT_SETS, FovPipeline, PipelineConfig

    a = parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s: %(message)s")
    table = pd.read_csv(a.load_data)
    if a.csv_image_key:
        n0 = len(table)
        table = qc_filter(table, pd.read_csv(os.path.join(a.csv_image_key, "Image.csv")))
        log.info("image QC filter: %d of %d sites kept", len(table), n0)
    else:
        log.info("No csv_image_key provided — skipping image QC filtering.")
    chans = list(a.channels)
    C = len(chans)
    plate = a.plate or (str(table["Metadata_Plate"].iloc[0]) if "Metadata_Plate" in table else "plate")
    time = a.time or (str(table["Metadata_Timepoint"].iloc[0]) if "Metadata_Timepoint" in table else "0")
    files = [[os.path.join(a.data_path, str(r[f"FileName_{ch}"])) for ch in chans] for _, r in table.iterrows()]
    first = tiffio.imread(files[0][0])
    H, W = first.shape
    weights = a.weights
    if weights is None:
        cand = os.path.join(os.path.dirname(__file__), "weights", "cpnet_nuclei_synth.pt")
        weights = cand if os.path.exists(cand) else None
    B = max(1, min(a.batch, len(files)))
    cfg = PipelineConfig(H=H, W=W, C=C, batch=B, channels=tuple(chans), weights=weights)
    illum = _illum(a.illum_path, chans, H, W)
    n_pipes = max(1, min(a.pipes, (len(files) + B - 1) // B))
    streams, pipes = [], []
    for _ in range(n_pipes):
        st = torch.cuda.Stream(device=torch.device("cuda", a.device))
        with torch.cuda.stream(st):
            pipes.append(FovPipeline(Device(a.device), cfg, illum))
        streams.append(st)
    out = PlateTables(chans)

    def read_fov(paths):
        planes = []
        for p in paths:
            if os.path.exists(p):
                x = tiffio.imread(p)
                if x.shape != (H, W):
                    raise ValueError(f"{p}: shape {x.shape}, expected {(H, W)}")
                planes.append(x.astype(np.uint16, copy=False))
            else:
                log.warning("missing plane %s: zeros used", p)
                planes.append(np.zeros((H, W), np.uint16))
        return np.stack(planes)

    hosts = [torch.empty((B * C, H, W), dtype=torch.int16, pin_memory=True) for _ in range(n_pipes)]
    batches = [list(range(i, min(i + B, len(files)))) for i in range(0, len(files), B)]
    inflight = []  # (batch index, pipeline, slot, upload event)

    def record(bi, res):
        idx = batches[bi]
        for k, row_i in enumerate(idx):
            img_no = int(table.index[row_i]) + 1   # the LoadData row, also after QC filtering
            meta = table.iloc[row_i].to_dict()
            q = res.qc[k * C:(k + 1) * C]
            counts = {s: int(res.hdr[s][k]["n_objects"]) for s in OBJECT_SETS}
            out.add_image(img_no, meta, q["slope"], q["pct_max"], counts)
            for s in OBJECT_SETS:
                out.add_objects(s, img_no, res.objects[s][k]["label"], res.feats[s][k])
        log.info("batch %d/%d: %d FOVs", bi + 1, len(batches), len(idx))

    with concurrent.futures.ThreadPoolExecutor(max_workers=max(1, a.threads)) as pool:
        pending = [pool.submit(read_fov, files[i]) for i in batches[0]]
        for bi, idx in enumerate(batches):
            fovs = [f.result() for f in pending]
            if bi + 1 < len(batches):  # decode the next batch while this one runs
                pending = [pool.submit(read_fov, files[i]) for i in batches[bi + 1]]
            p_i = bi % n_pipes
            # the pinned staging buffer of this pipeline is free once its last upload completed
            for _, q, _, up in inflight:
                if q is pipes[p_i]:
                    up.synchronize()
            host = hosts[p_i]
            hn = host.numpy().view(np.uint16).reshape(B, C, H, W)
            hn[:len(fovs)] = np.stack(fovs)
            hn[len(fovs):] = 0
            with torch.cuda.stream(streams[p_i]):
                pipes[p_i].raw.copy_(host, non_blocking=True)
                up = torch.cuda.Event()
                up.record(streams[p_i])
                slot = pipes[p_i].run()
            inflight.append((bi, pipes[p_i], slot, up))
            if len(inflight) > n_pipes:   # results in batch order, one step behind the GPU
                obi, q, sl, _ = inflight.pop(0)
                record(obi, q.fetch(sl))
        while inflight:
            obi, q, sl, _ = inflight.pop(0)
            record(obi, q.fetch(sl))
    d = out.write(a.out, plate, time)
    log.info("tables written to %s", d)
    return d


if __name__ == "__main__":
    run()
