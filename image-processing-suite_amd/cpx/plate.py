"""Plate/time measurement run: LoadData CSV + TIFF planes -> the four CSV tables.

Replaces the CellProfiler job that Feature_extraction_opt.py:159-177 launches per (plate, time)
(LoadData CSV in, per-object tables synced to `<base>/<plate>/<time>/`), with the GPU pipeline
of cpx.pipeline: flat-field + QC -> Cellpose-restated segmentation -> Cells/Cytoplasm -> object
tables -> features, in batches of FOVs resident in HBM.  Host threads decode the next batch's
TIFFs while the GPU works on the current one.

  python -m cpx.plate --load-data load_data_P01_24_illum.csv [more LoadData files ...] \
      --data-path IMAGES --illum-path ILLUM --channels DNA ER RNA AGP Mito --out RESULTS

Channel files come from FileName_<ch> (relative to --data-path); flat-fields from
<ch>_illum.npy or Illum<ch>.npy (as the QC tool); plate and time from Metadata_Plate /
Metadata_Timepoint unless given.  Every LoadData file is one (plate, time) job.

Multi-GPU (the reference's per-GPU consumers Cellpose_GPU_s3fs.py:269-300 and
per-(plate, time) jobs Feature_extraction_opt.py:63-76): one process per GPU (`cpx.launch`, or
torchrun with RANK / WORLD_SIZE); the ranks claim the batches of each (plate, time) job from a
shared per-job counter (WorkQueue, --queue: a rank that finishes sooner claims more) or, without
--queue, each drains its static well shard (wells dealt round-robin in first-appearance order);
each writes its rows as parquet parts; the parts are merged into the final CSVs sorted by
(ImageNumber, ObjectNumber), byte-identical for any number of processes.  No collective touches
the data path.  Batches always hold --batch FOVs (the tail is zero-padded), so every process runs
the same kernels on the same batch shape.
"""
from __future__ import annotations

import argparse
import concurrent.futures
import glob
import json
import logging
import os
import shutil
import sys
import time
import time as _time  # run() binds `time` to the job's timepoint

import numpy as np

# Hardware queues: with HIP's default of four per process the plate run's two pipelines hardly
# overlap on the GPU — kernels of both ran together 3-5 % of the time, also with the uploads moved
# onto the result-copy stream (`profiles/r05ai_plate_overlap_q4.txt`, `r05ap_plate_overlap.txt`)
# — against 39 % with eight (`r05aj_plate_overlap_q8.txt`); plate bench 362.8 -> 378.5 FOV/s on
# 768 FOVs and 368 -> 391 on 1,536 (means of `r05aj_plate_bench.jsonl`, `r05ap_plate_bench.jsonl`).
# HIP reads it when the process first uses the GPU, so it takes effect when this module is
# imported first (`python -m cpx.plate`, cpx.launch's ranks).  A lower value in the environment
# (the GPU boxes export HIP's default of 4) is raised; CPX_PLATE_HW_QUEUES overrides the 8.
PLATE_HW_QUEUES = int(os.environ.get("CPX_PLATE_HW_QUEUES", "8"))
_HW_QUEUES_LATE = False  # the raise came after HIP was initialised in this process (no effect)
if int(os.environ.get("GPU_MAX_HW_QUEUES") or 4) < PLATE_HW_QUEUES:
    _torch = sys.modules.get("torch")
    _HW_QUEUES_LATE = bool(_torch is not None and _torch.cuda.is_initialized())
    os.environ["GPU_MAX_HW_QUEUES"] = str(PLATE_HW_QUEUES)

log = logging.getLogger("cpx.plate")
# per job of the last run(): {"job", "fovs", "seconds", "threads", "batch", "pipes"} — decode, upload,
# GPU pipeline and table assembly, from the first decode to the last recorded site (pipeline
# construction excluded); the I/O-inclusive throughput of the drop-in (tools/plate_bench.py)
LAST_TIMING: list = []
PARTS = ".parts"


def parse_args(argv=None):
    ap = argparse.ArgumentParser(prog="python -m cpx.plate", description="GPU per-object measurement of one plate/time")
    ap.add_argument("--load-data", required=True, nargs="+", help="one LoadData CSV per (plate, time) job")
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
    ap.add_argument("--rank", type=int, default=int(os.environ.get("RANK", "0")),
                    help="this process's rank (well shard); default $RANK")
    ap.add_argument("--world", type=int, default=int(os.environ.get("WORLD_SIZE", "1")),
                    help="processes (GPUs) sharing the jobs; default $WORLD_SIZE")
    ap.add_argument("--queue", default=None,
                    help="with --world > 1: directory of the shared per-job batch counters (dynamic work "
                         "queue across the ranks; cpx.launch creates a fresh one); default: static well shards")
    ap.add_argument("--queue-token", default=os.environ.get("CPX_QUEUE_TOKEN"),
                    help="run identifier stored with the --queue counters: a counter left by another run "
                         "(another token) starts over instead of reading as exhausted (cpx.launch sets one)")
    ap.add_argument("--cpnet-precision", choices=("f16x3", "bf16", "fp32"), default="f16x3",
                    help="CPnet arithmetic (PipelineConfig.cpnet_precision): f16x3 = split-fp16 MFMA kernels "
                         "at the fp32 network's accuracy (default; a FOV whose activations leave the fp16 "
                         "range is re-run in fp32), fp32 = the eager PyTorch module, bf16 = native bf16")
    ap.add_argument("--no-merge", action="store_true",
                    help="with --world > 1: leave the parts for cpx.launch / merge_parts")
    ap.add_argument("--ws-rounds", type=int, nargs=2, default=None, metavar=("RELAX", "LABEL"),
                    help="Cells watershed rounds enqueued per batch (default: PipelineConfig.ws_rounds)")
    return ap.parse_args(argv)


def shard_rows(table, rank: int, world: int):
    """Row positions of `rank`: wells dealt round-robin in first-appearance order (all sites of
    a well on one rank); rows without Metadata_Well are dealt one by one."""
    if world <= 1:
        return list(range(len(table)))
    if "Metadata_Well" in table:
        order = {}
        wells = [order.setdefault(w, len(order)) for w in table["Metadata_Well"].astype(str)]
        return [i for i, w in enumerate(wells) if w % world == rank]
    return [i for i in range(len(table)) if i % world == rank]


class WorkQueue:
    """Batch counter of one (plate, time) job shared by the ranks of one node: a file advanced
    under an exclusive flock, so each rank claims the next unclaimed batch of --batch consecutive
    LoadData rows and a rank whose batches finish sooner claims more (the reference's GPU consumers
    draw sites from one shared queue, Cellpose_GPU_s3fs.py:269-300).  The merged tables do not
    depend on which rank measured a site (merge_parts sorts the rows)."""

    def __init__(self, qdir: str, key: str, token: str | None = None):
        os.makedirs(qdir, exist_ok=True)
        self.path = os.path.join(qdir, f"{key}.ctr")
        self.token = token or "-"
        if any(c.isspace() for c in self.token):
            raise ValueError("WorkQueue token must not contain whitespace")

    def take(self) -> int:
        """Claim the next batch index.  The counter file holds "<token> <next>"; a counter written
        under another token (a reused --queue directory) restarts at 0 for this run."""
        import fcntl
        fd = os.open(self.path, os.O_RDWR | os.O_CREAT, 0o644)
        try:
            fcntl.flock(fd, fcntl.LOCK_EX)
            raw = os.read(fd, 256).decode().split()
            k = int(raw[1]) if len(raw) == 2 and raw[0] == self.token else 0
            if raw and k == 0:
                log.warning("%s: counter of another run (%s) found; restarting it for token %s",
                            self.path, " ".join(raw), self.token)
            os.lseek(fd, 0, os.SEEK_SET)
            os.ftruncate(fd, 0)
            os.write(fd, f"{self.token} {k + 1}".encode())
            return k
        finally:
            os.close(fd)  # releases the lock


def batch_source(table, a, job_index: int):
    """Lists of table row positions, one per GPU batch, for this rank: claimed from the job's
    WorkQueue (--queue, world > 1) or this rank's static well shard (shard_rows)."""
    B = max(1, a.batch)
    if a.queue and a.world > 1:
        q = WorkQueue(a.queue, f"job{job_index:04d}", getattr(a, "queue_token", None))
        nb = (len(table) + B - 1) // B
        first = True
        while True:
            k = q.take()
            if k >= nb:
                if first and nb and not getattr(a, "queue_token", None):
                    log.error("%s: the job's counter is already exhausted on this rank's first claim (%d >= %d "
                              "batches): a --queue directory reused without --queue-token?", q.path, k, nb)
                return
            first = False
            yield list(range(k * B, min(len(table), (k + 1) * B)))
    else:
        mine = shard_rows(table, a.rank, a.world)
        for i in range(0, len(mine), B):
            yield mine[i:i + B]


def job_dir(out, plate, time):
    return os.path.join(out, str(plate), str(time))


def write_part(d, rank, world, frames: dict):
    """One rank's rows of one (plate, time) job as parquet (exact dtypes and floats)."""
    pdir = os.path.join(d, PARTS, f"r{rank:04d}of{world:04d}")
    os.makedirs(pdir, exist_ok=True)
    for name, df in frames.items():
        df.to_parquet(os.path.join(pdir, f"{name}.parquet"), index=False)
    return pdir


def merge_parts(d, world=None):
    """Concatenate the ranks' parts of job directory d into the final CSVs (rows sorted by
    ImageNumber, then ObjectNumber) and remove the parts."""
    import pandas as pd

    from .csvout import write_frame_csv
    parts = sorted(glob.glob(os.path.join(d, PARTS, "r*of*")))
    if world is not None and len(parts) != world:
        raise RuntimeError(f"{d}: {len(parts)} parts, expected {world}")
    names = sorted({os.path.splitext(f)[0] for p in parts for f in os.listdir(p)})
    for name in names:
        blocks = [pd.read_parquet(os.path.join(p, name + ".parquet")) for p in parts
                  if os.path.exists(os.path.join(p, name + ".parquet"))]
        blocks = [b for b in blocks if len(b)] or blocks[:1]
        df = pd.concat(blocks, ignore_index=True)
        keys = [k for k in ("ImageNumber", "ObjectNumber") if k in df.columns]
        if keys and len(df):
            df = df.sort_values(keys, kind="stable").reset_index(drop=True)
        write_frame_csv(df, os.path.join(d, f"{name}.csv"))
    shutil.rmtree(os.path.join(d, PARTS), ignore_errors=True)
    return d


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


def _job_meta(a, load_data):
    """(table after the QC filter, plate, time) of one LoadData job."""
    import pandas as pd
    table = pd.read_csv(load_data)
    if a.csv_image_key:
        n0 = len(table)
        table = qc_filter(table, pd.read_csv(os.path.join(a.csv_image_key, "Image.csv")))
        log.info("image QC filter: %d of %d sites kept", len(table), n0)
    else:
        log.info("No csv_image_key provided — skipping image QC filtering.")
    plate = a.plate or (str(table["Metadata_Plate"].iloc[0]) if "Metadata_Plate" in table else "plate")
    time = a.time or (str(table["Metadata_Timepoint"].iloc[0]) if "Metadata_Timepoint" in table else "0")
    return table, plate, time


def run(argv=None):
    """Run every LoadData job's share of this rank; returns the job directories."""
    import pandas as pd
    from . import tiffio
    from .csvout import PlateTables
    from .pipeline import OBJECT_SETS

    a = parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s: %(message)s")
    if _HW_QUEUES_LATE:
        log.warning("GPU_MAX_HW_QUEUES was raised to %d after HIP was initialised in this process, so "
                    "the pipelines keep HIP's default hardware queues and overlap less; import "
                    "cpx.plate before any GPU call (python -m cpx.plate / cpx.launch do)", PLATE_HW_QUEUES)
    chans = list(a.channels)
    C = len(chans)
    LAST_TIMING.clear()
    state = {}  # pipelines, created for the first job's plane geometry and reused
    dirs = []
    for ji, load_data in enumerate(a.load_data):
        table, plate, time = _job_meta(a, load_data)
        # one rank: each FOV's rows formatted as it finishes and streamed into the job's CSVs
        out = PlateTables(chans, eager_csv=a.world == 1,
                          stream_dir=job_dir(a.out, plate, time) if a.world == 1 else None)
        status = []  # per site: the reference's results_dict entry (Cellpose_GPU_s3fs.py:123-125,219-223)
        d = job_dir(a.out, plate, time)
        try:
            nsites = _run_sites(a, table, batch_source(table, a, ji), chans, state, out, status)
            if nsites:
                LAST_TIMING.append({"job": os.path.basename(load_data), "fovs": nsites, **state["timing"]})
            site_status = pd.DataFrame(status, columns=["ImageNumber", "status", "n_cells"]) \
                .sort_values("ImageNumber", kind="stable").reset_index(drop=True)
            t_csv = _time.perf_counter()
            if a.world > 1:
                frames = out.frames()
                frames["site_status"] = site_status
                write_part(d, a.rank, a.world, frames)
            else:
                os.makedirs(d, exist_ok=True)
                frames = out.frames(objects=False)
                frames["site_status"] = site_status
                for name, df in frames.items():
                    df.to_csv(os.path.join(d, f"{name}.csv"), index=False)
                for t in OBJECT_SETS:  # the object tables, natively formatted (csvout.format_object_rows)
                    out.write_objects(d, t)
        finally:
            # on an error: the streamed partial tables are removed and the writer threads and
            # format pool stopped, so a failed job leaves no truncated object CSV behind
            out.close()
        if LAST_TIMING and nsites:
            LAST_TIMING[-1]["tables_write_s"] = round(_time.perf_counter() - t_csv, 3)
        log.info("rank %d/%d: %d sites of %s/%s -> %s", a.rank, a.world, nsites, plate, time, d)
        dirs.append(d)
    if a.world > 1:
        with open(os.path.join(a.out, f".cpx_jobs_r{a.rank:04d}.json"), "w") as f:
            json.dump(dirs, f)
        if not a.no_merge:
            _torchrun_merge(a, dirs)
    return dirs[0] if len(dirs) == 1 else dirs


def _torchrun_merge(a, dirs):
    """Under torchrun (a process group can be formed): barrier on gloo, rank 0 merges."""
    import torch.distributed as dist
    if not dist.is_available() or "MASTER_ADDR" not in os.environ:
        return
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=a.rank, world_size=a.world)
    dist.barrier()
    if a.rank == 0:
        for d in dirs:
            merge_parts(d, a.world)
    dist.barrier()


def _run_sites(a, table, source, chans, state, out, status):
    """Measure the batches `source` yields (lists of table row positions); returns the number of
    sites measured."""
    import torch
    from . import tiffio
    from .device import Device
    from .pipeline import OBJECT_SETS, FovPipeline, PipelineConfig
    C = len(chans)
    source = iter(source)
    first = next(source, None)
    if first is None:
        return 0

    def site_files(r):
        return [os.path.join(a.data_path, str(table.iloc[r][f"FileName_{ch}"])) for ch in chans]

    H = W = None
    # this job's plane geometry, from the first readable plane of this batch (else of the job)
    for fs in map(site_files, [*first, *range(len(table))]):
        try:
            H, W = tiffio.imread(fs[0]).shape
            break
        except Exception:  # noqa: BLE001
            continue
    if H is None:
        raise RuntimeError("no readable plane in this job")
    if "pipes" in state and (state["H"], state["W"]) != (H, W):
        # pipelines are sized for one plane geometry: rebuild them for this job's
        log.info("plane geometry %s -> %s: rebuilding the GPU pipelines", (state["H"], state["W"]), (H, W))
        state.clear()
        torch.cuda.synchronize()
    if "pipes" not in state:
        weights = a.weights
        if weights is None:
            cand = os.path.join(os.path.dirname(__file__), "weights", "cpnet_nuclei_synth.pt")
            weights = cand if os.path.exists(cand) else None
        B = max(1, a.batch)
        cfg = PipelineConfig(H=H, W=W, C=C, batch=B, channels=tuple(chans), weights=weights,
                             cpnet_precision=getattr(a, "cpnet_precision", "f16x3"))
        if a.ws_rounds:
            cfg.ws_rounds = tuple(a.ws_rounds)
        illum = _illum(a.illum_path, chans, H, W)
        from .device import pipeline_streams
        streams, pipes = [], []
        # unrestricted CUs here: with its uploads and result copies beside the pipelines the plate
        # measured 372-389 FOV/s with CU-split streams against 367-403 without (`gpurun_out/r05au`,
        # `r05az`; the HBM-resident bench gains from the split)
        split = "none"
        for st in pipeline_streams(a.device, max(1, a.pipes), split):
            with torch.cuda.stream(st):
                pipes.append(FovPipeline(Device(a.device), cfg, illum))
            streams.append(st)
        hosts = [torch.empty((B * C, H, W), dtype=torch.int16, pin_memory=True) for _ in pipes]
        state.update(pipes=pipes, streams=streams, hosts=hosts, B=B, H=H, W=W)
    pipes, streams, hosts = state["pipes"], state["streams"], state["hosts"]
    B, H, W = state["B"], state["H"], state["W"]
    n_pipes = len(pipes)

    # where the time goes (tools/plate_bench.py): host seconds the main thread waited for the
    # decode threads / for fetch (GPU + D2H), decode-thread seconds, table assembly seconds, and
    # GPU milliseconds of the uploads and of the pipeline steps (HIP events on the stream)
    tm = {"decode_wait_s": 0.0, "decode_thread_s": 0.0, "fetch_wait_s": 0.0, "tables_s": 0.0,
          "h2d_gpu_ms": 0.0, "pipeline_gpu_ms": 0.0}

    def read_fov(paths, dst):
        """Decode the site's C planes straight into dst [C][H][W] (a slice of the pinned staging
        buffer); False when any of them cannot be read (missing, undecodable, other shape): the
        reference's producer then sends (site_id, None) and the consumer records the site as
        {'status': 'empty', 'n_cells': 0} (Cellpose_GPU_s3fs.py:76-87, 123-136)."""
        t0 = time.perf_counter()
        try:
            for c, p in enumerate(paths):
                tiffio.read_into(p, dst[c])
            return True
        except Exception as e:  # noqa: BLE001
            log.error("failed on site %s: %s", paths, e)
            dst[...] = 0
            return False
        finally:
            tm["decode_thread_s"] += time.perf_counter() - t0

    batches = [first]  # row positions per batch, grown as batches are claimed
    inflight = []  # (batch index, pipeline, slot, upload event, empty flags)
    uploads = [None] * n_pipes  # last upload event per staging buffer
    t_start = time.perf_counter()

    def record(bi, res, empty):
        idx = batches[bi]
        for k, row_i in enumerate(idx):
            img_no = int(table.index[row_i]) + 1   # the LoadData row, also after QC filtering
            meta = table.iloc[row_i].to_dict()
            if empty[k]:  # unreadable site: no measurements, no object rows
                nan = [float("nan")] * C
                out.add_image(img_no, meta, nan, nan, {s: 0 for s in OBJECT_SETS})
                status.append({"ImageNumber": img_no, "status": "empty", "n_cells": 0})
                continue
            q = res.qc[k * C:(k + 1) * C]
            counts = {s: int(res.hdr[s][k]["n_objects"]) for s in OBJECT_SETS}
            if res.failed is not None and res.failed[k]:  # segmentation step failed for this site
                out.add_image(img_no, meta, q["slope"], q["pct_max"], counts)
                status.append({"ImageNumber": img_no, "status": "empty", "n_cells": 0})
                continue
            out.add_image(img_no, meta, q["slope"], q["pct_max"], counts)
            for s in OBJECT_SETS:
                out.add_objects(s, img_no, res.objects[s][k]["label"], res.feats[s][k])
            n = counts["Nuclei"]
            status.append({"ImageNumber": img_no, "status": "success" if n else "empty", "n_cells": n})
        log.info("batch %d: %d FOVs", bi + 1, len(idx))

    def decode(bi, pool):
        """Decode batch bi into its pipeline's pinned staging buffer (after that buffer's last
        upload completed); the tail of a short batch is zero-filled."""
        p_i = bi % n_pipes
        if uploads[p_i] is not None:
            uploads[p_i].synchronize()
        hn = hosts[p_i].numpy().view(np.uint16).reshape(B, C, H, W)
        idx = batches[bi]
        hn[len(idx):] = 0
        return [pool.submit(read_fov, site_files(r), hn[k]) for k, r in enumerate(idx)]

    def retire():
        obi, q, sl, evs, em = inflight.pop(0)
        t0 = time.perf_counter()
        res = q.fetch(sl)
        t1 = time.perf_counter()
        record(obi, res, em)
        tm["fetch_wait_s"] += t1 - t0
        tm["tables_s"] += time.perf_counter() - t1
        tm["h2d_gpu_ms"] += evs[0].elapsed_time(evs[1])
        tm["pipeline_gpu_ms"] += evs[2].elapsed_time(evs[3])

    with concurrent.futures.ThreadPoolExecutor(max_workers=max(1, a.threads)) as pool:
        pending = decode(0, pool)
        bi = 0
        while bi < len(batches):
            t0 = time.perf_counter()
            empty = [not f.result() for f in pending]
            tm["decode_wait_s"] += time.perf_counter() - t0
            p_i = bi % n_pipes
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            # the upload runs on the device's upload stream, so it overlaps this pipeline's
            # previous batch and the other pipelines' kernels, and the result fetches (on the copy
            # stream) never wait behind it; the pipeline's stream waits for it.  pipes[p_i].raw
            # is the staging buffer of the pipeline's next result slot, whose previous batch was
            # fetched (retired) before this one was claimed
            cs = FovPipeline.upload_stream(torch.device("cuda", a.device))
            with torch.cuda.stream(cs):
                evs[0].record(cs)
                pipes[p_i].raw.copy_(hosts[p_i], non_blocking=True)
                evs[1].record(cs)
            uploads[p_i] = evs[1]
            streams[p_i].wait_event(evs[1])
            with torch.cuda.stream(streams[p_i]):
                evs[2].record(streams[p_i])
                slot = pipes[p_i].run()
                evs[3].record(streams[p_i])
            inflight.append((bi, pipes[p_i], slot, evs, empty))
            nxt = next(source, None)  # claim and decode the next batch while this one runs
            if nxt is not None:
                batches.append(nxt)
                pending = decode(bi + 1, pool)
            if len(inflight) > n_pipes:   # results in batch order, one step behind the GPU
                retire()
            bi += 1
        while inflight:
            retire()
    secs = time.perf_counter() - t_start
    nsites = sum(len(b) for b in batches)
    state["timing"] = {"seconds": secs, "threads": a.threads, "batch": B, "pipes": n_pipes,
                       **{k: round(v, 3) for k, v in tm.items()}}
    log.info("%d sites in %.2f s: %.1f FOV/s (decode threads %d, batch %d, pipelines %d)",
             nsites, secs, nsites / max(secs, 1e-9), a.threads, B, n_pipes)
    return nsites


if __name__ == "__main__":
    run()
