"""Multi-process plate runs (cpx.plate / cpx.launch): well shards,
per-rank parquet parts, merge into CSVs sorted by (ImageNumber, ObjectNumber) — byte-identical
to one process.  CPU: world-2 gloo ranks with a stub measurement; GPU: two real pipeline
processes on the one GPU vs one process."""
import argparse
import filecmp
import json
import os
import socket
import time
import zlib

import numpy as np
import pandas as pd
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from cpx import plate
from cpx.csvout import OBJECT_TABLES, PlateTables


def _table(n_wells=7, sites=3):
    rows = []
    for w in range(n_wells):
        for s in range(sites):
            rows.append({"Metadata_Plate": "P01", "Metadata_Well": f"C{w + 1:02d}", "Metadata_Site": s + 1,
                         "Metadata_Timepoint": 24, "FileName_DNA": f"w{w}s{s}.tiff"})
    return pd.DataFrame(rows)


def _stub_frames(table, rows, chans=("DNA",)):
    """Deterministic fake measurements of the given LoadData rows."""
    out = PlateTables(list(chans))
    status = []
    for i in rows:
        img = i + 1
        rng = np.random.default_rng(img)
        k = int(rng.integers(0, 4))
        out.add_image(img, table.iloc[i].to_dict(), rng.standard_normal(1), rng.random(1),
                      {t: k for t in OBJECT_TABLES})
        for t in OBJECT_TABLES:
            out.add_objects(t, img, np.arange(1, k + 1), rng.standard_normal((k, len(out.cols))))
        status.append({"ImageNumber": img, "status": "success" if k else "empty", "n_cells": k})
    f = out.frames()
    f["site_status"] = pd.DataFrame(status, columns=["ImageNumber", "status", "n_cells"])
    return f


def test_shard_rows_keeps_wells_together():
    t = _table()
    parts = [plate.shard_rows(t, r, 3) for r in range(3)]
    assert sorted(sum(parts, [])) == list(range(len(t)))
    for r, p in enumerate(parts):
        assert {w % 3 for w in t.iloc[p]["Metadata_Well"].str[1:].astype(int) - 1} == {r}
    assert plate.shard_rows(t, 0, 1) == list(range(len(t)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, d):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = _table()
        plate.write_part(d, rank, world, _stub_frames(t, plate.shard_rows(t, rank, world)))
        dist.barrier()
        if rank == 0:
            plate.merge_parts(d, world)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gloo_world2_parts_merge_byte_identical(tmp_path):
    t = _table()
    one = tmp_path / "one"
    one.mkdir()
    for name, df in _stub_frames(t, list(range(len(t)))).items():
        df.to_csv(one / f"{name}.csv", index=False)
    two = tmp_path / "two"
    two.mkdir()
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, str(two))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert not (two / plate.PARTS).exists()
    for name in ("Image", *OBJECT_TABLES, "site_status"):
        assert filecmp.cmp(one / f"{name}.csv", two / f"{name}.csv", shallow=False), name


@pytest.mark.gpu
def test_launch_two_processes_one_gpu_byte_identical(tmp_path, dev):
    """cpx.launch with two ranks on the one GPU == one cpx.plate process, byte for byte; a
    missing plane gives the reference's 'empty' site in both."""
    from cpx import launch, tiffio
    from cpx.synth import synth_fovs
    n, C, H, W = 6, 2, 384, 416
    chans = ["DNA", "AGP"]
    raw = synth_fovs(n, C, H, W, dev.torch_device, seed=9).cpu().numpy().view(np.uint16)
    imgdir = tmp_path / "images"
    imgdir.mkdir()
    rows = []
    for f in range(n):
        row = {"Metadata_Plate": "P03", "Metadata_Well": f"D{f // 2 + 1:02d}", "Metadata_Site": f % 2 + 1,
               "Metadata_Timepoint": 6}
        for c, ch in enumerate(chans):
            name = f"f{f}c{c}.tiff"
            if not (f == 3 and c == 1):  # one missing plane -> empty site
                tiffio.imwrite(str(imgdir / name), raw[f * C + c])
            row[f"FileName_{ch}"] = name
        rows.append(row)
    ld = tmp_path / "ld.csv"
    pd.DataFrame(rows).to_csv(ld, index=False)
    common = ["--load-data", str(ld), "--data-path", str(imgdir), "--channels", *chans,
              "--batch", "2", "--threads", "2", "--pipes", "1"]
    d1 = plate.run(common + ["--out", str(tmp_path / "one"), "--world", "1", "--rank", "0"])
    dirs = launch.main(["--gpus", "2", "--devices", "0,0", "--", *common, "--out", str(tmp_path / "two")])
    d2 = dirs[0]
    st = pd.read_csv(os.path.join(d1, "site_status.csv"))
    assert st.loc[st.ImageNumber == 4, "status"].item() == "empty"
    for name in ("Image", *OBJECT_TABLES, "site_status"):
        assert filecmp.cmp(os.path.join(d1, f"{name}.csv"), os.path.join(d2, f"{name}.csv"), shallow=False), name


def _claimer(qdir, n_batches, out_path, delay):
    import time as _t
    a = argparse.Namespace(queue=qdir, world=3, rank=0, batch=4)
    table = pd.DataFrame({"x": range(4 * n_batches - 1)})  # last batch short
    got = []
    for rows in plate.batch_source(table, a, 0):
        got.append(rows)
        _t.sleep(delay)
    with open(out_path, "w") as f:
        json.dump(got, f)


def test_work_queue_claims_every_batch_once(tmp_path):
    """Three processes drain one job's WorkQueue: every batch (4 consecutive rows, the last one
    short) is claimed by exactly one of them, and the slow claimer takes fewer."""
    ctx = mp.get_context("spawn")
    n = 23
    outs = [str(tmp_path / f"r{r}.json") for r in range(3)]
    procs = [ctx.Process(target=_claimer, args=(str(tmp_path / "q"), n, outs[r], d))
             for r, d in enumerate((0.002, 0.002, 0.05))]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    claimed = [json.load(open(o)) for o in outs]
    flat = sorted((b for c in claimed for b in c), key=lambda b: b[0])
    assert flat == [list(range(4 * k, min(4 * n - 1, 4 * k + 4))) for k in range(n)]
    assert len(claimed[2]) < len(claimed[0]) + len(claimed[1])


def test_work_queue_reused_directory(tmp_path, caplog):
    """A --queue directory left by an earlier run: with a new --queue-token (cpx.launch passes
    one) the stale counter restarts and every batch is claimed; without a token the exhausted
    counter is reported instead of silently yielding nothing."""
    table = pd.DataFrame({"x": range(10)})
    q = str(tmp_path / "q")
    old = argparse.Namespace(queue=q, world=2, rank=0, batch=4, queue_token="run1")
    assert [r for r in plate.batch_source(table, old, 0)] == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9]]
    new = argparse.Namespace(queue=q, world=2, rank=0, batch=4, queue_token="run2")
    assert [r for r in plate.batch_source(table, new, 0)] == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9]]
    bare = argparse.Namespace(queue=q, world=2, rank=0, batch=4, queue_token=None)
    with open(os.path.join(q, "job0000.ctr"), "w") as f:
        f.write("- 3")  # an exhausted counter of an earlier token-less run
    with caplog.at_level("ERROR", logger="cpx.plate"):
        assert list(plate.batch_source(table, bare, 0)) == []
    assert "already exhausted" in caplog.text


# ---- configs[3]'s job shape at world size 8 (multi-GPU readiness without hardware)
# 8 plates x 4 times = 32 (plate, time) jobs, one LoadData CSV each (Feature_extraction_opt.py:
# 63-76 fans them out), drained by eight ranks from the shared WorkQueue of cpx.plate exactly as
# on an 8-GPU node; the per-site GPU measurement is replaced by a deterministic CPU stub of what
# FovPipeline.fetch hands plate.run (the same add_image / add_objects / status calls).

W8_CHANS = ("DNA", "AGP")


def _w8_jobs(tmp, n_plates=8, times=(6, 12, 24, 48), wells=3, sites=2):
    paths = []
    for p in range(n_plates):
        for t in times:
            rows = [{"Metadata_Plate": f"P{p + 1:02d}", "Metadata_Well": f"B{w + 1:02d}", "Metadata_Site": s + 1,
                     "Metadata_Timepoint": t, **{f"FileName_{c}": f"p{p}t{t}w{w}s{s}{c}.tiff" for c in W8_CHANS}}
                    for w in range(wells) for s in range(sites)]
            path = os.path.join(tmp, f"ld_P{p + 1:02d}_{t}.csv")
            pd.DataFrame(rows).to_csv(path, index=False)
            paths.append(path)
    return paths


def _w8_stub_run_sites(claims_path):
    """A _run_sites that measures each claimed batch with a seeded stub (no GPU) and logs the
    claimed rows per job to claims_path."""
    def run_sites(a, table, source, chans, state, out, status):
        n = 0
        job = f"{table['Metadata_Plate'].iloc[0]}/{table['Metadata_Timepoint'].iloc[0]}"
        for rows in source:
            with open(claims_path, "a") as f:
                f.write(json.dumps({"job": job, "rows": rows}) + "\n")
            time.sleep(0.02)  # (so that every rank gets to claim, as slower GPU batches would)
            for r in rows:
                img = int(table.index[r]) + 1
                meta = table.iloc[r].to_dict()
                rng = np.random.default_rng([zlib.crc32(job.encode()), img])
                k = int(rng.integers(0, 5))
                out.add_image(img, meta, rng.standard_normal(len(chans)), rng.random(len(chans)),
                              {t: k for t in OBJECT_TABLES})
                for t in OBJECT_TABLES:
                    out.add_objects(t, img, rng.permutation(np.arange(1, k + 1)),
                                    rng.standard_normal((k, len(out.cols))))
                status.append({"ImageNumber": img, "status": "success" if k else "empty", "n_cells": k})
                n += 1
        state["timing"] = {}
        return n
    return run_sites


def _w8_rank(rank, world, port, argv, claims_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    plate._run_sites = _w8_stub_run_sites(claims_path)
    plate.run(argv + ["--rank", str(rank), "--world", str(world)])
    dist.destroy_process_group()


def test_gloo_world8_work_queue_configs3_jobs(tmp_path):
    """Eight gloo ranks drain 32 jobs (8 plates x 4 times, 2 FOVs per batch) from one WorkQueue:
    every batch of every job is claimed exactly once, the merged <plate>/<time>/ CSVs equal a
    one-process run byte for byte, and the per-rank claim counts are reported."""
    jobs = _w8_jobs(str(tmp_path))
    common = ["--load-data", *jobs, "--data-path", str(tmp_path), "--channels", *W8_CHANS, "--batch", "2"]
    # one process
    plate._run_sites, keep = _w8_stub_run_sites(str(tmp_path / "claims_w1.jsonl")), plate._run_sites
    try:
        plate.run(common + ["--out", str(tmp_path / "one"), "--world", "1", "--rank", "0"])
    finally:
        plate._run_sites = keep
    # eight ranks, one shared queue
    world, port = 8, _port()
    argv = common + ["--out", str(tmp_path / "eight"), "--queue", str(tmp_path / "queue"), "--queue-token", "w8"]
    claims = [str(tmp_path / f"claims_r{r}.jsonl") for r in range(world)]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_w8_rank, args=(r, world, port, argv, claims[r])) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    got = {}
    per_rank = []
    for r, c in enumerate(claims):
        lines = [json.loads(x) for x in open(c)] if os.path.exists(c) else []
        per_rank.append(len(lines))
        for x in lines:
            got.setdefault(x["job"], []).append(x["rows"])
    print("[world8] batches claimed per rank:", per_rank, flush=True)
    assert len(got) == len(jobs)
    for job, batches in got.items():  # 6 rows per job -> batches [0,1], [2,3], [4,5], once each
        assert sorted(batches) == [[0, 1], [2, 3], [4, 5]], (job, batches)
    assert sum(per_rank) == 3 * len(jobs)
    for p in range(8):
        for t in (6, 12, 24, 48):
            d1, d8 = tmp_path / "one" / f"P{p + 1:02d}" / str(t), tmp_path / "eight" / f"P{p + 1:02d}" / str(t)
            assert not (d8 / plate.PARTS).exists()
            for name in ("Image", *OBJECT_TABLES, "site_status"):
                assert filecmp.cmp(d1 / f"{name}.csv", d8 / f"{name}.csv", shallow=False), (p, t, name)
