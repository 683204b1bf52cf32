"""One process per GPU for the plate/time measurement runs.

    python -m cpx.launch --gpus 8 -- --load-data ld_P01_6.csv ld_P01_24.csv ... \\
        --data-path IMAGES --illum-path ILLUM --channels DNA ER RNA AGP Mito --out RESULTS

Starts N `cpx.plate` processes (rank r sees only GPU devices[r] through HIP_VISIBLE_DEVICES,
as the reference pins each consumer with CUDA_VISIBLE_DEVICES, Cellpose_GPU_s3fs.py:97,295);
the ranks claim the batches of every (plate, time) job from shared per-job counters (a fresh
cpx.plate --queue directory per run: a rank that finishes sooner claims more) and write their rows
as parts; once all exit cleanly the launcher merges every job's parts into the final CSVs.  The launcher itself
never touches a GPU.  --devices repeats a device to run several ranks on one GPU (tests).
"""
from __future__ import annotations

import argparse
import glob
import json
import logging
import os
import shutil
import subprocess
import sys
import time

from .plate import merge_parts, parse_args as plate_args

log = logging.getLogger("cpx.launch")


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--" not in argv:
        raise SystemExit("usage: python -m cpx.launch --gpus N [--devices 0,1,..] -- <cpx.plate args>")
    k = argv.index("--")
    ap = argparse.ArgumentParser(prog="python -m cpx.launch")
    ap.add_argument("--gpus", type=int, required=True)
    ap.add_argument("--devices", default=None, help="comma list of device ids per rank (default 0..N-1)")
    a = ap.parse_args(argv[:k])
    rest = argv[k + 1:]
    pa = plate_args(rest)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s: %(message)s")
    n = a.gpus
    devs = [int(x) for x in a.devices.split(",")] if a.devices else list(range(n))
    if len(devs) != n:
        raise SystemExit(f"--devices lists {len(devs)} ids for {n} ranks")
    os.makedirs(pa.out, exist_ok=True)
    for f in glob.glob(os.path.join(pa.out, ".cpx_jobs_r*.json")):
        os.remove(f)
    pkg_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # fresh shared batch counters for this run (cpx.plate.WorkQueue): ranks claim batches
    token = f"{os.getpid()}_{time.time_ns()}"
    qdir = os.path.join(pa.out, f".cpx_queue_{token}")
    os.makedirs(qdir)
    procs = []
    for r in range(n):
        env = dict(os.environ, HIP_VISIBLE_DEVICES=str(devs[r]), RANK=str(r), WORLD_SIZE=str(n))
        env.pop("MASTER_ADDR", None)  # no process group: the launcher merges
        env["PYTHONPATH"] = pkg_root + os.pathsep + env.get("PYTHONPATH", "")
        cmd = [sys.executable, "-m", "cpx.plate", *rest, "--rank", str(r), "--world", str(n),
               "--device", "0", "--no-merge", "--queue", qdir, "--queue-token", token]
        procs.append(subprocess.Popen(cmd, env=env))
    rcs = [p.wait() for p in procs]
    shutil.rmtree(qdir, ignore_errors=True)
    if any(rcs):
        raise SystemExit(f"rank exit codes {rcs}: parts left unmerged under {pa.out}")
    dirs = []
    for r in range(n):
        with open(os.path.join(pa.out, f".cpx_jobs_r{r:04d}.json")) as f:
            for d in json.load(f):
                if d not in dirs:
                    dirs.append(d)
        os.remove(os.path.join(pa.out, f".cpx_jobs_r{r:04d}.json"))
    for d in dirs:
        merge_parts(d, n)
        log.info("merged %d parts -> %s", n, d)
    return dirs


if __name__ == "__main__":
    main()
