"""Host budget of the plate CLI's TIFF decode for 8 GPUs, without the GPU.

cpx.plate decodes each site's C uncompressed 2080 x 2080 uint16 planes with a thread pool
(tiffio.read_into: header parse + readinto straight into the staging buffer).  One GPU at R
FOV/s needs R x 43.3 MB/s of decode; 8 GPUs need 8 such pools on one host.  This runs P pools
(processes) of T threads each concurrently over the same page-cached files for a fixed time and
reports the aggregate and per-pool decode rate in GB/s and FOV/s (43.3 MB per FOV).

  python tools/decode_budget.py [--pools 1 8] [--threads 16] [--seconds 8] [--fovs 48]
"""
import argparse
import json
import multiprocessing as mp
import os
import shutil
import sys
import tempfile
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))

FOV_BYTES = 5 * 2080 * 2080 * 2


def _pool(files, threads, seconds, q):
    import numpy as np
    from cpx import tiffio
    stop = time.perf_counter() + seconds
    done = [0] * threads

    def work(t):
        buf = np.empty((2080, 2080), np.uint16)
        i = t
        while time.perf_counter() < stop:
            tiffio.read_into(files[i % len(files)], buf)
            done[t] += 1
            i += threads
    ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    q.put((sum(done), time.perf_counter() - t0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pools", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--fovs", type=int, default=48)
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()
    import numpy as np
    from cpx import tiffio
    root = tempfile.mkdtemp(prefix="cpx_decode_", dir=a.dir)
    try:
        rng = np.random.default_rng(0)
        files = []
        for f in range(a.fovs):
            for c in range(5):
                p = os.path.join(root, f"f{f}_c{c}.tiff")
                tiffio.imwrite(p, rng.integers(0, 65535, (2080, 2080), dtype=np.uint16))
                files.append(p)
        plane = os.path.getsize(files[0])
        out = {"metric": "host TIFF decode rate (cpx.tiffio.read_into, page-cached uncompressed planes)",
               "plane_bytes": plane, "threads_per_pool": a.threads, "cpu_count": os.cpu_count(),
               "affinity": len(os.sched_getaffinity(0)), "runs": []}
        ctx = mp.get_context("fork")
        for P in a.pools:
            q = ctx.Queue()
            procs = [ctx.Process(target=_pool, args=(files, a.threads, a.seconds, q)) for _ in range(P)]
            for pr in procs:
                pr.start()
            res = [q.get() for _ in procs]
            for pr in procs:
                pr.join()
            gbs = [n * plane / s / 1e9 for n, s in res]
            out["runs"].append({"pools": P, "aggregate_GBs": round(sum(gbs), 2),
                                "per_pool_GBs": [round(x, 2) for x in gbs],
                                "per_pool_FOVs": [round(x * 1e9 / FOV_BYTES, 1) for x in gbs]})
            print(json.dumps(out["runs"][-1]), flush=True)
        print(json.dumps(out), flush=True)
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
