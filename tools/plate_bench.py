"""I/O-inclusive throughput of the drop-in (configs[3]'s streamed input): the
plate CLI (cpx.plate) on uncompressed 2080 x 2080 x 5ch TIFFs on local disk — host TIFF decode
threads, pinned upload, the GPU pipeline, the table assembly and the four CSV files — timed from
the first decode to the last recorded site, plus the job's CSV write (`value`; the rate up to the
last site alone is `value_excluding_csv`).  A warm-up job (pipeline construction, graph capture)
runs first; the timed job's FOV/s is printed as one JSON line.

  python tools/plate_bench.py [--fovs 96] [--repeat 1] [--threads 16] [--batch 48] [--pipes 2]

--repeat R lists the timed job's FOV files R times (R x --fovs LoadData rows, distinct
ImageNumbers, every file decoded again each time): a steady-state run of many batches without
R x the TIFFs on disk."""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))
# as `python -m cpx.plate` runs: at least eight hardware queues (cpx/plate.py's PLATE_HW_QUEUES),
# set before this process first uses the GPU
_hwq = int(os.environ.get("CPX_PLATE_HW_QUEUES", "8"))
if int(os.environ.get("GPU_MAX_HW_QUEUES") or 4) < _hwq:
    os.environ["GPU_MAX_HW_QUEUES"] = str(_hwq)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fovs", type=int, default=96)
    ap.add_argument("--warm", type=int, default=48)
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--batch", type=int, default=48)
    ap.add_argument("--pipes", type=int, default=2)
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()
    import numpy as np
    import pandas as pd
    import torch
    from cpx import plate, shard, tiffio
    from cpx.synth import synth_fovs, synth_illum
    chans = ["DNA", "ER", "RNA", "AGP", "Mito"]
    C, H, W = 5, 2080, 2080
    root = tempfile.mkdtemp(prefix="cpx_platebench_", dir=a.dir)
    try:
        img, ill = os.path.join(root, "images"), os.path.join(root, "illum")
        os.makedirs(img)
        os.makedirs(ill)
        illum = synth_illum(C, H, W, seed=1)
        for c, ch in enumerate(chans):
            np.save(os.path.join(ill, f"{ch}_illum.npy"), illum[c])
        wells = shard.plate_wells(384)
        lds = []
        t0 = time.perf_counter()
        for job, n in (("warm", a.warm), ("timed", a.fovs)):
            rows = []
            for i0 in range(0, n, 16):
                k = min(16, n - i0)
                raw = synth_fovs(k, C, H, W, "cuda", seed=1000 * len(lds) + i0).cpu().numpy().view(np.uint16)
                for j in range(k):
                    f = i0 + j
                    row = {"Metadata_Plate": "P01", "Metadata_Well": wells[f % 384], "Metadata_Site": 1,
                           "Metadata_Timepoint": 24 if job == "timed" else 6}
                    for c, ch in enumerate(chans):
                        name = f"{job}_f{f}_c{c}.tiff"
                        tiffio.imwrite(os.path.join(img, name), raw[j * C + c])
                        row[f"FileName_{ch}"] = name
                    rows.append(row)
            if job == "timed" and a.repeat > 1:
                rows = [dict(r, Metadata_Well=wells[(i * n + f) % 384], Metadata_Site=1 + (i * n + f) // 384)
                        for i in range(a.repeat) for f, r in enumerate(rows)]
            ld = os.path.join(root, f"ld_{job}.csv")
            pd.DataFrame(rows).to_csv(ld, index=False)
            lds.append(ld)
        gen_s = time.perf_counter() - t0
        torch.cuda.synchronize()
        plate.run(["--load-data", *lds, "--data-path", img, "--illum-path", ill, "--channels", *chans,
                   "--out", os.path.join(root, "out"), "--batch", str(a.batch), "--threads", str(a.threads),
                   "--pipes", str(a.pipes)])
        t = [x for x in plate.LAST_TIMING if x["job"] == "ld_timed.csv"][0]
        tif_bytes = a.repeat * sum(os.path.getsize(os.path.join(img, f)) for f in os.listdir(img) if f.startswith("timed"))
        csv_s = t.get("tables_write_s", 0.0)
        print(json.dumps({"metric": "I/O-inclusive FOV/s (cpx.plate on uncompressed TIFFs, local disk, CSVs written)",
                          "value": round(t["fovs"] / (t["seconds"] + csv_s), 2), "unit": "FOV/s",
                          "value_excluding_csv": round(t["fovs"] / t["seconds"], 2), "csv_write_s": csv_s,
                          "fovs": t["fovs"],
                          "unique_fovs": a.fovs, "repeat": a.repeat,
                          "seconds": round(t["seconds"], 3), "decode_threads": t["threads"], "batch": t["batch"],
                          "pipelines": t["pipes"], "tiff_GB": round(tif_bytes / 1e9, 3),
                          "tiff_decode_GBs": round(tif_bytes / 1e9 / t["seconds"], 2),
                          "cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
                          "generation_s": round(gen_s, 1),
                          # where the time goes (cpx.plate._run_sites): main-thread waits on the TIFF
                          # decode threads and on fetch (GPU + D2H), the decode threads' own seconds,
                          # table assembly, and the GPU time of the uploads and of the pipeline steps
                          "split": {k: t[k] for k in ("decode_wait_s", "decode_thread_s", "fetch_wait_s",
                                                      "tables_s", "h2d_gpu_ms", "pipeline_gpu_ms")}}),
              flush=True)
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
