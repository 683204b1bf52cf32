"""Per-time profile step throughput on one GPU.

The hot reduction of Pycyto_pertime.py is the per-well mean of the object tables (:69-72):
`objects x features` fp64 values, resident in HBM, reduced with pandas' Kahan group mean
(cpx_group_kahan_accumulate + cpx_group_mean_finalize), timed with HIP events on the launch
stream; algorithmic bytes = 8 B per value + 4 B per row index.  The same table through pandas
`groupby(keys).mean()` (the reference's call, one core) is the CPU baseline, and the whole
per-time step (merge, normalise, feature selection, similarities) is timed for both the GPU
engine and the oracle pipeline on the same in-memory tables.

python tools/profiles_bench.py [--wells 384 --sites 9 --objects 300 --reps 10]
"""
import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cpx.profiles import KEYS, IMAGE_META, ProfileEngine, profile_time  # noqa: E402
from synth_tables import plate_tables  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--wells", type=int, default=384)
    ap.add_argument("--sites", type=int, default=9)
    ap.add_argument("--objects", type=int, default=300)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-pipeline", action="store_true")
    ap.add_argument("--cprofile", default="", help="write a cProfile summary of the GPU pipeline here")
    a = ap.parse_args()
    t0 = time.perf_counter()
    tb = plate_tables(n_wells=a.wells, sites=a.sites, objects=a.objects, n_feat=None, seed=1)
    t_gen = time.perf_counter() - t0
    print(f"# tables generated in {t_gen:.1f} s", flush=True)
    eng = ProfileEngine()
    td = eng.td
    nuc = tb["Nuclei"].merge(tb["Image"][IMAGE_META], on="ImageNumber", how="left")
    nuc = nuc.drop(["ImageNumber", "Metadata_Site", "Metadata_ConcLevel"], axis=1)
    cols = [c for c in nuc.columns if c not in KEYS]
    gb = nuc.groupby(KEYS, sort=True)
    codes = gb.ngroup().to_numpy()
    G = int(codes.max()) + 1
    order = np.argsort(codes, kind="stable").astype(np.int32)
    offs = np.zeros(G + 1, dtype=np.int32)
    np.cumsum(np.bincount(codes, minlength=G), out=offs[1:])
    vals = torch.from_numpy(np.ascontiguousarray(nuc[cols].to_numpy(dtype=np.float64))).to(td)
    o_t = torch.from_numpy(order).to(td)
    f_t = torch.from_numpy(offs).to(td)
    n, K = vals.shape
    sumx = torch.zeros((G, K), dtype=torch.float64, device=td)
    comp, nobs = torch.zeros_like(sumx), torch.zeros((G, K), dtype=torch.int64, device=td)
    out = torch.empty_like(sumx)

    def step():
        sumx.zero_(); comp.zero_(); nobs.zero_()
        eng.dev.group_kahan(vals, o_t, f_t, sumx, comp, nobs)
        eng.dev.group_finalize(sumx, nobs, out)
    step()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream(td)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.reps):
        step()
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    print(f"# gpu group mean {ms:.3f} ms", flush=True)
    byt = n * K * 8 + n * 4 + 3 * G * K * 8
    # CPU baseline: the reference's pandas call on the same table (one core)
    t0 = time.perf_counter()
    ref = nuc.groupby(KEYS, as_index=False).mean(numeric_only=True)
    t_pd = time.perf_counter() - t0
    exact = bool(np.array_equal(out.cpu().numpy(), ref[cols].to_numpy(), equal_nan=True))
    res = {"workload": f"per-well mean of one object table: {n} objects x {K} columns, {G} wells",
           "gpu_ms": round(ms, 4), "objects_per_s": round(n / ms * 1e3), "achieved_GBs": round(byt / ms / 1e6, 1),
           "hbm_frac": round(byt / ms / 1e6 / 8000.0, 4), "bit_exact_vs_pandas": exact,
           "cpu_pandas_ms": round(t_pd * 1e3, 1), "cpu_cores": 1, "table_gen_s": round(t_gen, 1)}
    if not a.no_pipeline:
        import profiles_oracle as po
        print("# pipelines", flush=True)
        with tempfile.TemporaryDirectory() as d:
            args = (tb["Image"], tb["Nuclei"], tb["Cells"], tb["Cytoplasm"], "Plate_1", "T1")
            t0 = time.perf_counter()
            if a.cprofile:
                import cProfile
                import pstats
                pr = cProfile.Profile()
                pr.enable()
            profile_time(eng, *args, os.path.join(d, "g.csv"))
            t_g = time.perf_counter() - t0
            if a.cprofile:
                pr.disable()
                with open(a.cprofile, "w") as f:
                    pstats.Stats(pr, stream=f).sort_stats("cumulative").print_stats(40)
            t0 = time.perf_counter()
            po.pycyto_pertime(*args, os.path.join(d, "c.csv"))
            t_c = time.perf_counter() - t0
        res["pipeline_s"] = {"gpu_engine": round(t_g, 2), "cpu_oracle": round(t_c, 2),
                             "note": "same in-memory tables, host pandas plumbing included"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
