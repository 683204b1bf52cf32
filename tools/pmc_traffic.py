"""HBM traffic per pipeline step from rocprofv3 PMC counter passes over bench.py.

Two separate passes (MI355X_MICROARCH.md "rocprofv3 PMC slots": FETCH_SIZE and WRITE_SIZE do
not fit one pass), each `rocprofv3 --pmc <counter> -- python bench.py ...`.  One pipeline step =
the dispatches between two consecutive k_illum_correct launches (every step starts with it);
the last complete step is used.  gfx950 correction (MI355X_MICROARCH.md "HBM"): FETCH_SIZE
reports half the bytes of wide coalesced reads -> doubled; WRITE_SIZE is taken as is.  Both are
in KB (rocprofv3 units) -> bytes.

  python tools/pmc_traffic.py FETCH_DIR WRITE_DIR --out profiles/pmc_r01.json
where *_DIR hold the run_counter_collection.csv of each pass.
"""
import argparse
import collections
import csv
import glob
import json
import os


FAMILIES = [
    ("illum", ("k_illum_correct", "k_illum_finish")),
    ("qc_rps", ("k_qc_",)),
    ("seg_prep", ("k_pct_", "k_seg_tiles")),
    ("cpnet", ("k_conv3x3", "k_conv_x3", "k_cpnet_", "igemm", "SubTensorOp", "Cijk", "at::native", "native::",
               "elementwise", "reduce_kernel", "naive_conv")),
    ("seg_post", ("k_seg_average", "k_dyn_", "k_seed_", "k_assign", "k_relabel", "k_flow_error",
                  "k_apply_bad", "k_count_bad", "k_upsample", "k_lab2idx", "k_fill_")),
    ("cells", ("k_edt_", "k_ws_")),
    ("features", ("k_stats_init", "k_label_stats", "k_objects_finalize",
                  "k_crop_offsets", "k_obj_stage", "k_shape", "k_tex_", "k_intensity_texture", "k_crops")),
]


def family(name):
    for fam, keys in FAMILIES:
        if any(k in name for k in keys):
            return fam
    return "other"


def load(d, counter):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not path:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = [r for r in csv.DictReader(open(path[0])) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    starts = [i for i, r in enumerate(rows) if "k_illum_correct" in r["Kernel_Name"]]
    if len(starts) < 2:
        raise SystemExit(f"{counter}: fewer than two pipeline steps in {path[0]}")
    step = rows[starts[-2]:starts[-1]]
    per_kernel = collections.defaultdict(float)
    per_fam = collections.defaultdict(float)
    for r in step:
        v = float(r["Counter_Value"]) * 1024.0  # KB -> bytes
        short = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        short = short.replace("void ", "")[:80]
        per_kernel[short] += v
        per_fam[family(r["Kernel_Name"])] += v
    return per_kernel, per_fam, len(step)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--out", required=True)
    ap.add_argument("--batch", type=int, default=32, help="FOVs per bench step (bench.py --batch)")
    ap.add_argument("--precision", default="f16x3", help="bench.py --cpnet-precision of the passes")
    a = ap.parse_args()
    fk, ff, n1 = load(a.fetch_dir, "FETCH_SIZE")
    wk, wf, n2 = load(a.write_dir, "WRITE_SIZE")
    fams = sorted(set(ff) | set(wf))
    out = {
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over bench.py; "
                  "one step = dispatches between consecutive k_illum_correct launches; "
                  "bytes = 2 x FETCH_SIZE (gfx950 wide-read correction) + WRITE_SIZE, KB x 1024",
        "fovs_per_step": a.batch,
        "cpnet_precision": a.precision,
        "dispatches_per_step": [n1, n2],
        "per_family_bytes_per_step": {f: {"read": 2.0 * ff.get(f, 0.0), "write": wf.get(f, 0.0),
                                          "total": 2.0 * ff.get(f, 0.0) + wf.get(f, 0.0)} for f in fams},
        "top_kernels_bytes_per_step": dict(sorted(
            ((k, 2.0 * fk.get(k, 0.0) + wk.get(k, 0.0)) for k in set(fk) | set(wk)),
            key=lambda kv: -kv[1])[:25]),
    }
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for f, v in out["per_family_bytes_per_step"].items():
        print(f"{f:18s} read {v['read'] / 1e9:8.3f} GB  write {v['write'] / 1e9:8.3f} GB per step")


if __name__ == "__main__":
    main()
