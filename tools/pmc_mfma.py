"""MFMA utilisation of the CPnet kernels from one rocprofv3 counter pass over bench.py.

  rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -- python bench.py ...
  python tools/pmc_mfma.py DIR --out profiles/r02_pmc_mfma.json

MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts matrix-core cycles summed over the chip
(32 per v_mfma_f32_32x32x16_bf16, 16 per 16x16x32); GRBM_GUI_ACTIVE is summed over the 8 XCDs,
so a dispatch's cycles = GRBM_GUI_ACTIVE / 8 and its MFMA utilisation =
busy / (cycles x 256 CUs x 4 SIMDs).  Aggregated per kernel name over the last complete
pipeline step (dispatches between two consecutive k_illum_correct launches).
"""
import argparse
import collections
import csv
import glob
import json
import os

SIMDS = 256 * 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", required=True)
    ap.add_argument("--match", default="k_conv3x3,k_conv_x3,k_cpnet_,Cijk,igemm",
                    help="comma-separated kernel-name substrings to report")
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)
    if not path:
        raise SystemExit(f"no counter_collection.csv under {a.dir}")
    per = collections.defaultdict(dict)  # dispatch -> {counter: value, name}
    for r in csv.DictReader(open(path[0])):
        d = per[int(r["Dispatch_Id"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["name"] = r["Kernel_Name"]
    ids = sorted(per)
    starts = [i for i in ids if "k_illum_correct" in per[i]["name"]]
    if len(starts) >= 2:
        ids = [i for i in ids if starts[-2] <= i < starts[-1]]
    keys = [k for k in a.match.split(",") if k]
    agg = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for i in ids:
        d = per[i]
        if not any(k in d["name"] for k in keys):
            continue
        short = d["name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:90]
        g = agg[short]
        g[0] += d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        g[1] += d.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        g[2] += 1
    rows = {k: {"dispatches": v[2], "mfma_busy_cycles": v[0], "kernel_cycles": v[1],
                "mfma_util": v[0] / (v[1] * SIMDS) if v[1] else None}
            for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])}
    busy = sum(v[0] for v in agg.values())
    cyc = sum(v[1] for v in agg.values())
    out = {"method": __doc__.strip().splitlines()[0] + " (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE/8)",
           "dispatches_in_step": len(ids),
           "total": {"mfma_busy_cycles": busy, "kernel_cycles": cyc,
                     "mfma_util": busy / (cyc * SIMDS) if cyc else None},
           "per_kernel": rows}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["total"]))


if __name__ == "__main__":
    main()
