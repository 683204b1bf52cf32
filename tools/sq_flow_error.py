"""Per-step SQ_INSTS_VALU of the register flow-error kernels from a rocprofv3 --pmc pass of
bench.py (--pipes 1): writes the JSON bench.py's roofline_all.flow_error_reg reads.

  python tools/sq_flow_error.py DIR --fovs 48 --out profiles/r06_sq_flow_error.json"""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--fovs", type=int, default=48)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)[0]
    valu = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "k_flow_error_reg" not in name or r["Counter_Name"] != "SQ_INSTS_VALU":
            continue
        key = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        valu[key] += float(r["Counter_Value"])
        disp[key].add(r["Dispatch_Id"])
    steps = max(len(v) for v in disp.values())  # one dispatch of each register kernel per step
    out = {"fovs_per_step": a.fovs, "steps": steps, "valu_per_step": sum(valu.values()) / steps,
           "per_kernel": {k: {"valu_per_step": valu[k] / steps, "dispatches": len(disp[k])} for k in valu},
           "source": os.path.relpath(path)}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
