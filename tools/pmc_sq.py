"""Per-kernel summary of a rocprofv3 --pmc counter_collection.csv (any counters): sum of each
counter over the dispatches of each kernel (name prefix), plus dispatch counts.

  python tools/pmc_sq.py DIR [--match k_flow_error,k_dyn_follow]"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)
    if not path:
        raise SystemExit(f"no counter_collection.csv under {a.dir}")
    keys = [k for k in a.match.split(",") if k]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path[0])):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:60]
        if keys and not any(k in name for k in keys):
            continue
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add(r["Dispatch_Id"])
    for name in sorted(acc, key=lambda n: -max(acc[n].values())):
        c = acc[name]
        print(f"{name}  dispatches={len(disp[name])}")
        for k in sorted(c):
            print(f"    {k:28s} {c[k]:.4g}")
        if "SQ_WAVE_CYCLES" in c and "SQ_ACTIVE_INST_VALU" in c:
            print(f"    VALU-active / wave-cycles = {c['SQ_ACTIVE_INST_VALU'] / c['SQ_WAVE_CYCLES']:.3f}")
        if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_INST_ANY" in c:
            print(f"    wait-inst / wave-cycles   = {c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']:.3f}")
        if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_ANY" in c:
            print(f"    wait-any / wave-cycles    = {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f}")


if __name__ == "__main__":
    main()
