"""Steady-state kernel summary from a rocprofv3 kernel-trace CSV of bench.py.

Keeps only the dispatches of the last `--steps` pipeline steps (a step starts at each
`k_illum_correct` launch) so MIOpen find / warm-up kernels are excluded, then aggregates by
kernel name.  Usage: python tools/prof_summary.py <run_kernel_trace.csv> [--steps 4] [--md]
"""
import argparse
import csv
import collections


def short(n):
    if "anonymous namespace)::" in n:
        n = n.split("::", 1)[1]
    return n.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--md", action="store_true")
    ap.add_argument("--top", type=int, default=40, help="kernels listed (by time per step)")
    ap.add_argument("--series", default=None,
                    help="also list the per-dispatch durations (us) of this kernel in the last step")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_illum_correct" in r["Kernel_Name"]]
    if len(starts) < a.steps + 1:
        sel = rows
    else:
        # the bench's instrumented steps launch illum outside run(); use the steps before them
        sel = rows[starts[-a.steps - 1]: starts[-1]]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = short(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += d
    tot = sum(v[1] for v in agg.values())
    n_steps = a.steps
    items = sorted(agg.items(), key=lambda kv: -kv[1][1])
    if a.md:
        print("| kernel | calls/step | avg us | us/step | % |")
        print("|---|---:|---:|---:|---:|")
    for k, (c, t) in items[:a.top]:
        if a.md:
            print(f"| `{k}` | {c / n_steps:.1f} | {t / c:.1f} | {t / n_steps:.1f} | {100 * t / tot:.1f} |")
        else:
            print(f"{k:70s} calls/step={c / n_steps:6.1f} avg_us={t / c:9.1f} us/step={t / n_steps:9.1f} {100 * t / tot:5.1f}%")
    print(f"total kernel time per step: {tot / n_steps / 1e3:.3f} ms over {len(sel)} dispatches")
    if a.series and len(starts) >= 2:
        last = rows[starts[-2]: starts[-1]]
        ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
              for r in last if a.series in r["Kernel_Name"]]
        print(f"\n`{a.series}` dispatches of one step (us): " + " ".join(f"{d:.0f}" for d in ds))


if __name__ == "__main__":
    main()
