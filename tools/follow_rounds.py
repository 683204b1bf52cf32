"""Development: per-round durations of the flow-following launches (k_dyn_follow, one launch per
round of K steps) in a rocprofv3 kernel trace: the launches are taken in dispatch order in
groups of `--rounds` (one cpx_seg_masks call each) and the mean duration of each round index is
printed, with the mean of the other kernels of one call for scale.

  python tools/follow_rounds.py run_kernel_trace.csv [--rounds 31] [--skip 2]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--rounds", type=int, default=31)
    ap.add_argument("--skip", type=int, default=2, help="calls to skip (warm-up)")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if "k_dyn_follow" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r.get("Correlation_Id") or r.get("Dispatch_Id") or r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    calls = [durs[i:i + a.rounds] for i in range(0, len(durs) - a.rounds + 1, a.rounds)][a.skip:]
    if not calls:
        print("no complete calls")
        return
    tot = 0.0
    for k in range(a.rounds):
        m = sum(c[k] for c in calls) / len(calls)
        tot += m
        print(f"round {k:2d}: {m:8.1f} us")
    print(f"per call: {tot:.1f} us over {len(calls)} calls")


if __name__ == "__main__":
    main()
