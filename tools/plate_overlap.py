"""Development: how much the plate CLI's batches overlap on the GPU.  From a rocprofv3 kernel
trace of `tools/plate_bench.py`, over the last `--seconds` of the trace (the timed job, whose
length plate_bench prints), report the union of kernel intervals (GPU busy), the sum of kernel
time over it, the share of time with 0 / 1 / >= 2 kernels running, and the same per HIP queue
or stream column the trace carries.

  python tools/plate_overlap.py run_kernel_trace.csv --seconds 2.1
"""
import argparse
import csv
import collections


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--seconds", type=float, required=True)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    t1 = max(int(r["End_Timestamp"]) for r in rows)
    t0 = t1 - int(a.seconds * 1e9)
    ev = []
    per_q = collections.Counter()
    qcol = next((c for c in ("Stream_Id", "Queue_Id") if c in rows[0]), None)
    ksum = 0
    for r in rows:
        s, e = max(int(r["Start_Timestamp"]), t0), int(r["End_Timestamp"])
        if e <= s:
            continue
        ev.append((s, 1))
        ev.append((e, -1))
        ksum += e - s
        if qcol:
            per_q[r[qcol]] += e - s
    ev.sort()
    level, last = 0, t0
    dur = collections.Counter()
    for t, d in ev:
        dur[min(level, 2)] += t - last
        level += d
        last = t
    dur[0] += t1 - last
    tot = t1 - t0
    busy = dur[1] + dur[2]
    print(f"window {tot / 1e6:.1f} ms: busy {busy / tot * 100:.1f} %, idle {dur[0] / tot * 100:.1f} %, "
          f"one kernel {dur[1] / tot * 100:.1f} %, >= 2 kernels {dur[2] / tot * 100:.1f} %, "
          f"kernel time / busy {ksum / max(busy, 1):.2f}")
    if qcol:
        for q, v in sorted(per_q.items(), key=lambda x: -x[1]):
            print(f"  {qcol} {q}: kernel time {v / 1e6:.1f} ms ({v / tot * 100:.1f} % of the window)")


if __name__ == "__main__":
    main()
