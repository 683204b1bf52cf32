"""Development: fraction of wall time during which at least one kernel runs (union of kernel
intervals) in the timed region of a rocprofv3 kernel trace, and the overlap factor
(sum of kernel durations / union)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
# timed region: the last 60 % of the trace (after warmup / setup)
t0 = iv[int(len(iv) * 0.4)][0]
t1 = max(e for _, e in iv)
iv = [(max(s, t0), e) for s, e in iv if e > t0]
union = 0
cur_s, cur_e = None, None
for s, e in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            union += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
total = t1 - t0
busy = sum(e - s for s, e in iv)
print(f"window {total / 1e6:.1f} ms: GPU busy {union / total * 100:.1f} %, kernel-time / busy-time {busy / union:.2f}")

# busiest 100-ms windows (the timed steps), union coverage per window
def coverage(a, b):
    u, cs, ce = 0, None, None
    for s, e in iv:
        s, e = max(s, a), min(e, b)
        if e <= s:
            continue
        if ce is None or s > ce:
            if ce is not None:
                u += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        u += ce - cs
    return u / (b - a)
W = 100_000_000
covs = [coverage(t, t + W) for t in range(t0, t1 - W, W // 4)]
covs.sort()
print(f"100-ms windows: max coverage {covs[-1] * 100:.1f} %, 90th pct {covs[int(len(covs) * 0.9)] * 100:.1f} %")
