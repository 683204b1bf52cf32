"""Development: for the dispatches of one kernel longer than a threshold in a rocprofv3 kernel
trace, print the stream, grid / workgroup sizes and the kernels dispatched just before and after
it on the same stream (to find where a copy or a slow launch comes from).

  python tools/trace_neighbors.py run_kernel_trace.csv --match copyBuffer --min-us 500 [--last 3]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", required=True)
    ap.add_argument("--min-us", type=float, default=500.0)
    ap.add_argument("--last", type=int, default=3)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    scol = next((c for c in ("Stream_Id", "Queue_Id") if c in rows[0]), None)
    hits = [i for i, r in enumerate(rows) if a.match in r["Kernel_Name"]
            and (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 >= a.min_us]
    for i in hits[-a.last:]:
        r = rows[i]
        sid = r.get(scol) if scol else None
        same = [j for j in range(len(rows)) if not scol or rows[j].get(scol) == sid]
        k = same.index(i)
        def nm(j):
            return rows[j]["Kernel_Name"].split("(")[0][:60]
        prev = [nm(j) for j in same[max(0, k - 3):k]]
        nxt = [nm(j) for j in same[k + 1:k + 4]]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        grid = [r.get(c) for c in ("Grid_Size_X", "Grid_Size", "Workgroup_Size_X", "Workgroup_Size") if c in r]
        print(f"{nm(i)} {dur:.0f} us {scol}={sid} grid/wg={grid}")
        print(f"   before: {prev}")
        print(f"   after:  {nxt}")


if __name__ == "__main__":
    main()
