"""Per-dispatch durations (us) of kernels matching a substring, in launch order, from a
rocprofv3 kernel-trace CSV.  python tools/trace_dispatch.py run_kernel_trace.csv k_ws_ [--last N]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else len(rows)
for r in rows[-last:]:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    print(f"{n:40s} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:10.1f}")
