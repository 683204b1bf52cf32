"""Development: list the runtime copy/fill kernels of one bench step with their neighbours
(from a rocprofv3 kernel_trace.csv), to find where device copies come from."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# one step: between the last two k_illum_correct launches
ill = [i for i, r in enumerate(rows) if "k_illum_correct" in r["Kernel_Name"]]
a, b = ill[-2], ill[-1]
for i in range(a, b):
    r = rows[i]
    n = r["Kernel_Name"]
    if "rocclr" in n:
        prev = rows[i - 1]["Kernel_Name"][:50]
        nxt = rows[i + 1]["Kernel_Name"][:50]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print(f"{n[:32]:32s} grid {r.get('Grid_Size', r.get('Grid_Size_X', '?')):>10} wg {r.get('Workgroup_Size', '?'):>5} "
              f"{dur:8.1f} us | after {prev} | before {nxt}")
