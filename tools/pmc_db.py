"""Print per-kernel PMC counter averages (and kernel-trace durations) from rocprofv3 run_results.db
files (rocpd SQLite output).

python tools/pmc_db.py DIR [DIR ...] [--filter k_conv]
"""
import argparse
import collections
import glob
import os
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    for d in a.dirs:
        for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
            con = sqlite3.connect(db)
            try:
                rows = con.execute("select kernel_name, counter_name, value, dispatch_id from counters_collection").fetchall()
            except sqlite3.OperationalError:
                rows = []
            acc = collections.defaultdict(list)
            for k, c, v, did in rows:
                if a.filter in k:
                    acc[(k.split("(")[0][:70], c)].append(v)
            for (k, c), vs in sorted(acc.items()):
                print(f"{db}: {k:70s} {c:28s} n={len(vs):3d} avg={sum(vs) / len(vs):.4g}")
            try:
                kr = con.execute("select name, avg(duration), count(*) from (select kernel_name as name, end - start as duration from kernels) group by name").fetchall()
            except sqlite3.OperationalError:
                kr = []
            for name, dur, cnt in kr:
                if a.filter in name and not rows:
                    print(f"{db}: {name.split('(')[0][:70]:70s} avg {dur / 1e3:.1f} us x{cnt}")


if __name__ == "__main__":
    main()
