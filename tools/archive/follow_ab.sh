#!/bin/bash
# Development A/B of the segmentation post-processing (tools/follow_bench.py): the in-tree
# libcpx vs tools/_var variants named on the command line, plus a kernel trace of the default
# build with the per-round k_dyn_follow durations.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/follow
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/follow_bench.py > $O/default.log 2>&1
for v in "$@"; do
  CPX_LIB=$R/tools/_var/libcpx_$v.so timeout -k 10 200 python -u tools/follow_bench.py > $O/$v.log 2>&1
done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python -u tools/follow_bench.py > $O/kt.log 2>&1
python - $O/kt/run_kernel_trace.csv > $O/rounds.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_dyn_follow" in r["Kernel_Name"]]
print("k_dyn_follow dispatches (us), last 31:", " ".join(f"{d:.0f}" for d in ds[-31:]), "sum", f"{sum(ds[-31:]):.0f}")
PY
rm -rf $O/kt
echo done
