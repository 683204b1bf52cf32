# Round 5: rehearsal after the compacted result fetch (each FOV's own rows gathered on the device,
# one contiguous D2H per table): smoke(), the whole -m gpu suite, a bench and its kernel trace.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05aq
mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 60 --stage-steps 1 > $O/bench.log 2>&1
tail -1 $O/bench.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('bench', d['value'], d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt -o run -- \
  python -u bench.py --pipes 1 --steps 6 --warmup 2 --no-cpu-baseline --stage-steps 1 > $O/kt.log 2>&1
python tools/prof_summary.py /tmp/kt/run_kernel_trace.csv --steps 4 --md --series copyBuffer > $O/k.md
python tools/follow_rounds.py /tmp/kt/run_kernel_trace.csv > $O/follow_rounds.txt
rm -rf /tmp/kt
grep -E "copyBuffer|index_select|indexSelect|total|dispatches of one step" $O/k.md
echo done
