# Development GPU pass: the whole -m gpu suite (as the driver runs it), then a short bench line.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/full
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 12 > $O/bench.log 2>&1
echo done
