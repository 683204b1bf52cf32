# Round-4 evidence pass: the default bench line, kernel traces, PMC traffic / MFMA passes
# (tools/profile_round.sh -> gpurun_out/round/) and the I/O-inclusive plate bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/profile_round.sh
timeout -k 10 500 python -u tools/plate_bench.py --fovs 192 --warm 48 --threads 16 > gpurun_out/round/plate_bench.log 2>&1
echo done
