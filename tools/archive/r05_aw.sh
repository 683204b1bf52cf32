# Round 5: probe — CU-masked streams under rocprofv3 (the two-pipeline trace of the final profile
# pass segfaulted once they became the default).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05aw
mkdir -p $O
cd $R
timeout -k 10 120 python -u tools/probe/cu_mask_prof.py halves > $O/plain.log 2>&1; echo "plain rc=$?"; tail -3 $O/plain.log
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d /tmp/pp -o run -- python -u tools/probe/cu_mask_prof.py none > $O/prof_none.log 2>&1; echo "prof none rc=$?"; grep -E "^ok|^env|^streams" $O/prof_none.log
rm -rf /tmp/pp
echo done
