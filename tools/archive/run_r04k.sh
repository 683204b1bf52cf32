# Feature fallback tail: objects per FOV that go to the fallback kernels, and cpx_features time
# with more fallback blocks per FOV (CPX_FB_PER_FOV).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04k
mkdir -p $O
cd $R
for fb in 0 40 0 40 100; do
  CPX_FB_PER_FOV=$fb timeout -k 10 300 python -u tools/tex_bench.py --batch 48 --reps 7 > $O/tex_$fb.log 2>&1
  grep "features\[" $O/tex_$fb.log | sed "s/^/fb $fb /"
done
grep "fallback" $O/tex_0.log
echo done
