# round-5 session r: planned segmentation A/B (r05r: 16x6 vs 32x3 vs 32x3 at 6 waves;
# r05r2: a diagnostic build that derives each segment's frame arithmetically,
# no metadata loads or barrier: the cost of the frame search).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05r
mkdir -p $O
ROUNDS=4 LIB_B=ab/abx_seg_nometa.so timeout -k 10 300 python -u tools/probe_segment_planned.py > $O/seg_ab_nometa.log 2>&1
rc=$?; tail -2 $O/seg_ab_nometa.log; exit $rc
