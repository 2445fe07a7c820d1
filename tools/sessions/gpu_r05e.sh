# round-5 session e: planned segmentation A/B, the unconditional trailing barrier
# (ab/abx_seg_bar.so, -DTCS_SEG_LAST_BARRIER) against the in-tree form that skips it when no tile follows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05e
mkdir -p $O
ROUNDS=4 LIB_B=ab/abx_seg_bar.so timeout -k 10 300 python -u tools/probe_segment_planned.py > $O/seg_ab_bar.log 2>&1
rc=$?; tail -2 $O/seg_ab_bar.log; exit $rc
