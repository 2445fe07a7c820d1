# round-5 session d: planned segmentation A/B, nontemporal payload loads
# (ab/abx_seg_nt.so) against the in-tree build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05d
mkdir -p $O
ROUNDS=4 LIB_B=ab/abx_seg_nt.so timeout -k 10 300 python -u tools/probe_segment_planned.py > $O/seg_ab_nt.log 2>&1
rc=$?; tail -2 $O/seg_ab_nt.log; exit $rc
