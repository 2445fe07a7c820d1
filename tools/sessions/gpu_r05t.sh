# round-5 session t: planned segmentation A/B - the tree's kernel (one tile per
# block, window then data) against the persistent prefetching form
# (segment_planned_pf_kernel, -DTCS_SEG_PREFETCH=k: grid = k x the resident
# blocks, the next tile's window loaded under the current tile's build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05t
mkdir -p $O
ROUNDS=4 LIB_B=ab/abx_seg_pf1.so,ab/abx_seg_pf2.so timeout -k 10 300 python -u tools/probe_segment_planned.py > $O/seg_ab_pf.log 2>&1
rc=$?; tail -2 $O/seg_ab_pf.log; exit $rc
