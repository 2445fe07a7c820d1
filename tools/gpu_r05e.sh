# round-5 session e: planned segmentation A/B, the wave-independent kernel
# (ab/abx_seg_wave.so, -DTCS_PLANNED_WAVE) against the in-tree block form.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05e
mkdir -p $O
ROUNDS=4 LIB_B=ab/abx_seg_wave.so timeout -k 10 300 python -u tools/probe_segment_planned.py > $O/seg_ab_wave.log 2>&1
rc=$?; tail -2 $O/seg_ab_wave.log; exit $rc
