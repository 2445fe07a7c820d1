#!/bin/bash
# r06ar: the segmentation kernel's TCP sum with 32-bit v_dot2 accumulation
# (segment.hip TULIPS_SEG_L4_DOT2, as the frame kernels since r06al) against
# the product: segmentation tests on the variant, then probe_segment_planned.py
# with the variant's planned entry beside the product's (outputs compared with
# the product's prologue form after every timed replay).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06ar
mkdir -p $OUT
LIB=tulips_amd/libtulips_csum.so
cp $LIB /tmp/lib_tree.so
cp ab_libs/lib_segd2.so $LIB
timeout -k 10 400 python -u -m pytest tests/test_segment.py -q -m gpu -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $OUT/pytest_segd2.log 2>&1
rc=$?
cp /tmp/lib_tree.so $LIB
tail -2 $OUT/pytest_segd2.log
[ $rc -eq 0 ] || { echo "STOP: segmentation tests on the variant rc=$rc"; exit $rc; }
LIB_B=ab_libs/lib_segd2.so ROUNDS=${ROUNDS:-3} timeout -k 10 400 python -u \
  tools/sessions/probes/probe_segment_planned.py > $OUT/probe.log 2>&1
rc=$?; tail -4 $OUT/probe.log; exit $rc
