#!/bin/bash
# r06ad: segmentation with the output IPv4 header's sum from the frame's
# header words (segment.hip TULIPS_SEG_IP_FROM_HEADER: no masked sums over
# chunks 0..2 and no subgroup reduction for it) against the product build.
# First the segmentation tests on the variant, then probe_segment_planned.py
# with the variant's planned entry timed beside the product's (its outputs
# compared byte for byte with the product's prologue form after every timed
# replay), 3 rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06ad
mkdir -p $OUT
LIB=tulips_amd/libtulips_csum.so
cp $LIB /tmp/lib_tree.so
cp ab_libs/lib_segip.so $LIB
timeout -k 10 400 python -u -m pytest tests/test_segment.py -q -m gpu -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $OUT/pytest_segip.log 2>&1
rc=$?
cp /tmp/lib_tree.so $LIB
tail -2 $OUT/pytest_segip.log
[ $rc -eq 0 ] || { echo "STOP: segmentation tests on the variant rc=$rc"; exit $rc; }
LIB_B=ab_libs/lib_segip.so ROUNDS=${ROUNDS:-3} timeout -k 10 400 python -u \
  tools/sessions/probes/probe_segment_planned.py > $OUT/probe.log 2>&1
rc=$?; tail -4 $OUT/probe.log; exit $rc
