#!/bin/bash
# r06ab: the IPv4 header's checksum taken from the broadcast header words
# (frames.hip TULIPS_FRAME_IP_FROM_HEADER: no range sum and no subgroup
# reduction for it) against the product build. First the frame tests on the
# variant (every alignment, generation, fields, the golden flags), then the
# frame ops alternated 3 times (probe_gen_defer.py: validate / generate /
# fields, serial and 4-branch, arena regenerated and checked).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06ab
mkdir -p $OUT
LIB=tulips_amd/libtulips_csum.so
cp $LIB /tmp/lib_tree.so
cp ab_libs/lib_iphdr.so $LIB
timeout -k 10 400 python -u -m pytest tests/test_frames.py -q -m gpu -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $OUT/pytest_iphdr.log 2>&1
rc=$?
cp /tmp/lib_tree.so $LIB
tail -2 $OUT/pytest_iphdr.log
[ $rc -eq 0 ] || { echo "STOP: frame tests on the variant rc=$rc"; exit $rc; }
TAG=r06ab LIBS="base iphdr" ROUNDS=3 PROBE=tools/sessions/probes/probe_gen_defer.py \
  bash tools/sessions/probes/ab_libs.sh
