#!/bin/bash
# A/B of library builds on one box: ab_libs/lib_<name>.so for each name in
# $LIBS is copied over tulips_amd/libtulips_csum.so in turn and $PROBE runs
# in a fresh process, $ROUNDS alternations; the tree's own build is put back
# at the end. First the frame/segment GPU tests on the tree's build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
export TMPDIR=/tmp
LIB=tulips_amd/libtulips_csum.so
cp $LIB /tmp/lib_tree.so
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -q -x -m gpu -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "STOP pytest rc=$rc"; exit $rc; }
fi
for r in $(seq 1 ${ROUNDS:-3}); do
  for name in $LIBS; do
    cp ab_libs/lib_$name.so $LIB || exit 1
    timeout -k 10 ${PROBE_TIMEOUT:-180} python -u $PROBE > $OUT/${name}_$r.log 2>&1
    rc=$?
    echo "$r $name $(tail -1 $OUT/${name}_$r.log)"
    [ $rc -eq 0 ] || { cp /tmp/lib_tree.so $LIB; echo "STOP probe rc=$rc"; exit $rc; }
  done
done
cp /tmp/lib_tree.so $LIB
