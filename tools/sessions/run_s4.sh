#!/bin/bash
# Span form comparison session (under gpurun): the arena parity suite, then
# tools/probe_gen.py over the split forms (twice).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_span.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/s4_test.log 2>&1; rc=$?
tail -3 gpurun_out/s4_test.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  PROBE_PIPE=1 PROBE_SIZES=${PROBE_SIZES:-1024,65536,98304} PROBE_GEOMS=${PROBE_GEOMS:-split6,s4_5,s4_6,s4_7,s4_8} timeout -k 10 300 python -u tools/probe_gen.py > gpurun_out/s4_probe_$rep.log 2>&1 || exit 1
  grep '^{' gpurun_out/s4_probe_$rep.log
done
