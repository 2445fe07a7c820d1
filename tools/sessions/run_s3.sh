#!/bin/bash
# Split-form span kernel session (under gpurun): the arena parity suite, then
# the s3 stride A/B probe (tools/ab_probe.sh; `make s3ab` first).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_span.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/s3_test.log 2>&1; rc=$?
tail -5 gpurun_out/s3_test.log
[ $rc -ne 0 ] && exit $rc
AB_ORDER="${AB_ORDER:-s3s1 s3s16 s3s1 s3s16}" PROBE_SIZES=${PROBE_SIZES:-65536,98304} PROBE_GEOMS=${PROBE_GEOMS:-span8,s3_4,s3_5,s3_6,s3_7,s3_8} bash tools/ab_probe.sh
