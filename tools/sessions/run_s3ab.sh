#!/bin/bash
# Split-form span A/B (under gpurun): parity of the most different variant,
# then tools/ab_probe.sh over AB_ORDER (`make s3ab` first).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp tulips_amd/libtulips_csum.so gpurun_out/lib_product.so
cp tools/ab_s3c32w512.so tulips_amd/libtulips_csum.so
timeout -k 10 300 python -u -m pytest tests/test_span.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/s3ab_test.log 2>&1; rc=$?
tail -2 gpurun_out/s3ab_test.log
[ $rc -ne 0 ] && exit $rc
AB_ORDER="${AB_ORDER:-s3c8w1024 s3c32w1024 s3c8w512 s3c32w512 s3c8w1024 s3c32w1024 s3c8w512 s3c32w512}" PROBE_SIZES=${PROBE_SIZES:-65536,98304} PROBE_GEOMS=${PROBE_GEOMS:-split6,s3_7} bash tools/ab_probe.sh
