#!/bin/bash
# Session q: frame and multi-device GPU tests on the tree build (flag bytes gathered in LDS), then A/B of the flag store forms: current (byte per subgroup), LDS-gathered per workgroup, nontemporal byte stores; then the no-store diagnostic (timing only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_frames.py tests/test_multi.py -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/q_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/q_pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=r04q LIBS="cur blk ntstore" ROUNDS=3 PROBE_OPS=validate PROBE=tools/probe_frames_ops.py timeout -k 10 500 bash tools/ab_libs.sh || exit 1
TAG=r04q2 LIBS="cur nostore" ROUNDS=2 PROBE_OPS=validate NOCHECK=1 PROBE=tools/probe_frames_ops.py timeout -k 10 300 bash tools/ab_libs.sh
