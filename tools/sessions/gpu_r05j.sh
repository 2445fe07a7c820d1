# round-5 session j: F9000 subgroup geometry A/B (64 x 12, the round 1-4
# default, against 64 x 9 / 64 x 10, which hold a 9000 B segment in one
# batch with fewer redundant loads, and 64 x 8), then the parity suite of
# every geometry.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05j
mkdir -p $O
ROUNDS=5 PROBE_LENS=9000 PROBE_GEOMS=64:12:256,64:9:256,64:10:256,64:8:256 \
  timeout -k 10 500 python -u tools/probe_fixed.py > $O/fixed9000.log 2>&1 || { tail -5 $O/fixed9000.log; exit 1; }
grep '^{' $O/fixed9000.log
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -m gpu tests/test_gpu_parity.py > $O/parity.log 2>&1; rc=$?; tail -1 $O/parity.log; exit $rc
