# round-5 session h: F1500 subgroup geometry A/B, 32 lanes x 3 chunks (96
# chunks: a 1500 B segment at any alignment in one batch, no redundant
# loads) against the default 32 x 4 and 32 x 4 / 512; serial chains of 256
# launches over the 16 rotated batches, median of 3 replays, 5 rounds; then
# the geometry parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05h
mkdir -p $O
ROUNDS=5 PROBE_LENS=1500 PROBE_GEOMS=32:4:256,32:3:256,32:3:512 timeout -k 10 300 python -u tools/probe_fixed.py > $O/fixed.log 2>&1 || { tail -5 $O/fixed.log; exit 1; }
cat $O/fixed.log | grep '^{'
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/parity.log 2>&1; rc=$?; tail -2 $O/parity.log; exit $rc
