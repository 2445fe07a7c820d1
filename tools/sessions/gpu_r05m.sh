# round-5 session m: frame kernel geometry A/B, 32 lanes x 3 chunks (96
# chunks, 62 VGPRs, 8 waves/SIMD) against the 16 x 6 default (78 VGPRs, 6
# waves) and 32 x 4, validate / generate / compact fields, serial chains of
# 128 launches over 8 rotated bursts, median of 3 replays, 5 rounds; then the
# frame tests (every geometry against the oracle and the reference fixtures).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05m
mkdir -p $O
ROUNDS=5 PROBE_NT=1 PROBE_GEOS=16x6,32x3,32x4 timeout -k 10 500 python -u tools/probe_frames.py > $O/frames.log 2>&1 || { tail -5 $O/frames.log; exit 1; }
grep '^{' $O/frames.log
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -m gpu tests/test_frames.py > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; exit $rc
