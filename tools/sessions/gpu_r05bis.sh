# round-5 session: bisect the captured-graph replay SIGSEGV by job kind
# (tests/test_fuzz.py::test_fuzz_captured_graphs, TULIPS_FUZZ_KINDS); the
# chain stops at the first kind that crashes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05bis
mkdir -p $O
for k in ${KINDS:-any planned arena verify validate segment}; do
  echo "== $k"
  TULIPS_FUZZ_GRAPH_DESTROY=1 TULIPS_FUZZ_KINDS=$k TULIPS_FUZZ_SECONDS=${SECS:-40} timeout -k 10 120 python -u -m pytest tests/test_fuzz.py -x -q -s -m gpu -k graphs -p no:cacheprovider --timeout 100 --timeout-method thread > $O/$k.log 2>&1
  rc=$?
  echo "   rc=$rc $(grep -h 'fuzz graphs:' $O/$k.log | tail -1)"
  [ $rc -eq 0 ] || exit $rc
done
