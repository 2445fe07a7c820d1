# round-5 session a: the new / changed GPU tests (captured segmentation,
# RSS router on alternating streams), the driver's bench command, then the
# whole GPU suite and smoke. Every step has its own limit; the first failure
# ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05a
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step new 420 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
  tests/test_segment.py tests/test_stream_state.py tests/test_multi.py tests/test_gpucsum_device.py
step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step suite 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests
step smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()"
