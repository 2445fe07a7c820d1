# round-5 session b: the decorator / segmentation / drop-in GPU tests, the
# driver's bench command, the whole GPU suite, smoke, then the ZIPF
# priority A/B (tools/probe_span_prio.py). Every step has its own
# limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05b
mkdir -p $O
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step new 420 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpucsum_device.py tests/test_segment.py tests/test_dropin.py tests/test_span.py tests/test_multi.py tests/test_frames.py::test_frames_tuned_rejects_bad_geometry
step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step suite 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests
step smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()"
step span_prio 300 python -u tools/probe_span_prio.py
