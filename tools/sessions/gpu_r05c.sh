# round-5 session c: planned segmentation A/B (window-start fix against the
# previous build, ab/abx_seg_prev.so) and its tests, then the driver's
# bench command. Every step has its own limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05c
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step seg_tests 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_segment.py tests/test_gpucsum_device.py tests/test_dropin.py
LIB_B=ab/abx_seg_prev.so step seg_ab 300 python -u tools/probe_segment_planned.py
step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
