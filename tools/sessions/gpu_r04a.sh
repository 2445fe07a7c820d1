# round-4 session a: the new GPU tests first, then the whole GPU suite,
# smoke, the default bench line. Every step under its own time limit; the
# script stops at the first failure.
set -u
O=gpurun_out/r04a
mkdir -p $O
run() { # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  tail -4 $O/$name.log
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; exit $rc; fi
}
run new 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_frames.py::test_gpu_zero_copy_tag_wraparound tests/test_frames.py::test_gpu_zero_copy_pinned_range_reused \
  tests/test_multi.py::test_mctx_device_staged_copies tests/test_multi.py::test_mctx_rss_fragments_go_to_slot0 \
  tests/test_gpucsum_device.py
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python -u bench.py
cp $O/bench.log $O/bench.json
run suite 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests
