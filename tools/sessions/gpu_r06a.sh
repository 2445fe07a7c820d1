#!/bin/bash
# r06a: graph ownership by user objects, the native
# runtime checker (next #3) and the trimmed product ABI (next #4): first
# contact, then smoke and the driver-form bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06a
timeout -k 10 60 tests/native/_build/runtime_check user-object > gpurun_out/r06a/uo_native.json 2>&1 &&
timeout -k 10 1000 python -u -m pytest -v --timeout 600 --timeout-method thread \
    tests/test_graph_lifetime.py tests/test_native_runtime.py tests/test_stream_state.py \
    "tests/test_fuzz.py::test_fuzz_captured_graphs" \
    "tests/test_frames.py::test_gpu_zero_copy_tag_wraparound" \
    "tests/test_segment.py::test_gpu_copy_slots_ceiling_kernel" \
    tests/test_gpu_parity.py > gpurun_out/r06a/pytest.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06a/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/r06a/bench.json 2> gpurun_out/r06a/bench.err
rc=$?
tail -40 gpurun_out/r06a/pytest.log
tail -3 gpurun_out/r06a/smoke.log
tail -c 600 gpurun_out/r06a/bench.json
exit $rc
