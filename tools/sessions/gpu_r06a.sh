#!/bin/bash
# r06a: graph ownership by user objects and the native
# runtime checker (next #3), first contact.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06a
timeout -k 10 60 tests/native/_build/runtime_check user-object > gpurun_out/r06a/uo_native.json 2>&1 &&
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread \
    tests/test_graph_lifetime.py tests/test_native_runtime.py tests/test_stream_state.py \
    "tests/test_fuzz.py::test_fuzz_captured_graphs" > gpurun_out/r06a/pytest.log 2>&1
rc=$?
tail -30 gpurun_out/r06a/pytest.log
exit $rc
