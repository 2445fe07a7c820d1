#!/bin/bash
# r06m: the library's allocations and frees made in relaxed capture mode (a
# first call beside another thread's global-mode capture), checked by the new
# graph-lifetime test, then the stream-state, segmentation and native tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06m
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    tests/test_graph_lifetime.py tests/test_stream_state.py tests/test_segment.py \
    tests/test_native_runtime.py > gpurun_out/r06m/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06m/pytest.log | tail -14; exit $rc
