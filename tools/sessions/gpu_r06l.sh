#!/bin/bash
# r06l: the graph-lifetime and native-runtime tests as pytest runs them.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06l
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread \
    tests/test_graph_lifetime.py tests/test_native_runtime.py > gpurun_out/r06l/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|SKIPPED|ERROR|passed|failed" gpurun_out/r06l/pytest.log | tail -14; exit $rc
