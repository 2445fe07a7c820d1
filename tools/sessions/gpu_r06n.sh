#!/bin/bash
# r06n: the concurrent global-mode capture test alone, full traceback.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06n
timeout -k 10 300 python -u -m pytest -x -v --tb=long --timeout 200 --timeout-method thread -p no:cacheprovider \
    "tests/test_graph_lifetime.py::test_first_calls_beside_a_global_mode_capture_in_another_thread" \
    > gpurun_out/r06n/pytest.log 2>&1
rc=$?; tail -60 gpurun_out/r06n/pytest.log; exit $rc
