#!/bin/bash
# r06y: graph ownership across six host threads on /opt/rocm 7.2
# (runtime_check thread-churn), with the rest of the native suite.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06y
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_native_runtime.py > gpurun_out/r06y/pytest.log 2>&1
rc=$?; grep -E "thread_churn|\"graphs\"|mismatches|growth|PASSED|FAILED|passed|failed" gpurun_out/r06y/pytest.log | tail -20; exit $rc
