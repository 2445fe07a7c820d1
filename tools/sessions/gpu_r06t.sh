#!/bin/bash
# r06t: the native capture-neutrality check on /opt/rocm 7.2 and the native
# suite beside it.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06t
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_native_runtime.py > gpurun_out/r06t/pytest.log 2>&1
rc=$?; grep -E "capture_neutral|PASSED|FAILED|passed|failed" gpurun_out/r06t/pytest.log | tail -14; exit $rc
