#!/bin/bash
# r06w: the §8f kernels through the C ABI on /opt/rocm 7.2 against the golden
# fixtures (runtime_check fixtures), with the rest of the native suite.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06w
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_native_runtime.py > gpurun_out/r06w/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|\"ok\": false" gpurun_out/r06w/pytest.log | tail -14; exit $rc
