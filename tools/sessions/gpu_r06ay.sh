#!/bin/bash
# r06ay: the native-runtime tests after their runner moved to Popen (a stalled
# checker's threads and wait channels are read before it is killed).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06ay
timeout -k 10 500 python -u -m pytest -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    -m gpu tests/test_native_runtime.py > gpurun_out/r06ay/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06ay/pytest.log; exit $rc
