#!/bin/bash
# r06aa: every offset-taking entry point on a 4.5 GiB arena with its inputs
# past the 4 GiB line (tests/test_large.py).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06aa
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_large.py > gpurun_out/r06aa/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|assert|passed|failed" gpurun_out/r06aa/pytest.log | tail -20; exit $rc
