#!/bin/bash
# r06p: host-buffer contexts and multi-device workers in relaxed capture mode;
# the whole GPU suite (the concurrent-capture test now with contexts).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06p
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r06p/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06p/pytest.log | tail -14; exit $rc
