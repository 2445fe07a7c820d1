#!/bin/bash
# r06ah: the whole GPU suite again, verbose (one line per test, so the
# harness sees progress), with the native fixtures run now limited to 90 s and
# reporting its phase markers if it stalls as in r06ae.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06ah
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -8; exit $rc
