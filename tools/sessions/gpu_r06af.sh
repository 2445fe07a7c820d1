#!/bin/bash
# r06af: r06ae's whole-suite run went silent for 180 s after test_multi's
# skipped real-peer tests (killed by the harness, GPU answering). The tests
# from there on, verbose, each under its own 150 s limit (thread method, so a
# stuck test is named with its stack), written straight to the log.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06af
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -v -s --durations=0 --timeout 150 --timeout-method thread \
    -p no:cacheprovider -m gpu tests/test_multi.py tests/test_native_runtime.py \
    tests/test_oracle.py tests/test_rss.py tests/test_segment.py 2>&1 | tee $OUT/pytest.log
