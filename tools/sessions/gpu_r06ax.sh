#!/bin/bash
# r06ax: every part of tests/test_fuzz.py on the final tree, new seed (8),
# 120 s per part.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06ax
TULIPS_FUZZ_SEED=8 TULIPS_FUZZ_SECONDS=120 timeout -k 10 1100 python -u -m pytest -v -s \
    --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu tests/test_fuzz.py \
    2>&1 | tee gpurun_out/r06ax/fuzz.log | grep --line-buffered -E "fuzz|PASSED|FAILED|passed|failed"
