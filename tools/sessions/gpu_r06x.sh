#!/bin/bash
# r06x: the round's fuzz campaign on the final tree - every part of
# tests/test_fuzz.py with a new seed (3) and 100 s per part.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06x
TULIPS_FUZZ_SEED=3 TULIPS_FUZZ_SECONDS=100 timeout -k 10 1000 python -u -m pytest -v -s \
    --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu tests/test_fuzz.py \
    2>&1 | tee gpurun_out/r06x/fuzz.log | grep --line-buffered -E "fuzz|PASSED|FAILED|passed|failed"
