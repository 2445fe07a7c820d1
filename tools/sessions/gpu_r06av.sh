#!/bin/bash
# r06av: the fuzz parts that drive the final range-sum form (frames and
# segmentation, runts and truncated frames among them; the host context's frame and
# TSO paths), new seed 7, 150 s each.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06av
TULIPS_FUZZ_SEED=7 TULIPS_FUZZ_SECONDS=150 timeout -k 10 600 python -u -m pytest -v -s \
    --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu \
    "tests/test_fuzz.py::test_fuzz_frames_and_segmentation_vs_oracle" \
    "tests/test_fuzz.py::test_fuzz_host_context_vs_oracle" \
    2>&1 | tee gpurun_out/r06av/fuzz.log | grep --line-buffered -E "fuzz|PASSED|FAILED|passed|failed"
