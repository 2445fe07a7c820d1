#!/bin/bash
# r06at: the fuzz parts that drive the segmentation dot2 sums of r06ar (frames and
# segmentation, runts and truncated frames among them; the host context's frame and
# TSO paths), new seed 6, 200 s each.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06at
TULIPS_FUZZ_SEED=6 TULIPS_FUZZ_SECONDS=200 timeout -k 10 600 python -u -m pytest -v -s \
    --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu \
    "tests/test_fuzz.py::test_fuzz_frames_and_segmentation_vs_oracle" \
    "tests/test_fuzz.py::test_fuzz_host_context_vs_oracle" \
    2>&1 | tee gpurun_out/r06at/fuzz.log | grep --line-buffered -E "fuzz|PASSED|FAILED|passed|failed"
