#!/bin/bash
# r06aj: the fuzz parts that drive the kernels changed after r06x (frames and
# segmentation with the header-derived IPv4 sums; the host context's frame and
# TSO paths), new seed 4, 150 s each.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06aj
TULIPS_FUZZ_SEED=4 TULIPS_FUZZ_SECONDS=150 timeout -k 10 600 python -u -m pytest -v -s \
    --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu \
    "tests/test_fuzz.py::test_fuzz_frames_and_segmentation_vs_oracle" \
    "tests/test_fuzz.py::test_fuzz_host_context_vs_oracle" \
    2>&1 | tee gpurun_out/r06aj/fuzz.log | grep --line-buffered -E "fuzz|PASSED|FAILED|passed|failed"
