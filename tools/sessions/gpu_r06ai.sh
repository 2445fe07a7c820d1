#!/bin/bash
# r06ai: the evidence session on the tree with the header-derived IPv4 sums
# (tools/gpu_check.sh: GPU tests, smoke, bench in both forms, rocprofv3 stats,
# PMC passes, world-8 rehearsal).
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r06ai bash tools/gpu_check.sh
