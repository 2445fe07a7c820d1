#!/bin/bash
# r06q: the round's final evidence session on the final tree
# (tools/gpu_check.sh: GPU tests, smoke, bench in both forms, rocprofv3 stats,
# PMC passes, world-8 rehearsal).
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r06q bash tools/gpu_check.sh
