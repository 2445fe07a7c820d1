#!/bin/bash
# r06aw: the evidence session on the final tree (tools/gpu_check.sh: GPU
# tests, smoke, bench in both forms, rocprofv3 stats, PMC passes, world-8
# rehearsal), so the committed rocprof / PMC summaries are the final tree's.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r06aw bash tools/gpu_check.sh
