#!/bin/bash
# r06r: in-place generation with the field stores deferred behind the next
# frame's loads (frames.hip TULIPS_GEN_DEFER_STORES) against the product
# build, alternated 3 times on one box (probe_gen_defer.py: serial and
# 4-branch fractions, the arena regenerated and checked before and after).
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r06r LIBS="base defer" ROUNDS=3 PROBE=tools/sessions/probes/probe_gen_defer.py \
  PROBE_OPS="generate fields" ROUNDS_INNER=2 bash tools/sessions/probes/ab_libs.sh
