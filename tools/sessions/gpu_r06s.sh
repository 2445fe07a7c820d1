#!/bin/bash
# r06s: where in-place generation's time goes. The product build against a
# diagnostic build whose field stores land in the unread padding of each
# 2 KiB slot (scattered sub-line writes to lines no load touches); parity
# checks of the generate op are off for both (GEN_DIAG=1), fields are not timed here (their check needs correct headers).
cd "$GRAFT_REPO_ROOT" || exit 1
GEN_DIAG=1 TAG=r06s LIBS="base padstore" ROUNDS=3 PROBE=tools/sessions/probes/probe_gen_defer.py \
  PROBE_OPS="generate" bash tools/sessions/probes/ab_libs.sh
