#!/bin/bash
# r06k: graph ownership under multi-branch churn on /opt/rocm's runtime, the
# memory check in two halves (the second half's graphs must leave nothing).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06k
mkdir -p $OUT
timeout -k 10 100 tests/native/_build/runtime_check graph-churn-stateful 60 $RANDOM > $OUT/churn_stateful.log 2>&1
rc=$?; echo "rc=$rc"; grep mismatch $OUT/churn_stateful.log | head -4; tail -1 $OUT/churn_stateful.log | cut -c1-400
exit $rc
