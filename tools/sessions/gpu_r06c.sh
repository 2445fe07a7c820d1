#!/bin/bash
# r06c: the round's evidence session (tools/gpu_check.sh: GPU tests, smoke,
# bench in both forms, rocprofv3 stats, PMC passes, world-8 rehearsal), then
# the graph-launch fault characterised once more: the
# multi-branch churn on /opt/rocm's runtime (native, library calls), then the
# torch-only churn with synchronised teardown on torch's runtime. A crash ends
# the script there.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r06c bash tools/gpu_check.sh || exit $?
OUT=gpurun_out/prof_r06c
echo "== native graph churn ($(date +%T))"
timeout -k 10 90 tests/native/_build/runtime_check graph-churn 60 1 > $OUT/churn_native.log 2>&1
rc=$?; echo "   rc=$rc"; tail -2 $OUT/churn_native.log
[ $rc -eq 0 ] || exit $rc
echo "== torch churn, SYNCDROP=1 ($(date +%T))"
SYNCDROP=1 SECS=60 timeout -k 10 90 python -u tools/probe_graph_churn.py > $OUT/churn_syncdrop.log 2>&1
rc=$?; echo "   rc=$rc"; tail -2 $OUT/churn_syncdrop.log
exit $rc
