#!/bin/bash
# r06d: (1) A/B of the fixed-stride kernel's per-chunk sum as v_dot2 16-bit
# half sums (ab/lib_dot2.so, -DTCS_DOT2_PARTIAL) against the tree, F1500 and
# F9000 serial and 4-branch, with their load-pattern ceilings; (2) the
# multi-branch graph churn on /opt/rocm's runtime (native, replays poisoned in
# stream order); (3) the torch-only churn with synchronised teardown on
# torch's runtime. A crash ends the script there.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06d
mkdir -p $OUT
echo "== A/B dot2 ($(date +%T))"
ROUNDS=4 LIB_B=ab/lib_dot2.so timeout -k 10 300 python -u tools/sessions/probes/probe_fixed_ab.py > $OUT/ab_dot2.log 2>&1
rc=$?; echo "   rc=$rc"; tail -4 $OUT/ab_dot2.log
[ $rc -eq 0 ] || exit $rc
echo "== native graph churn ($(date +%T))"
timeout -k 10 90 tests/native/_build/runtime_check graph-churn 60 1 > $OUT/churn_native.log 2>&1
rc=$?; echo "   rc=$rc"; tail -2 $OUT/churn_native.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== torch churn, SYNCDROP=1 ($(date +%T))"
SYNCDROP=1 SECS=60 timeout -k 10 90 python -u tools/probe_graph_churn.py > $OUT/churn_syncdrop.log 2>&1
rc=$?; echo "   rc=$rc"; tail -2 $OUT/churn_syncdrop.log
exit $rc
