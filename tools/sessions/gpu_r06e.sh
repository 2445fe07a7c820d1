#!/bin/bash
# r06e: the replay mismatches of the native multi-branch churn on /opt/rocm's
# runtime (r06c/r06d: 6-7 per 60 s), located: default, poison completed before
# each launch (CHURN_PRESYNC), device-wide wait after each replay
# (CHURN_DEVSYNC). rc 1 = mismatches (continue); anything else ends the script.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06e
mkdir -p $OUT
for v in default presync devsync; do
  case $v in
    presync) export CHURN_PRESYNC=1; unset CHURN_DEVSYNC;;
    devsync) export CHURN_DEVSYNC=1; unset CHURN_PRESYNC;;
    *) unset CHURN_PRESYNC CHURN_DEVSYNC;;
  esac
  echo "== churn $v ($(date +%T))"
  timeout -k 10 60 tests/native/_build/runtime_check graph-churn 40 $RANDOM > $OUT/churn_$v.log 2>&1
  rc=$?; echo "   rc=$rc"; grep mismatch $OUT/churn_$v.log | head -6; tail -1 $OUT/churn_$v.log | cut -c1-200
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
unset CHURN_PRESYNC CHURN_DEVSYNC
echo "== serial rate on /opt/rocm's runtime ($(date +%T))"
timeout -k 10 120 tests/native/_build/runtime_check serial-rate 1500 16 3b5bf0998c6646e9 > $OUT/rate_f1500.json 2>&1 &&
timeout -k 10 120 tests/native/_build/runtime_check serial-rate 9000 4 c6f7507092dc6a32 > $OUT/rate_f9000.json 2>&1
rc=$?; cut -c1-300 $OUT/rate_f1500.json $OUT/rate_f9000.json; exit $rc
