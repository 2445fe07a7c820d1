#!/bin/bash
# r06h: the multi-branch launch-order mismatches on /opt/rocm's runtime with no
# graph ever destroyed (CHURN_NODROP, 8 graphs) against the churn (kernel
# poison both), 40 s each. rc 1 = mismatches (continue).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06h
mkdir -p $OUT
export CHURN_KERNEL_POISON=1
for v in nodrop churn nodrop2; do
  case $v in nodrop*) export CHURN_NODROP=1;; *) unset CHURN_NODROP;; esac
  echo "== $v ($(date +%T))"
  timeout -k 10 60 tests/native/_build/runtime_check graph-churn 40 $RANDOM > $OUT/churn_$v.log 2>&1
  rc=$?; echo "   rc=$rc"; grep mismatch $OUT/churn_$v.log | head -3; tail -1 $OUT/churn_$v.log | cut -c1-160
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
