#!/bin/bash
# r06i: does one root node per graph (every branch behind it) restore the
# launch order on /opt/rocm's runtime? Kernel poison; no-destroy and churn
# forms, 40 s each, with CHURN_ONE_ROOT. rc 1 = mismatches (continue).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06i
mkdir -p $OUT
export CHURN_KERNEL_POISON=1 CHURN_ONE_ROOT=1
for v in nodrop churn; do
  case $v in nodrop*) export CHURN_NODROP=1;; *) unset CHURN_NODROP;; esac
  echo "== one root, $v ($(date +%T))"
  timeout -k 10 60 tests/native/_build/runtime_check graph-churn 40 $RANDOM > $OUT/churn_root_$v.log 2>&1
  rc=$?; echo "   rc=$rc"; grep mismatch $OUT/churn_root_$v.log | head -3; tail -1 $OUT/churn_root_$v.log | cut -c1-160
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
