#!/bin/bash
# r06j: which end of the replay is unordered on /opt/rocm's runtime? Each
# mismatch re-read after the device idles (right = the kernel finished after
# the sync; still poisoned = it ran before the poison). Kernel poison,
# no-destroy form (most replays), 40 s; then the churn form, 40 s.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06j
mkdir -p $OUT
export CHURN_KERNEL_POISON=1
for v in nodrop churn; do
  case $v in nodrop*) export CHURN_NODROP=1;; *) unset CHURN_NODROP;; esac
  echo "== $v ($(date +%T))"
  timeout -k 10 60 tests/native/_build/runtime_check graph-churn 40 $RANDOM > $OUT/churn_$v.log 2>&1
  rc=$?; echo "   rc=$rc"; grep mismatch $OUT/churn_$v.log | head -6; tail -1 $OUT/churn_$v.log | cut -c1-160
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
unset CHURN_KERNEL_POISON CHURN_NODROP
echo "== stateful multi-branch churn, graph ownership ($(date +%T))"
timeout -k 10 100 tests/native/_build/runtime_check graph-churn-stateful 60 $RANDOM > $OUT/churn_stateful.log 2>&1
rc=$?; echo "   rc=$rc"; grep mismatch $OUT/churn_stateful.log | head -4; tail -1 $OUT/churn_stateful.log | cut -c1-300
exit $rc
