#!/bin/bash
# r06f: is the multi-branch launch's missing order after the launch stream's
# earlier work specific to hipMemsetAsync? The native churn with the poison
# written by a kernel (CHURN_KERNEL_POISON) against hipMemsetAsync (default),
# 40 s each, on /opt/rocm's runtime. rc 1 = mismatches (continue).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06f
mkdir -p $OUT
for v in kernel memset kernel2; do
  case $v in kernel*) export CHURN_KERNEL_POISON=1;; *) unset CHURN_KERNEL_POISON;; esac
  echo "== churn poison=$v ($(date +%T))"
  timeout -k 10 60 tests/native/_build/runtime_check graph-churn 40 $RANDOM > $OUT/churn_$v.log 2>&1
  rc=$?; echo "   rc=$rc"; grep mismatch $OUT/churn_$v.log | head -4; tail -1 $OUT/churn_$v.log | cut -c1-160
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
