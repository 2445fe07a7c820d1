#!/bin/bash
# Session h2: the extras child alone, up to 8 fresh processes, to see how
# often the segmentation pipeline graph's first replay faults (faulthandler
# stack kept); the script ends at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04h2
mkdir -p $OUT
for r in $(seq 1 8); do
  timeout -k 10 200 python bench.py --extras-child > $OUT/out_$r.json 2> $OUT/err_$r.log
  rc=$?
  echo "run $r rc=$rc last: $(grep '^\[bench' $OUT/err_$r.log | tail -1)"
  if [ $rc -ne 0 ]; then grep -A8 "Fatal Python" $OUT/err_$r.log | head -10; exit $rc; fi
done
exit 0
