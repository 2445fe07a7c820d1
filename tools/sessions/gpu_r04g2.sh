#!/bin/bash
# Session g2: the driver's bench form three times in fresh processes, with
# faulthandler and per-stage progress on stderr (a run on one box died with
# SIGSEGV and no output); stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04g2
mkdir -p $OUT
for r in 1 2 3; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/out_$r.json 2> $OUT/err_$r.log
  rc=$?
  echo "run $r rc=$rc $(grep -c '^\[bench' $OUT/err_$r.log) stages; last: $(grep '^\[bench' $OUT/err_$r.log | tail -1)"
  if [ $rc -ne 0 ]; then grep -v amdgpu.ids $OUT/err_$r.log | tail -40; exit $rc; fi
  python -c "import json; d=json.loads(open('$OUT/out_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['parity'], d['roofline']['frac'])"
done
