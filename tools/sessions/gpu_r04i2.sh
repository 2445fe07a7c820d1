#!/bin/bash
# Session i2: the driver's exact bench command, 10 fresh processes back to
# back on one box (extras in their child process); stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04i2
mkdir -p $OUT
for r in $(seq 1 10); do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/out_$r.json 2> $OUT/err_$r.log
  rc=$?
  if [ $rc -ne 0 ]; then echo "run $r rc=$rc"; grep -v amdgpu.ids $OUT/err_$r.log | tail -20; exit $rc; fi
  python3 -c "import json; d=json.loads(open('$OUT/out_$r.json').read().strip().splitlines()[-1]); x=d['extras']; print($r, d['value'], d['value_replays']['median'], d['roofline']['frac'], d['parity'], 'extras', 'error' if 'error' in x else len(x), x.get('F9000',{}).get('parity'), x.get('ZIPF',{}).get('parity'), d['cpu_baseline']['value'])"
done
