#!/bin/bash
# Session m: headline at the driver's form (--steps 20 --warmup 5) with the
# branch count chosen by step count (2) against 16, alternated; then the
# default 1,024-step form at both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04m
mkdir -p $OUT
row() {  # row <label> <args...>
  local label=$1; shift
  timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline "$@" > $OUT/run.log 2>&1 || { echo "STOP $label"; tail -5 $OUT/run.log; exit 1; }
  tail -1 $OUT/run.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', d['config']['streams'], d['value'], d.get('value_replays',{}).get('median'), d['parity'])"
}
for r in 1 2 3; do
  row "$r steps20" --steps 20 --warmup 5
  row "$r steps20" --steps 20 --warmup 5 --streams 16
done
row "1024" --steps 1024 --warmup 16 --streams 2
row "1024" --steps 1024 --warmup 16
