#!/bin/bash
# Session x: the headline's spread in the driver's form - 10 fresh processes
# of `bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline`
# back to back on one box, then 3 of the default 1,024-step form.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04x
mkdir -p $OUT
run() {  # run <label> <args...>
  local label=$1; shift
  timeout -k 10 200 python bench.py --gpus 1 --no-extras --no-cpu-baseline "$@" > $OUT/run.log 2>&1 || { echo "STOP $label"; tail -5 $OUT/run.log; exit 1; }
  tail -1 $OUT/run.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', d['steps'], d['config']['streams'], d['value'], d['value_replays']['median'], d['roofline']['avg_launch_us'], d['parity'], flush=True)"
}
for r in $(seq 1 10); do run "$r" --steps 20 --warmup 5; done
for r in 1 2 3; do run "L$r" --steps 1024 --warmup 32; done
