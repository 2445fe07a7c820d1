#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash / abort / timeout ends the
# script (exit codes >= 2 other than pytest's 1 = "tests failed").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r01}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
rocminfo 2>/dev/null | grep -m1 -E "gfx9" || true
step pytest_gpu 900 python -m pytest tests -q -m gpu -x -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
cat gpurun_out/bench.log | tail -1 > gpurun_out/bench_$TAG.json
export TMPDIR=/tmp
step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --no-cpu-baseline --steps 320
python tools/trace_bursts.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/prof_$TAG/bursts_F1500.jsonl
cat gpurun_out/prof_$TAG/bursts_F1500.jsonl
echo "== done"
