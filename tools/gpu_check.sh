#!/bin/bash
# One GPU-box session (run under gpurun): parity tests, smoke, bench, then
# rocprofv3 evidence for the bench workload — kernel-trace + stats (timing
# agreement) and separate --pmc passes (FETCH_SIZE, WRITE_SIZE, EA read
# requests) for HBM traffic. Summarise here afterwards with
#   python tools/pmc_traffic.py gpurun_out/prof_$TAG profiles $TAG
# Each GPU step has its own time limit; a crash / abort / timeout ends the
# script (pytest's rc 1 = "tests failed" is reported and also ends it).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
rocminfo 2>/dev/null | grep -m1 -E "gfx9" || true
step pytest_gpu 600 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
tail -1 $OUT/bench.log > $OUT/bench.json
step stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python bench.py --no-cpu-baseline
python tools/trace_bursts.py $OUT/stats/run_kernel_trace.csv --all > $OUT/bursts_all.jsonl
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --no-cpu-baseline --steps 64 --warmup 16
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python bench.py --no-cpu-baseline --steps 64 --warmup 16
step pmc_rdreq 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $OUT/pmc_rdreq -o run -- python bench.py --no-cpu-baseline --steps 64 --warmup 16
echo "== done"
