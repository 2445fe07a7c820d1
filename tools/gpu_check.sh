#!/bin/bash
# One GPU-box session (run under gpurun): parity tests, smoke, bench, then
# rocprofv3 evidence for the bench workload - kernel-trace + stats (timing
# agreement) and separate --pmc passes (FETCH_SIZE, WRITE_SIZE) for HBM
# traffic - and the world-8 rehearsal (8 gloo ranks sharing GPU 0, every
# N>1 leg at world 8). The summaries (tools/pmc_traffic.py) are made on the
# box under gpurun_out/prof_$TAG/summary; copy them into profiles/ here.
# Each GPU step has its own time limit; a crash / abort / timeout ends the
# script (pytest's rc 1 = "tests failed" is reported and also ends it).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04}
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
if [ -z "${PROF_ONLY:-}" ]; then   # PROF_ONLY=1: the rocprofv3 steps alone
step pytest_gpu 600 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py
tail -1 $OUT/bench.log > $OUT/bench.json
# the driver's form (python3 bench.py --gpus 1 --steps 20 --warmup 5)
step bench_driver 400 python bench.py --gpus 1 --steps 20 --warmup 5
tail -1 $OUT/bench_driver.log > $OUT/bench_driver.json
fi
# bench.py runs its side measurements in a child process, which rocprofv3
# does not follow: the headline (--no-extras) and the extras child
# (--extras-child) are profiled as two programs and their CSVs merged; the
# aligned-stride legs are left out of those passes (same kernels and grids as
# the rotated F1500 / F9000 batches, so their counters would mix)
step stats 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_h -o run -- python bench.py --no-cpu-baseline --no-extras
BENCH_EXTRAS_SKIP=aligned_strides step stats_x 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_x -o run -- python bench.py --extras-child
step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_h -o run -- python bench.py --no-cpu-baseline --no-extras --steps 64 --warmup 16
BENCH_EXTRAS_SKIP=aligned_strides step pmc_fetch_x 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_x -o run -- python bench.py --extras-child
step pmc_write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_h -o run -- python bench.py --no-cpu-baseline --no-extras --steps 64 --warmup 16
BENCH_EXTRAS_SKIP=aligned_strides step pmc_write_x 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_x -o run -- python bench.py --extras-child
python tools/merge_csv.py $OUT/stats/run_kernel_trace.csv $OUT/stats_h/run_kernel_trace.csv $OUT/stats_x/run_kernel_trace.csv
python tools/merge_csv.py $OUT/stats/run_kernel_stats.csv $OUT/stats_h/run_kernel_stats.csv $OUT/stats_x/run_kernel_stats.csv
python tools/merge_csv.py $OUT/pmc_fetch/run_counter_collection.csv $OUT/pmc_fetch_h/run_counter_collection.csv $OUT/pmc_fetch_x/run_counter_collection.csv
python tools/merge_csv.py $OUT/pmc_write/run_counter_collection.csv $OUT/pmc_write_h/run_counter_collection.csv $OUT/pmc_write_x/run_counter_collection.csv
rm -rf $OUT/stats_h $OUT/stats_x $OUT/pmc_fetch_h $OUT/pmc_fetch_x $OUT/pmc_write_h $OUT/pmc_write_x
python tools/trace_bursts.py $OUT/stats/run_kernel_trace.csv --all > $OUT/bursts_all.jsonl
# summaries on the box (the raw traces would push gpurun_out past what gpurun
# copies back, 64 MiB): profiles-ready files under $OUT/summary, raw CSVs dropped
mkdir -p $OUT/summary
python tools/pmc_traffic.py $OUT $OUT/summary $TAG > $OUT/summary/pmc_traffic.log 2>&1 || true
rm -f $OUT/stats/run_kernel_trace.csv $OUT/pmc_fetch/run_counter_collection.csv \
      $OUT/pmc_write/run_counter_collection.csv
# (no launcher: bench.py starts torch.distributed.run itself, as under the
# driver's `python bench.py --gpus 8`)
[ -n "${PROF_ONLY:-}" ] && { echo "== done (profiles only)"; exit 0; }
step rehearsal_w8 600 python bench.py --gpus 8 --dist-backend gloo --one-device --steps 64 --warmup 16 --no-cpu-baseline
tail -1 $OUT/rehearsal_w8.log > $OUT/rehearsal_w8.json
echo "== done"
