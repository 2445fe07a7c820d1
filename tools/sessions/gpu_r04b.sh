# round-4 session b (one GPU call): the GPU suite, smoke, the bench line,
# rocprofv3 stats + PMC passes, the self-launched world-8 rehearsal, then the
# A/B probes (frame validation geometries, tail-shaped ZIPF cut, graph
# branches). Every step has its own limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_r04b
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
step pytest_gpu 420 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
grep '^{' $OUT/bench.log > $OUT/bench.json
step stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python bench.py --no-cpu-baseline
python tools/trace_bursts.py $OUT/stats/run_kernel_trace.csv --all > $OUT/bursts_all.jsonl
step pmc_fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --no-cpu-baseline --steps 64 --warmup 16
step pmc_write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python bench.py --no-cpu-baseline --steps 64 --warmup 16
step rehearsal_w8 300 python bench.py --gpus 8 --dist-backend gloo --one-device --steps 64 --warmup 16 --no-cpu-baseline
grep '^{' $OUT/rehearsal_w8.log > $OUT/rehearsal_w8.json
step frames_fps 200 python -u tools/probe_frames_fps.py
step span_tail 300 python -u tools/probe_span_tail.py
echo "== done"
