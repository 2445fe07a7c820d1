# round-5 session i: the GPU suite and the bench (driver form twice, 1,024
# steps once) with the 32 x 3 F1500 default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05i
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step suite 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests
step bench_d1 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_d2 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_1024 400 python -u bench.py
for f in bench_d1 bench_d2 bench_1024; do tail -1 $O/$f.log > $O/$f.json; done
python - <<'PY'
import json
for f in ("bench_d1", "bench_d2", "bench_1024"):
    d = json.load(open(f"gpurun_out/r05i/{f}.json"))
    print(f, d["value"], d["roofline"]["frac"], d["roofline"]["avg_launch_us"], d["roofline"]["kernel"], d["summary"])
PY
