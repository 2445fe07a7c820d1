# round-4 session e: the start delay at the driver's 20 steps (on / off,
# alternated) and a re-sweep of frame-validation geometries after round 3's
# DPP reductions
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_r04e
mkdir -p $OUT
for r in 1 2 3; do for dl in 0 200; do
  timeout -k 10 150 python bench.py --no-extras --no-cpu-baseline --steps 20 --warmup 5 --start-delay-us $dl > $OUT/s.json 2>/dev/null || exit $?
  python -c "import json;d=json.loads([l for l in open('$OUT/s.json') if l.startswith('{')][-1]);print($r,'delay',$dl,d['value'],d['value_replays']['median'],d['roofline']['avg_launch_us'],d['parity'],flush=True)" | tee -a $OUT/delay20.log
done; done
timeout -k 10 150 python bench.py --no-extras --no-cpu-baseline > $OUT/s.json 2>/dev/null || exit $?
python -c "import json;d=json.loads([l for l in open('$OUT/s.json') if l.startswith('{')][-1]);print('1024 steps delay 200',d['value'],d['value_replays']['median'],d['roofline']['avg_launch_us'],d['parity'],flush=True)" | tee -a $OUT/delay20.log
GEOMS="16x6 32x4 64x2 16x8 16x4" ROUNDS=2 timeout -k 10 300 python -u tools/probe_frames_fps.py > $OUT/geoms.log 2>&1
rc=$?; tail -1 $OUT/geoms.log; exit $rc
