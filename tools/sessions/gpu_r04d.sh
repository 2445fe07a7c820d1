# round-4 session d: SQ instruction counters over F1500, frame validation and
# the ZIPF arena kernel (a short dedicated workload; only a summary is kept)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_r04d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d /tmp/pmc_sq -o run -- python tools/pmc_sq_target.py > $OUT/pmc_sq.log 2>&1
rc=$?; tail -2 $OUT/pmc_sq.log; [ $rc -ne 0 ] && exit $rc
python tools/pmc_sq_summary.py /tmp/pmc_sq/run_counter_collection.csv > $OUT/pmc_sq.json
cat $OUT/pmc_sq.json | head -80
# the driver's bench form (--steps 20 --warmup 5): value by graph branches
for r in 1 2 3; do for s in 4 8 16 32; do
  timeout -k 10 150 python bench.py --no-extras --no-cpu-baseline --steps 20 --warmup 5 --streams $s > $OUT/s.json 2>/dev/null || exit $?
  python -c "import json;d=json.loads([l for l in open('$OUT/s.json') if l.startswith('{')][-1]);print($r,$s,d['value'],d['value_replays']['median'],d['roofline']['avg_launch_us'],d['parity'],flush=True)" | tee -a $OUT/streams20.log
done; done
