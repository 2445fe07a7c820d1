# round-4 session c: headline graph branches 16 vs 32 (alternated), and one
# PMC pass of instruction counters over the bench's kernels (VALU / SALU /
# vector-memory instructions per wave) to price the frame kernels' arithmetic
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_r04c
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do for s in 16 32; do
  timeout -k 10 150 python bench.py --no-extras --no-cpu-baseline --streams $s > $OUT/s.json 2>/dev/null || exit $?
  python -c "import json;d=json.loads([l for l in open('$OUT/s.json') if l.startswith('{')][-1]);print($r,$s,d['value'],d['value_replays']['median'],d['roofline']['avg_launch_us'],d['parity'],flush=True)" | tee -a $OUT/streams.log
done; done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc_sq -o run -- python bench.py --no-cpu-baseline --steps 64 --warmup 16 > $OUT/pmc_sq.log 2>&1
echo "pmc rc=$?"
