#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box):
#  1. kernel-trace + stats of the default bench (timing agreement)
#  2. separate --pmc passes (FETCH_SIZE, then WRITE_SIZE) for HBM traffic
set -u
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -2 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
run bench 300 python bench.py
tail -1 $OUT/bench.log > $OUT/bench.json
run stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python bench.py --no-cpu-baseline
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --no-cpu-baseline --steps 64 --warmup 16
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python bench.py --no-cpu-baseline --steps 64 --warmup 16
run pmc_rdreq 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $OUT/pmc_rdreq -o run -- python bench.py --no-cpu-baseline --steps 64 --warmup 16
echo "== done"
