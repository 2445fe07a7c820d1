#!/bin/bash
# Instruction / cycle counters of the variable-length kernels (tools/pmc_var.py),
# two separate --pmc passes, each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_var
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS --output-format csv -d $OUT/p1 -o run -- python3 tools/pmc_var.py > $OUT/p1.log 2>&1 || { echo "p1 failed"; tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d $OUT/p2 -o run -- python3 tools/pmc_var.py > $OUT/p2.log 2>&1 || { echo "p2 failed"; tail -5 $OUT/p2.log; exit 1; }
for p in p1 p2; do
  f=$(ls $OUT/$p/*counter_collection.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 tools/pmc_var.py --summarise "$f" > $OUT/$p.summary.txt
  echo "== $p"; cat $OUT/$p.summary.txt
done
