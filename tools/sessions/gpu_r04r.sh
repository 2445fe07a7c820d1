#!/bin/bash
# Session r: where frame validation's waves spend their lifetime, against the
# same loads without the work (stream_slots_kernel) and F1500 - one rocprofv3
# --pmc pass (6 SQ counters) over tools/pmc_sq_target.py; only the summary
# comes back.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_r04r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d /tmp/pmc_sq -o run -- python tools/pmc_sq_target.py > $OUT/pmc_sq.log 2>&1
rc=$?; tail -2 $OUT/pmc_sq.log; [ $rc -ne 0 ] && exit $rc
python tools/pmc_sq_summary.py /tmp/pmc_sq/run_counter_collection.csv > $OUT/pmc_sq.json
cat $OUT/pmc_sq.json
