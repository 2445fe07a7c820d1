#!/bin/bash
# Headline `value` at several graph-branch counts, alternated on one box:
#   STREAMS="4 8" ROUNDS=4 bash tools/ab_streams.sh  (under gpurun)
# One line per run: round, branches, value, replay median, serial us.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 "${ROUNDS:-4}"); do for s in ${STREAMS:-4 8 4 8}; do
  timeout -k 10 120 python bench.py --no-extras --no-cpu-baseline --streams $s > gpurun_out/s3.json 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/s3.json').read().splitlines()[-1]);print($r,$s,d['value'],d['value_replays']['median'],d['roofline']['avg_launch_us'],flush=True)" | tee -a gpurun_out/${OUT:-streams3}.log
done; done
