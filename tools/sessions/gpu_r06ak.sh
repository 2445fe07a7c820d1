#!/bin/bash
# r06ak: is frame validation bound by VALU issue? One --pmc pass of SQ
# counters (waves, VALU / SALU / VMEM / LDS instructions, busy and wave
# cycles) over the frame ops probe (validate and fields only, one round).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r06ak
mkdir -p $OUT
PROBE_OPS="validate fields" ROUNDS=1 timeout -s KILL 120 rocprofv3 \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  --output-format csv -d $OUT/pmc -o run -- python tools/sessions/probes/probe_gen_defer.py > $OUT/probe.log 2>&1
rc=$?
python - <<'PY'
import csv, collections, glob
rows = list(csv.DictReader(open(glob.glob("gpurun_out/r06ak/pmc/**/run_counter_collection.csv", recursive=True)[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:90]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES":
        cnt[k] += 1
for k, v in agg.items():
    if "frame_kernel" not in k:
        continue
    n = cnt[k]
    w = v["SQ_WAVES"] / n
    print(k, "dispatches", n, "waves/disp", round(w),
          {c: round(v[c] / n / w, 1) for c in v if c != "SQ_WAVES"})
PY
rm -f $OUT/pmc/*/*/run_counter_collection.csv 2>/dev/null
exit $rc
