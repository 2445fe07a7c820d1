#!/bin/bash
# r06ao: the TCP range summed to the frame's end and reduced before the header
# is parsed (frames.hip TULIPS_FRAME_EARLY_L4; exact re-sum when the segment
# ends before the frame): el4 bounded to 6 waves/SIMD (spills ~11 VGPRs), el4u
# unbounded (110 VGPRs, 4 waves) for validation; against the product. Frame
# and segmentation tests on el4u, the frame ops alternated 3 times, SQ
# counters of the validate kernel per build.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06ao
mkdir -p $OUT
LIB=tulips_amd/libtulips_csum.so
cp $LIB /tmp/lib_tree.so
cp ab_libs/lib_el4u.so $LIB
timeout -k 10 400 python -u -m pytest tests/test_frames.py tests/test_segment.py -q -m gpu -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $OUT/pytest_el4u.log 2>&1
rc=$?
cp /tmp/lib_tree.so $LIB
tail -2 $OUT/pytest_el4u.log
[ $rc -eq 0 ] || { echo "STOP: tests on el4u rc=$rc"; exit $rc; }
cp ab_libs/lib_el4.so $LIB
timeout -k 10 400 python -u -m pytest tests/test_frames.py -q -m gpu -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $OUT/pytest_el4.log 2>&1
rc=$?
cp /tmp/lib_tree.so $LIB
tail -2 $OUT/pytest_el4.log
[ $rc -eq 0 ] || { echo "STOP: frame tests on the variant rc=$rc"; exit $rc; }
TAG=r06ao LIBS="base el4 el4u" ROUNDS=3 PROBE=tools/sessions/probes/probe_gen_defer.py \
  bash tools/sessions/probes/ab_libs.sh || exit $?
for name in base el4 el4u; do
  cp ab_libs/lib_$name.so $LIB
  PROBE_OPS="validate" ROUNDS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU \
    --output-format csv -d $OUT/pmc_$name -o run -- python tools/sessions/probes/probe_gen_defer.py \
    > $OUT/pmc_$name.log 2>&1 || { cp /tmp/lib_tree.so $LIB; exit 1; }
done
cp /tmp/lib_tree.so $LIB
python - <<'PY'
import csv, collections, glob
for name in ("base", "el4", "el4u"):
    f = glob.glob(f"gpurun_out/r06ao/pmc_{name}/**/run_counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "frame_kernel<0, 16, 6, true, 1>" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    w = agg["SQ_WAVES"]
    print(name, "VALU/wave", round(agg["SQ_INSTS_VALU"] / w, 1), "SALU/wave", round(agg["SQ_INSTS_SALU"] / w, 1))
PY
rm -f gpurun_out/r06ao/pmc_*/*/*/run_counter_collection.csv gpurun_out/r06ao/pmc_*/*/run_counter_collection.csv
