# WRITE_SIZE / FETCH_SIZE per segment_kernel dispatch of tools/probe_segment.py
# under each prebuilt tools/ab_<L>.so (separate --pmc passes); run under gpurun.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in ${SEGPROF_LIBS:-cur}; do
  cp tools/ab_$L.so tulips_amd/libtulips_csum.so
  for C in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/segpmc_${L}_$C -o run -- python3 tools/probe_segment.py > gpurun_out/segpmc_${L}_$C.log 2>&1
    python3 - gpurun_out/segpmc_${L}_$C/run_counter_collection.csv $L $C <<'PY'
import csv, sys
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1]))
     if "segment_kernel" in r["Kernel_Name"]]
print(sys.argv[2], sys.argv[3], len(v), "dispatches, mean", sum(v) / max(len(v), 1), "KiB-units")
PY
  done
done
