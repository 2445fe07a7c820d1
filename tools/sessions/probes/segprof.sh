# Kernel-trace stats of tools/probe_segment.py (segmentation alone, 50 calls)
# under each prebuilt tools/ab_<L>.so; run under gpurun.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in ${SEGPROF_LIBS:-old new2}; do
  cp tools/ab_$L.so tulips_amd/libtulips_csum.so
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/segprof_$L -o run -- python3 tools/probe_segment.py > gpurun_out/segprof_$L.log 2>&1
done
for L in ${SEGPROF_LIBS:-old new2}; do echo "== $L"; find gpurun_out/segprof_$L -name "*kernel_stats.csv" -exec cut -d, -f1-8 {} \; | python3 -c "import sys,csv; [print(r[0][:70], *r[1:8]) for r in csv.reader(sys.stdin)]" | grep -v "^\"Name" ; done
