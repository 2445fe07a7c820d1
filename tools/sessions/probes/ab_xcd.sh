#!/bin/bash
# A/B of the XCD cluster size (diagnostic; `make xcd_ab` here first, then
# run under gpurun). Swaps the prebuilt tools/libcsum_xcd<C>.so into place in
# the box's scratch copy, runs the bench without the CPU leg, and prints the
# per-kernel timings.
set -u
mkdir -p gpurun_out
for C in ${AB_ORDER:-1 8 1024 2 4 32 1 8}; do  # or any tools/libcsum_xcd<C>.so suffixes
  if [ -f tools/ab_$C.so ]; then cp tools/ab_$C.so tulips_amd/libtulips_csum.so; else cp tools/libcsum_xcd$C.so tulips_amd/libtulips_csum.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ab_c$C.json 2> gpurun_out/ab_c$C.err || exit 1
  python - "$C" <<'PY'
import json, sys
C = sys.argv[1]
d = json.load(open(f"gpurun_out/ab_c{C}.json")); e = d["extras"]
r = lambda k: (e[k]["avg_launch_us"], e[k].get("pipeline", {}).get("us_per_launch"))
print(f"C={C:>5} F1500 {d['roofline']['avg_launch_us']} {d['roofline']['pipeline']['us_per_launch']}"
      f" F9000 {r('F9000')} ZIPF {r('ZIPF')} seg {r('segment_TSO_64K_mss1460')}"
      f" val {r('frames_validate_F1514')} gen {r('frames_generate_F1514')} rss {r('rss_toeplitz_16M')}"
      f" e2e {e['e2e_host_F1500']['pinned']['GiBps']} {e['e2e_host_F1500']['pageable']['GiBps']}")
PY
done
