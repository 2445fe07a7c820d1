#!/bin/bash
# A/B of prebuilt diagnostic libraries under tools/probe_gen.py (run under
# gpurun): swaps tools/ab_<X>.so into place in the box's scratch copy for each
# X of AB_ORDER and prints the probe's lines.
set -u
export PROBE_PIPE=${PROBE_PIPE:-1}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for X in ${AB_ORDER}; do
  cp tools/ab_$X.so tulips_amd/libtulips_csum.so
  echo "== $X"
  timeout -k 10 200 python -u tools/probe_gen.py > gpurun_out/ab_probe_$X.log 2>&1 || exit 1
  grep '^{' gpurun_out/ab_probe_$X.log
done
