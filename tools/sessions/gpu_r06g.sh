#!/bin/bash
# r06g: the multi-branch launch order on torch's runtime (ROCm 7.0):
# tools/probe_graph_order.py, 30 s, graphs kept alive.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06g
timeout -k 10 120 python -u tools/probe_graph_order.py > gpurun_out/r06g/order_torch.json 2>&1
rc=$?; tail -2 gpurun_out/r06g/order_torch.json; exit $rc
