#!/bin/bash
# r06o: which calls of one thread break another thread's global-mode capture
# (tools/probe_capture_modes.py), on torch's runtime and on /opt/rocm's.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06o
timeout -k 10 400 python -u tools/probe_capture_modes.py torch > gpurun_out/r06o/torch.jsonl 2>&1 &&
timeout -k 10 400 python -u tools/probe_capture_modes.py opt > gpurun_out/r06o/opt.jsonl 2>&1
rc=$?; cat gpurun_out/r06o/*.jsonl; exit $rc
