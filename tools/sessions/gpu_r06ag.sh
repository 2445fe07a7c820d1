#!/bin/bash
# r06ag: r06ae's whole-suite run went silent inside
# test_native_section8f_kernels_against_fixtures. The same native command,
# with phase markers on stderr, 40 times in fresh processes (60 s limit each;
# the loop stops at the first failure or stall and prints where it stood).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06ag
timeout -k 10 900 python -u tools/sessions/diag_fixtures_loop.py 40 2>&1 | tee gpurun_out/r06ag/loop.log
