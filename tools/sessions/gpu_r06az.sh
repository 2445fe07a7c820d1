#!/bin/bash
# r06az: the whole GPU suite and smoke on the libraries build() produced last
# (the round-end state), nothing rebuilt on the box.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06az
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r06az/pytest.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06az/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r06az/pytest.log; tail -1 gpurun_out/r06az/smoke.log; exit $rc
