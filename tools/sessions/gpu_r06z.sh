#!/bin/bash
# r06z: the whole GPU suite and smoke() on the tree as it stands.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06z
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r06z/pytest.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06z/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r06z/pytest.log; tail -1 gpurun_out/r06z/smoke.log; exit $rc
