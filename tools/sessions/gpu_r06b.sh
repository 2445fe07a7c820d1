#!/bin/bash
# r06b: the whole GPU suite on the trimmed ABI, smoke, driver-form bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06b
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 600 --timeout-method thread tests \
    > gpurun_out/r06b/pytest.log 2>&1
rc=$?
tail -15 gpurun_out/r06b/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06b/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/r06b/bench.json 2> gpurun_out/r06b/bench.err
rc2=$?
tail -2 gpurun_out/r06b/smoke.log
tail -c 1500 gpurun_out/r06b/bench.json
exit $(( rc | rc2 ))
