#!/bin/bash
# r06u: the multi-device leg of bench.py in its own child process: the world-8
# rehearsal (8 gloo ranks sharing GPU 0) and the bench-launch GPU tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06u
timeout -k 10 300 python -u -m pytest -v --timeout 250 --timeout-method thread -p no:cacheprovider \
    tests/test_bench_launch.py -m gpu > gpurun_out/r06u/pytest.log 2>&1 &&
timeout -k 10 600 python bench.py --gpus 8 --dist-backend gloo --one-device --steps 64 --warmup 16 \
    --no-cpu-baseline > gpurun_out/r06u/rehearsal_w8.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r06u/pytest.log; tail -1 gpurun_out/r06u/rehearsal_w8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['multi_gpu']['library_scatter_from_gpu0'])[:800]); print(d['value'], d['parity'])"; exit $rc
