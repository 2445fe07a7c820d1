set -u
mkdir -p gpurun_out/r03b
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03b/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/r03b/pytest_gpu.log; exit $rc
