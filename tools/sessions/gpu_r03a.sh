set -u
mkdir -p gpurun_out/r03a
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03a/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/r03a/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r03a/bench.log 2>&1
rc=$?; tail -c 3000 gpurun_out/r03a/bench.log; exit $rc
