# round-4 session b: the whole GPU suite (then the 4-rank self-launched bench
# test, which the suite also holds, is timed there)
set -u
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1
rc=$?; tail -5 $O/suite.log; exit $rc
