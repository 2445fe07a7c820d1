set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_span.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/s3_test.log 2>&1; rc=$?
tail -5 gpurun_out/s3_test.log
[ $rc -ne 0 ] && exit $rc
PROBE_PIPE=1 PROBE_SIZES=1024,65536,98304 PROBE_GEOMS=span8,s3_4,s3_6,s3_8,s3_10,s2_8h2 timeout -k 10 300 python -u tools/probe_gen.py > gpurun_out/s3_probe.log 2>&1; rc=$?
cat gpurun_out/s3_probe.log | tail -5
exit $rc
