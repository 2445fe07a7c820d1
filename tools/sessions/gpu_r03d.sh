set -u
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_frames.py tests/test_gpucsum_device.py tests/test_dropin.py tests/test_multi.py -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
TULIPS_ZC_MODE=resident timeout -k 10 600 python -u -m pytest tests/test_frames.py -k zero_copy -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_res.log 2>&1
rc=$?; tail -3 $O/pytest_res.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 90 python tools/probes/zc_probe.py > $O/zc_launch.log 2>&1
rc=$?; cat $O/zc_launch.log; [ $rc -ne 0 ] && exit $rc
TULIPS_ZC_MODE=resident timeout -k 10 90 python tools/probes/zc_probe.py > $O/zc_res.log 2>&1
rc=$?; cat $O/zc_res.log; exit $rc
