# round-4 session b: the whole GPU suite, then the frame-validation A/B
set -u
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1
rc=$?; tail -5 $O/suite.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/probe_frames_fps.py > $O/frames_fps.log 2>&1
rc=$?; tail -3 $O/frames_fps.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/probe_span_tail.py > $O/span_tail.log 2>&1
rc=$?; tail -3 $O/span_tail.log; exit $rc
