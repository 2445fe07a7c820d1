# GPU tests, the low-latency probe, bench at N=1, then the world-8
# rehearsal: 8 gloo ranks sharing GPU 0, so every N>1 leg (the library's
# device-resident scatter included) runs at world 8 with the same code the
# driver's 8-GPU RCCL run takes.
set -u
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 60 python tools/probes/zc_probe.py > $O/zc_launch.log 2>&1
rc=$?; grep median $O/zc_launch.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_n1.log 2>&1
rc=$?; tail -c 400 $O/bench_n1.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 8 --dist-backend gloo \
  --one-device --steps 64 --warmup 16 --no-cpu-baseline > $O/bench_w8.log 2>&1
rc=$?; tail -c 2000 $O/bench_w8.log; exit $rc
