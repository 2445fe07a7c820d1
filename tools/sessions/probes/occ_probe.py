"""F1500 (16 rotated batches) through csum_kernel<32, 4> with dynamic LDS
capping the workgroups per CU (tools/probes/occ_probe.hip): 8 (no LDS), 7,
6, 5 and 4 workgroups of 4 waves per CU = waves per SIMD. Results compared
with the library's. Measurement only."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from tulips_amd import csum  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ol = C.CDLL(os.path.join(HERE, "libocc_probe.so"))
ol.occ_launch.restype = C.c_int
ol.occ_launch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream()
timer = bench.Timer(torch, stream)
NSEG, SEG = bench.NSEG, bench.SEG
bb = NSEG * SEG
ar = torch.empty(16 * bb + 256, dtype=torch.uint8, device=dev)
csum.fill_splitmix(ar, 16 * bb)
out = torch.empty(16 * NSEG, dtype=torch.int16, device=dev)
ref = torch.empty_like(out)
for b in range(16):
    assert csum.lib.tulips_csum_batch_fixed(ar.data_ptr() + b * bb, SEG, SEG, None, None, None,
                                            ref.data_ptr() + 2 * b * NSEG, NSEG, 0,
                                            stream.cuda_stream) == 0
LDS = {8: 0, 7: 21 * 1024, 6: 24 * 1024, 5: 30 * 1024, 4: 38 * 1024}
res = {}
for rnd in range(3):
    for wps, lds in LDS.items():
        def fn(i, st, lds=lds):
            b = i % 16
            assert ol.occ_launch(ar.data_ptr() + b * bb, out.data_ptr() + 2 * b * NSEG, NSEG, lds,
                                 st) == 0
        if rnd == 0:
            out.zero_()
            for i in range(16):
                fn(i, stream.cuda_stream)
            torch.cuda.synchronize()
            assert torch.equal(out, ref), wps
        ts = timer(fn, 64)
        tp = timer(fn, 64, branches=4)
        res.setdefault(wps, []).append((ts * 1e6, tp * 1e6))
        print(f"round {rnd} waves/SIMD {wps}: serial {ts * 1e6:6.2f} us  4-branch {tp * 1e6:6.2f} us",
              flush=True)
for wps, v in res.items():
    print(f"waves/SIMD {wps}: serial median {np.median([x[0] for x in v]):6.2f}  "
          f"4-branch median {np.median([x[1] for x in v]):6.2f}")
