"""Launches every span_tb.hip variant 32 times over 8 rotated ZIPF copies,
for a rocprofv3 --pmc pass (one counter set per run):
  rocprofv3 --pmc FETCH_SIZE -d gpurun_out/tbpmc_fetch -o run -- python tools/probes/span_tb_pmc.py
Kernels are told apart by name (the workgroup size is a template
argument). Measurement only."""
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
sl = C.CDLL(os.path.join(HERE, "libspan_tb.so"))
sl.span_early_launch.restype = C.c_int
sl.span_early_launch.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p,
                                 C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p]
dev = torch.device("cuda", 0)
NSEG = 65536
lens = bench.zipf_lengths(NSEG)
offs = np.zeros(NSEG, dtype=np.uint64)
np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
zb = int(lens.astype(np.int64).sum())
nz = 8
az = torch.empty(nz * zb + 256, dtype=torch.uint8, device=dev)
csum.fill_splitmix(az, nz * zb)
do = torch.from_numpy(offs.view(np.int64)).to(dev)
dl = torch.from_numpy(lens.view(np.int16).copy()).to(dev)
oz = torch.empty(nz * NSEG, dtype=torch.int16, device=dev)
slots = torch.zeros(1 << 18, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream().cuda_stream
for var in [int(x) for x in os.environ.get("VARIANTS", "0,1,2").split(",")]:
    for i in range(32):
        b = i % nz
        assert sl.span_early_launch(az.data_ptr() + b * zb, zb, do.data_ptr(), dl.data_ptr(),
                                    None, None, oz.data_ptr() + 2 * b * NSEG, NSEG, 0,
                                    slots.data_ptr(), 1 << 18, 0x5eed, var, st) == 0
    torch.cuda.synchronize()
print("done", zb)
