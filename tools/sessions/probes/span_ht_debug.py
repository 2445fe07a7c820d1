"""Debug helper for span-kernel variants: run one probe variant on the ZIPF
batch and list the segments whose result differs from the product's, with
their position relative to the 24 KiB ranges. Measurement/debug only."""
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
MH = int(os.environ.get("MH", "3"))
HT = int(os.environ.get("HT", "4096"))
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
NSEG = 65536
lens = bench.zipf_lengths(NSEG)
offs = np.zeros(NSEG, dtype=np.uint64)
np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
zb = int(lens.astype(np.int64).sum())
nz = 8
az = torch.empty(nz * zb + 256, dtype=torch.uint8, device=dev)
csum.fill_splitmix(az, nz * zb)
doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
dlens = torch.from_numpy(lens).to(dev)
ref = torch.zeros(NSEG, dtype=torch.uint16, device=dev)
got = torch.zeros(NSEG, dtype=torch.uint16, device=dev)
st = torch.cuda.current_stream().cuda_stream
sl = C.CDLL(os.path.join(HERE, "libspan_stamps.so"))
sl.span_probe_launch.restype = C.c_int
sl.span_probe_launch.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p,
                                 C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
ranges = zb // 24576 + 2
slots = torch.zeros(ranges, dtype=torch.int64, device=dev)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for bi in range(nz):
    base = az.data_ptr() + bi * zb
    assert csum.lib.tulips_csum_batch_arena(base, zb, doffs.data_ptr(), dlens.data_ptr(), None,
                                            None, None, ref.data_ptr(), NSEG, 0, st) == 0
    for rep in range(2):
        got.zero_()
        ev0.record()
        assert sl.span_probe_launch(base, zb, doffs.data_ptr(), dlens.data_ptr(),
                                    got.data_ptr(), NSEG, slots.data_ptr(), ranges, 7 + rep,
                                    None, 8, 1024, MH, HT, st) == 0
        ev1.record()
        torch.cuda.synchronize()
        r = ref.cpu().numpy()
        g = got.cpu().numpy()
        bad = np.nonzero(r != g)[0]
        A = base & ~15
        print(f"batch {bi} rep {rep}: {len(bad)} mismatches; base % 16 = {base & 15}; "
              f"{ev0.elapsed_time(ev1) * 1e3:.1f} us")
        W = 24576
        for i in bad[:6]:
            sa = base + int(offs[i])
            se = sa + int(lens[i])
            k0 = (sa - A) // W
            k1 = (se - 1 - A) // W
            x1 = A + (k0 + 1) * W
            print(f"  seg {i}: off {int(offs[i])} len {int(lens[i])} ranges {k0}..{k1} "
                  f"tail past first range {max(0, se - x1)} ref {r[i]:#06x} got {g[i]:#06x}")
