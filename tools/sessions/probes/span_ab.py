"""A/B of arena span-kernel variants on the ZIPF batch (configs[3]): tuning
group 0 (product), 8 (contiguous XCD eighths), 9 (early word guess, no
re-zero), 10 (both); 8 rotated copies, serial chain and 4 graph branches,
three alternations; parity against the reference ZIPF digest."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from tulips_amd import csum  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
stream = torch.cuda.current_stream()
timer = bench.Timer(torch, stream)
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
oz = torch.empty(nz * NSEG, dtype=torch.uint16, device=dev)
gold = bench.golden_digests()["ZIPF"]["fnv1a64"]
res = {}
for rnd in range(3):
    for grp in (0, 8, 9, 10):
        t = csum.Tuning(kind=csum.KIND_SPAN, unroll=6, group=grp, nontemporal=1)

        def fz(i, st, t=t):
            b = i % nz
            assert csum.lib.tulips_csum_batch_arena_tuned(
                az.data_ptr() + b * zb, zb, doffs.data_ptr(), dlens.data_ptr(), None, None,
                None, oz.data_ptr() + b * NSEG * 2, NSEG, 0, C.byref(t), st) == 0
        for i in range(nz):
            fz(i, stream.cuda_stream)
        ts = timer(fz, 80)
        tp = timer(fz, 80, branches=4)
        ok = bench.fnv1a_u16(oz[:NSEG].cpu().numpy().view(np.uint16)) == gold
        res.setdefault(grp, []).append((ts * 1e6, tp * 1e6, ok))
        print(f"round {rnd} group {grp:2d}: serial {ts * 1e6:6.2f} us  4-branch {tp * 1e6:6.2f} us "
              f"parity {'ok' if ok else 'MISMATCH'}", flush=True)
for grp, v in res.items():
    s = sorted(x[0] for x in v)
    p = sorted(x[1] for x in v)
    print(f"group {grp:2d}: serial median {s[1]:.2f} (min {s[0]:.2f}) 4-branch median {p[1]:.2f} "
          f"(min {p[0]:.2f})")
