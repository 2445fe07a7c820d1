"""Probe of the receive-validation latency paths, C-timed
(tulips_csum_time_validate): staged vs zero-copy, bursts of 1..1024 TCP
frames of 1514 B in page-locked 2 KiB slots; TULIPS_ZC_MODE=resident picks
the resident server. Also the reference CPU verify when oracle/_ref exists."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: E402
from tulips_amd import csum  # noqa: E402
import bench  # noqa: E402

mode = os.environ.get("TULIPS_ZC_MODE", "launch")
out = (C.c_double * 5)()
with csum.HostContext(0, chunk_bytes=4 << 20) as ctx:
    for nf in (1, 8, 64, 256, 1024):
        ar, offs, lens = bench.burst_frames(nf)
        pinned = torch.from_numpy(ar).pin_memory()
        flags = np.empty(nf, np.uint8)
        for name, path in (("staged", 0), ("zero_copy", 1)):
            rc = csum.lib.tulips_csum_time_validate(ctx._h, path, pinned.data_ptr(),
                                                    offs.ctypes.data, lens.ctypes.data, nf,
                                                    1000, flags.ctypes.data, out)
            print(f"{mode:8s} {name:9s} burst {nf:5d}: rc {rc} median {out[0]:7.2f} us p99 "
                  f"{out[1]:7.2f} min {out[2]:7.2f} gpu {out[4]:6.2f} ok "
                  f"{bool((flags == 0x0F).all())}", flush=True)
try:
    from oracle import Reference
    ref = Reference()
    f = ref.lib.ref_time_verify_burst
    f.restype = C.c_uint32
    f.argtypes = [C.c_void_p] * 3 + [C.c_uint32, C.c_uint32, C.c_void_p]
    for nf in (1, 8, 64, 256, 1024):
        ar, offs, lens = bench.burst_frames(nf)
        g = f(ar.ctypes.data, offs.ctypes.data, lens.ctypes.data, nf, 5000, C.addressof(out))
        print(f"cpu-ref   burst {nf:5d}: median {out[0]:7.3f} us p99 {out[1]:7.3f} good {g}")
except Exception as e:  # noqa: BLE001
    print("no reference:", e)
