"""Frame kernels on bench.py's frame workload (8 bursts x 65,536 TCP frames
of 1514 B in 2 KiB slots): the library's offsets form against SLOTS mode
(tools/probes/frames_slots.hip: frame i at base + i * 2048, chunk loads
issued with the length load). Flags and fields compared with the
library's. Measurement only."""
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
ol = C.CDLL(os.path.join(HERE, "libframes_slots.so"))
ol.frames_slots.restype = C.c_int
ol.frames_slots.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p,
                            C.c_void_p, C.c_void_p]
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream()
sh = stream.cuda_stream
timer = bench.Timer(torch, stream)
nf, slot, flen, nb = 65536, 2048, 1514, 8
ar = torch.empty(nb * nf * slot, dtype=torch.uint8, device=dev)
csum.fill_splitmix(ar, seed=0xF4A3E5)
v = ar.view(nb * nf, slot)
for off, val in ((12, 0x08), (13, 0), (14, 0x45), (15, 0), (16, 1500 >> 8), (17, 1500 & 0xFF),
                 (20, 0x40), (21, 0), (23, 6), (46, 0x50)):
    v[:, off] = val
fo = torch.arange(nf, dtype=torch.int64, device=dev) * slot
fl = torch.full((nf,), flen, dtype=torch.int16, device=dev)
flags = torch.empty(nb * nf, dtype=torch.uint8, device=dev)
fields = torch.empty(nb * nf, dtype=torch.int32, device=dev)
burst = nf * slot
for i in range(nb):
    assert csum.lib.tulips_csum_generate_frames(ar.data_ptr() + i * burst, fo.data_ptr(),
                                                fl.data_ptr(), nf, None, sh) == 0
ref = torch.empty_like(fields)
for i in range(nb):
    assert csum.lib.tulips_csum_generate_fields(ar.data_ptr() + i * burst, fo.data_ptr(),
                                                fl.data_ptr(), nf,
                                                ref.data_ptr() + 4 * i * nf, None, sh) == 0
torch.cuda.synchronize()
FORMS = ("offsets", "slots")
lib = csum.lib
res = {}
for rnd in range(3):
    for op, name in ((0, "validate"), (1, "generate"), (2, "fields")):
        for wps in FORMS:
            def fn(i, st, op=op, form=wps):
                b = i % nb
                if form == "slots":
                    assert ol.frames_slots(op, ar.data_ptr() + b * burst, slot, fl.data_ptr(), nf,
                                           flags.data_ptr() + b * nf,
                                           fields.data_ptr() + 4 * b * nf, st) == 0
                elif op == 0:
                    assert lib.tulips_csum_validate_frames(ar.data_ptr() + b * burst, fo.data_ptr(),
                                                           fl.data_ptr(), nf,
                                                           flags.data_ptr() + b * nf, None,
                                                           st) == 0
                elif op == 1:
                    assert lib.tulips_csum_generate_frames(ar.data_ptr() + b * burst, fo.data_ptr(),
                                                           fl.data_ptr(), nf,
                                                           flags.data_ptr() + b * nf, st) == 0
                else:
                    assert lib.tulips_csum_generate_fields(ar.data_ptr() + b * burst, fo.data_ptr(),
                                                           fl.data_ptr(), nf,
                                                           fields.data_ptr() + 4 * b * nf, None,
                                                           st) == 0
            if rnd == 0:
                for i in range(nb):
                    fn(i, sh)
                torch.cuda.synchronize()
                if op == 2:
                    assert torch.equal(fields, ref), wps
                else:
                    assert bool((flags == 0x0F).all().item()), (name, wps)
            ts = timer(fn, 64)
            tp = timer(fn, 64, branches=4)
            res.setdefault((name, wps), []).append((ts * 1e6, tp * 1e6))
            print(f"round {rnd} {name:8s} {wps:8s}: serial {ts * 1e6:6.2f} us  "
                  f"4-branch {tp * 1e6:6.2f} us", flush=True)
for (name, wps), v in res.items():
    print(f"{name:8s} {wps:8s}: serial median {np.median([x[0] for x in v]):6.2f}  "
          f"4-branch median {np.median([x[1] for x in v]):6.2f}")
