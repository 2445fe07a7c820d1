#!/usr/bin/env python3
"""Frame generation's field stores, A/B on the bench workload (8 bursts x
65,536 TCP frames of 1514 B in 2 KiB slots): the product's 2-byte field
stores vs diagnostic builds writing whole 16-byte chunks (genstore1) or the
frame's whole first 64-byte line (genstore2). Each variant's output frames
must equal the product's byte for byte. Serial and 4-branch pipelined
per-launch times."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tulips_amd import csum  # noqa: E402
import bench  # noqa: E402


def load(path):
    lib = C.CDLL(path)
    for name, (res, argt) in csum._SIGNATURES.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, argt
    return lib


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    timer = bench.Timer(torch, stream)
    nf, slot, flen, nb = 65536, 2048, 1514, 8
    ar = torch.empty(nb * nf * slot, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(ar, seed=0xF4A3E5)
    v = ar.view(nb * nf, slot)
    for off, val in ((12, 0x08), (13, 0), (14, 0x45), (15, 0), (16, 1500 >> 8),
                     (17, 1500 & 0xFF), (20, 0x40), (21, 0), (23, 6), (46, 0x50)):
        v[:, off] = val
    pristine = ar.clone()
    offs = torch.arange(nf, dtype=torch.int64, device=dev) * slot
    lens = torch.full((nf,), flen, dtype=torch.int16, device=dev)
    # odd-aligned frames too (fields straddling dwords/chunks) for parity
    offs_odd = offs + 7
    libs = {"product": csum.lib}
    for k in (4,):
        p = os.path.join(ROOT, "tools", f"libcsum_genstore{k}.so")
        if os.path.exists(p):
            libs[f"genstore{k}"] = load(p)
    ref = {}
    row = {}
    for name, lib in libs.items():
        for tag, o in (("aligned", offs), ("odd", offs_odd)):
            ar.copy_(pristine)
            assert lib.tulips_csum_generate_frames(ar.data_ptr(), o.data_ptr(), lens.data_ptr(),
                                                   nf, None, stream.cuda_stream) == 0
            torch.cuda.synchronize()
            h = ar[: nf * slot].cpu().numpy()
            if name == "product":
                ref[tag] = h
            else:
                row[f"{name}_{tag}_parity"] = "ok" if np.array_equal(h, ref[tag]) else "MISMATCH"
        ar.copy_(pristine)

        def fgen(i, st, lib=lib):
            b = i % nb
            lib.tulips_csum_generate_frames(ar.data_ptr() + b * nf * slot, offs.data_ptr(),
                                            lens.data_ptr(), nf, None, st)
        for i in range(nb):
            fgen(i, stream.cuda_stream)
        ts = float(np.median([timer(fgen, 64) for _ in range(3)]))
        tp = float(np.median([timer(fgen, 64, branches=4) for _ in range(3)]))
        row[name] = [round(ts * 1e6, 2), round(tp * 1e6, 2),
                     round(nf * flen / ts / 8e12, 4)]
        if name == "product":
            # temporal loads throughout (runtime knob)
            t0 = csum.Tuning(group=16, unroll=6, nontemporal=0)

            def fgt(i, st, t0=t0):
                b = i % nb
                lib.tulips_csum_frames_tuned(1, ar.data_ptr() + b * nf * slot, offs.data_ptr(),
                                             lens.data_ptr(), nf, None, None, t0, st)
            ts = float(np.median([timer(fgt, 64) for _ in range(3)]))
            tp = float(np.median([timer(fgt, 64, branches=4) for _ in range(3)]))
            row["product_temporal"] = [round(ts * 1e6, 2), round(tp * 1e6, 2),
                                       round(nf * flen / ts / 8e12, 4)]
            # capped grids: several frames per subgroup, a frame's field
            # stores in flight while the next frame streams in
            for mb, blk in ():
                tc = csum.Tuning(group=16, unroll=6, nontemporal=1, max_blocks=mb, block=blk)

                def fgc(i, st, tc=tc):
                    b = i % nb
                    assert lib.tulips_csum_frames_tuned(
                        1, ar.data_ptr() + b * nf * slot, offs.data_ptr(), lens.data_ptr(), nf,
                        None, None, tc, st) == 0
                ts = float(np.median([timer(fgc, 64) for _ in range(3)]))
                tp = float(np.median([timer(fgc, 64, branches=4) for _ in range(3)]))
                row[f"product_cap{mb}x{blk}"] = [round(ts * 1e6, 2), round(tp * 1e6, 2),
                                                 round(nf * flen / ts / 8e12, 4)]
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
