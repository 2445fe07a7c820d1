#!/usr/bin/env python3
"""A short workload for instruction-counter passes (run under rocprofv3
--pmc): 16 launches each of the F1500 checksum, frame validation, the
frames' slot-read pattern and the ZIPF arena kernel, bench.py's shapes. Measurement only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from tulips_amd import csum  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    lib = csum.lib
    NSEG, SEG = bench.NSEG, bench.SEG
    bb = NSEG * SEG
    a = torch.empty(4 * bb + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(a, 4 * bb)
    o = torch.empty(4 * NSEG, dtype=torch.uint16, device=dev)
    for i in range(16):
        b = i % 4
        lib.tulips_csum_batch_fixed(a.data_ptr() + b * bb, SEG, SEG, None, None, None,
                                    o.data_ptr() + b * NSEG * 2, NSEG, 0, st)
    nf, slot, flen = 65536, 2048, 1514
    ar = torch.empty(2 * nf * slot, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(ar, seed=0xF4A3E5)
    v = ar.view(2 * nf, slot)
    for off, val in ((12, 0x08), (13, 0), (14, 0x45), (15, 0), (16, 1500 >> 8),
                     (17, 1500 & 0xFF), (20, 0x40), (21, 0), (23, 6), (46, 0x50)):
        v[:, off] = val
    offs = torch.arange(nf, dtype=torch.int64, device=dev) * slot
    lens = torch.full((nf,), flen, dtype=torch.int16, device=dev)
    flags = torch.empty(2 * nf, dtype=torch.uint8, device=dev)
    for b in range(2):
        lib.tulips_csum_generate_frames(ar.data_ptr() + b * nf * slot, offs.data_ptr(),
                                        lens.data_ptr(), nf, None, st)
    for i in range(16):
        b = i % 2
        lib.tulips_csum_validate_frames(ar.data_ptr() + b * nf * slot, offs.data_ptr(),
                                        lens.data_ptr(), nf, flags.data_ptr() + b * nf, None, st)
    # the frames' own load pattern without their work (the read ceiling)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    for i in range(16):
        b = i % 2
        lib.tulips_csum_stream_read_slots(ar.data_ptr() + b * nf * slot, slot, flen, nf,
                                          sink.data_ptr(), st)
    lz = bench.zipf_lengths(NSEG)
    zo = np.zeros(NSEG, dtype=np.uint64)
    np.cumsum(lz[:-1], dtype=np.uint64, out=zo[1:])
    zb = int(lz.astype(np.int64).sum())
    az = torch.empty(zb + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(az, zb)
    doffs = torch.from_numpy(zo.view(np.int64)).to(dev)
    dlens = torch.from_numpy(lz).to(dev)
    oz = torch.empty(NSEG, dtype=torch.uint16, device=dev)
    for i in range(16):
        lib.tulips_csum_batch_arena(az.data_ptr(), zb, doffs.data_ptr(), dlens.data_ptr(),
                                    None, None, None, oz.data_ptr(), NSEG, 0, st)
    torch.cuda.synchronize()
    ok = bool((flags == 0x0F).all().item())
    print("pmc target done, flags ok" if ok else "pmc target: FLAGS MISMATCH", flush=True)


if __name__ == "__main__":
    main()
