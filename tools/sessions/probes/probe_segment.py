#!/usr/bin/env python3
"""Segmentation offload workload of bench.py's extras (1024 super-frames of
64,294 B, MSS 1460, 1536 B output slots), run REPS times back to back for a
rocprofv3 kernel trace: which of the five kernels (count, scan, add, runs,
segment) takes the time. Optional argv[1]: MSS. Calls rotate over NB
batches (input + output ~530 MB, above the 256 MB Infinity Cache) as
bench.py does."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from tulips_amd import csum  # noqa: E402


def main():
    mss = int(sys.argv[1]) if len(sys.argv) > 1 else 1460
    reps = 50
    dev = torch.device("cuda", 0)
    nsf, pay = 1024, 44 * 1460
    sflen, sslot = 54 + pay, 65536
    nb = 4
    sa = torch.empty(nb * nsf * sslot, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(sa, seed=0x7505)
    sv = sa.view(nb * nsf, sslot)
    tot = sflen - 14
    for off, val in ((12, 0x08), (13, 0), (14, 0x45), (15, 0), (16, tot >> 8),
                     (17, tot & 0xFF), (20, 0x40), (21, 0), (23, 6), (46, 0x50)):
        sv[:, off] = val
    offs = torch.arange(nsf, dtype=torch.int64, device=dev) * sslot
    lens = torch.full((nsf,), sflen - 65536, dtype=torch.int16, device=dev)
    nseg = nsf * (-(-pay // mss))
    stride = ((54 + mss + 15) // 16) * 16
    out = torch.empty(nb * nseg * stride, dtype=torch.uint8, device=dev)
    olen = torch.zeros(nseg, dtype=torch.int16, device=dev)
    first = torch.empty(nsf + 1, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    f = csum.lib.tulips_csum_segment_frames
    for i in range(reps):
        b = i % nb
        rc = f(sa.data_ptr() + b * nsf * sslot, offs.data_ptr(), lens.data_ptr(), nsf, mss,
               out.data_ptr() + b * nseg * stride, stride, nseg, olen.data_ptr(),
               first.data_ptr(), st)
        assert rc == 0
    # copy calibration: the same bytes read and written by a plain D2D copy
    # (__amd_rocclr_copyBuffer in the trace)
    nbytes = nsf * sflen
    for i in range(20):
        b = i % nb
        out[b * nseg * stride:b * nseg * stride + nbytes].copy_(
            sa[b * nsf * sslot:b * nsf * sslot + nbytes])
    torch.cuda.synchronize()
    assert int(first[nsf].item()) == nseg
    print("ok", nseg, "segments per call")


if __name__ == "__main__":
    main()
