#!/usr/bin/env python3
"""Does a launch's output store cost fixed time? (tuning tool)

Times (1) a plain 98 MB stream read with 0 / plain / nontemporal u16 stores of
65,536 results (tools/libprobe.so, built from tools/probe_kernels.hip) and
(2) the checksum kernel with plain vs nontemporal result stores.
"""
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

NSEG, L, NB = 65536, 1500, 16


def main():
    probe = C.CDLL(os.path.join(ROOT, "tools", "libprobe.so"))
    probe.probe_read_store.restype = C.c_int
    probe.probe_read_store.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                       C.c_int, C.c_uint32, C.c_void_p]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    timer = bench.Timer(torch, stream)
    bb = NSEG * L
    buf = torch.empty(NB * bb + 256, dtype=torch.uint8, device=dev)
    assert buf.numel() >= NB * bb
    csum.fill_splitmix(buf, NB * bb)
    out = torch.empty(NB * NSEG, dtype=torch.uint16, device=dev)
    B, O = buf.data_ptr(), out.data_ptr()
    work = []
    for mode in (0, 1, 2):
        for blocks in (2048, 8192):
            def fr(i, sh, mode=mode, blocks=blocks):
                b = i % NB
                probe.probe_read_store(B + b * bb, bb, O + b * NSEG * 2, NSEG, mode, blocks, sh)
            work.append((f"read store{mode} blk{blocks}", fr))
    for g, u, nt in ((16, 2, 0), (16, 2, 2), (16, 4, 1), (16, 4, 3), (32, 4, 1), (32, 4, 3)):
        t = csum.Tuning(group=g, unroll=u, nontemporal=nt, max_blocks=0)

        def fc(i, sh, t=t):
            b = i % NB
            csum.lib.tulips_csum_batch_fixed_tuned(B + b * bb, L, L, None, None, None,
                                                   O + b * NSEG * 2, NSEG, 0, t, sh)
        work.append((f"csum g{g} u{u} nt{nt}", fc))
    for _, fn in work:
        for i in range(3):
            fn(i, stream.cuda_stream)
    torch.cuda.synchronize()
    res = {}
    for r in range(5):
        for key, fn in work:
            res.setdefault(key, []).append(timer(fn, 32))
    for key, v in res.items():
        t = float(np.median(v))
        print(json.dumps({"probe": key, "us": round(t * 1e6, 2), "GBps": round(bb / t / 1e9, 1)}))


if __name__ == "__main__":
    main()
