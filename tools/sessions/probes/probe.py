#!/usr/bin/env python3
"""Diagnostic probes for the F1500 gap (tuning tool, not a test).

Separates per-launch ramp cost, alignment and per-segment overhead:
  F1500 x1     one 98 MB batch per launch (the bench step)
  F1500 x16    all 16 batches (1.57 GB) in ONE launch
  F1536        16-byte-multiple length and stride (no boundary fix-up)
  F1500s2048   OFED-like 2048 B stride
  READ 98MB    plain stream read of one 98 MB batch per launch
  READ 1.5GB   plain stream read of the whole shard per launch
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tulips_amd import csum  # noqa: E402
import bench  # noqa: E402

NSEG = 65536


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    timer = bench.Timer(torch, stream)
    lib = csum.lib
    total = 16 * NSEG * 2048 + 4096
    buf = torch.empty(total, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(buf, total)
    out = torch.empty(16 * NSEG, dtype=torch.uint16, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    B, O = buf.data_ptr(), out.data_ptr()
    geoms = [(16, 4, 1), (16, 2, 0), (32, 4, 1), (64, 8, 1), (64, 4, 1)]
    work = []
    for g, u, nt in geoms:
        t = csum.Tuning(group=g, unroll=u, nontemporal=nt, max_blocks=0)
        for name, L, stride, n, nb in (("F1500x1", 1500, 1500, NSEG, 16),
                                       ("F1500x16", 1500, 1500, 16 * NSEG, 1),
                                       ("F1536", 1536, 1536, NSEG, 16),
                                       ("F1500s2048", 1500, 2048, NSEG, 16),
                                       ("F9000", 9000, 9000, NSEG, 3)):
            def fn(i, sh, t=t, L=L, stride=stride, n=n, nb=nb):
                b = i % nb
                lib.tulips_csum_batch_fixed_tuned(B + b * n * stride, stride, L, None, None,
                                                  None, O, n, 0, t, sh)
            work.append((f"{name} g{g} u{u} nt{nt}", fn, n * L, 32 if n == NSEG else 4))
    for name, nbytes, nb in (("READ 98MB", NSEG * 1500, 16), ("READ 1.57GB", 16 * NSEG * 1500, 1)):
        def fr(i, sh, nbytes=nbytes, nb=nb):
            b = i % nb
            lib.tulips_csum_stream_read(B + b * nbytes, nbytes, sink.data_ptr(), 8192, sh)
        work.append((name, fr, nbytes, 32 if nb > 1 else 4))
    res = {}
    for key, fn, nbytes, reps in work:
        for i in range(3):
            fn(i, stream.cuda_stream)
    torch.cuda.synchronize()
    for r in range(5):
        for key, fn, nbytes, reps in work:
            t = timer(fn, reps)
            res.setdefault(key, []).append((nbytes / t / 1e9, t * 1e6))
    for key, v in res.items():
        gb = [x[0] for x in v]
        us = [x[1] for x in v]
        print(json.dumps({"probe": key, "GBps_median": round(float(np.median(gb)), 1),
                          "us_median": round(float(np.median(us)), 2)}))


if __name__ == "__main__":
    main()
