#!/usr/bin/env python3
"""Packed variable-length kernel with next-group metadata prefetch (sps=3)
against the double-buffered default (sps=2), on rotated ZIPF and fixed 668 B
batches (8 x 65,536 segments, HBM-resident), one launch at a time and on 4
overlapped graph branches, over grid caps (max_blocks; 2048 blocks = one
8-segment group per wave at 256 threads). Every geometry's results are
compared with the default's. Prints one JSON line per (workload, geometry).
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

N, NB = 65536, 8


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    timer = bench.Timer(torch, stream)
    lib = csum.lib
    shapes = {"zipf": bench.zipf_lengths(N), "v668": np.full(N, 668, np.uint16)}
    geoms = [("default", None)]
    for s, u in ((8, 4), (8, 2)):
        geoms.append((f"p{s}x{u}pf", csum.Tuning(kind=csum.KIND_PACKED, group=s, unroll=u,
                                                  nontemporal=1, block=256, sps=2)))
        for cap in (2048, 1792, 1024, 896, 512, 256):
            geoms.append((f"p{s}x{u}meta_cap{cap}",
                          csum.Tuning(kind=csum.KIND_PACKED, group=s, unroll=u, nontemporal=1,
                                      block=256, sps=3, max_blocks=cap)))
    out = torch.empty(NB * N, dtype=torch.uint16, device=dev)
    for name, lens in shapes.items():
        offs = np.zeros(N, np.uint64)
        np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
        nb = int(lens.astype(np.int64).sum())
        arena = torch.empty(NB * nb + 256, dtype=torch.uint8, device=dev)
        csum.fill_splitmix(arena, NB * nb)
        doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
        dlens = torch.from_numpy(lens).to(dev)
        ref = None
        for gname, t in geoms:
            def fn(i, sh, t=t):
                b = i % NB
                rc = lib.tulips_csum_batch_tuned(arena.data_ptr() + b * nb, doffs.data_ptr(),
                                                 dlens.data_ptr(), None, None, None,
                                                 out.data_ptr() + b * N * 2, N, 0, t, sh)
                assert rc == 0, rc
            out.zero_()
            for i in range(NB):
                fn(i, stream.cuda_stream)
            torch.cuda.synchronize()
            res = out.cpu().numpy()
            if ref is None:
                ref = res
            ok = bool(np.array_equal(res, ref))
            ts = float(np.median([timer(fn, 64) for _ in range(3)]))
            tp = float(np.median([timer(fn, 64, branches=4) for _ in range(3)]))
            print(json.dumps({"probe": name, "geom": gname, "us": round(ts * 1e6, 2),
                              "GBps": round(nb / ts / 1e9, 1), "pipe4_us": round(tp * 1e6, 2),
                              "pipe4_GBps": round(nb / tp / 1e9, 1), "same_as_default": ok}),
                  flush=True)
        del arena


if __name__ == "__main__":
    main()
