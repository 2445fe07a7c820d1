#!/usr/bin/env python3
"""PACKED vs HYBRID variable-length kernels on rotated (HBM-resident) batches.

Workloads (each: 8 batches of 65,536 segments with the same lengths and
different bytes, rotated so the 256 MB Infinity Cache cannot hold them):
  zipf   SURVEY.md §8c Zipf lengths (configs[3])
  v668   fixed 668 B (the Zipf mean) through offsets/lengths
  v1500  fixed 1500 B through offsets/lengths
  v64    fixed 64 B through offsets/lengths
Prints one JSON line per (workload, geometry) with us/launch and GB/s, and
checks every geometry's results against the default geometry's.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tulips_amd import csum  # noqa: E402
# archived kinds (round 3): only builds of tools/variants/ accept them; the
# product library rejects them (InvalidArgument)
KIND_HYBRID, KIND_BALANCED = 2, 4

import bench  # noqa: E402

N, NB = 65536, 8


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    timer = bench.Timer(torch, stream)
    lib = csum.lib
    shapes = {"zipf": bench.zipf_lengths(N), "v668": np.full(N, 668, np.uint16),
              "v1500": np.full(N, 1500, np.uint16), "v64": np.full(N, 64, np.uint16)}
    geoms = [("hybrid16x4", csum.Tuning(kind=KIND_HYBRID, group=16, unroll=4,
                                        nontemporal=1, sps=1))]
    only = os.environ.get("PROBE_GEOMS")
    for s, u, blk in ((4, 4, 256), (6, 4, 256), (8, 2, 256), (8, 4, 256), (8, 4, 512),
                      (8, 4, 1024), (12, 4, 256), (16, 2, 256), (16, 4, 256), (16, 8, 256),
                      (32, 4, 256), (32, 8, 256), (64, 4, 256), (64, 8, 256)):
        key = f"packed{s}x{u}b{blk}"
        if only and key not in only.split(","):
            continue
        geoms.append((key, csum.Tuning(kind=csum.KIND_PACKED, group=s, unroll=u,
                                       nontemporal=1, block=blk)))
    # double-buffered window loop (sps=2)
    for s, u, blk in ((4, 4, 256), (6, 4, 256), (8, 2, 256), (8, 4, 256),
                      (8, 4, 1024), (16, 2, 256), (16, 4, 256), (32, 4, 256)):
        key = f"packed{s}x{u}b{blk}pf"
        if only and key not in only.split(","):
            continue
        geoms.append((key, csum.Tuning(kind=csum.KIND_PACKED, group=s, unroll=u,
                                       nontemporal=1, block=blk, sps=2)))
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
            for i in range(NB):
                fn(i, stream.cuda_stream)
            torch.cuda.synchronize()
            res = out.cpu().numpy()
            if ref is None:
                ref = res
            ok = bool(np.array_equal(res, ref))
            ts = [timer(fn, 64) for _ in range(3)]
            tm = float(np.median(ts))
            print(json.dumps({"probe": name, "geom": gname, "us": round(tm * 1e6, 2),
                              "GBps": round(nb / tm / 1e9, 1), "same_as_default": ok}),
                  flush=True)
        del arena


if __name__ == "__main__":
    main()
