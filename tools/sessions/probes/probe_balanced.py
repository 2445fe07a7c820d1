#!/usr/bin/env python3
"""Workgroup-balanced (KIND_BALANCED) vs packed variable-length kernels.

Workloads: 8 rotated batches of 65,536 segments (zipf = SURVEY.md §8c,
v668 = the Zipf mean, v1500, v64) through offsets/lengths. Per geometry:
us per launch one at a time (serial chain in one HIP graph) and on 4 graph
branches, checked bit-exact against the packed default's results. One JSON
line per (workload, geometry).
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
    geoms = [("packed8x4pf", csum.Tuning(kind=csum.KIND_PACKED, group=8, unroll=4,
                                         nontemporal=1, block=256, sps=2))]
    for sg, u in ((4, 4), (8, 2), (8, 4), (16, 2), (16, 4), (32, 2)):
        geoms.append((f"vpacked{sg}x{u}",
                      csum.Tuning(kind=csum.KIND_PACKED, group=sg, unroll=u, nontemporal=1,
                                  block=256, sps=4)))
    for blk, u, sps in ((256, 2, 2), (512, 2, 2)):
        geoms.append((f"balanced{blk // 64}w_u{u}{'pp' if sps == 2 else 's'}",
                      csum.Tuning(kind=KIND_BALANCED, group=8, unroll=u,
                                  nontemporal=1, block=blk, sps=sps)))
    only = os.environ.get("PROBE_GEOMS")
    if only:
        geoms = [g for g in geoms if g[0] in only.split(",")]
    out = torch.empty(NB * N, dtype=torch.uint16, device=dev)
    for name, lens in shapes.items():
        offs = np.zeros(N, np.uint64)
        np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
        nb = int(lens.astype(np.int64).sum())
        arena = torch.empty(NB * nb + 256, dtype=torch.uint8, device=dev)
        csum.fill_splitmix(arena, NB * nb)
        doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
        dlens = torch.from_numpy(lens.view(np.int16)).to(dev)
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
            ts = [timer(fn, 64) for _ in range(3)]
            tp = [timer(fn, 64, branches=4) for _ in range(3)]
            tm, tpm = float(np.median(ts)), float(np.median(tp))
            print(json.dumps({"probe": name, "geom": gname, "us": round(tm * 1e6, 2),
                              "us_4branch": round(tpm * 1e6, 2),
                              "GBps": round(nb / tm / 1e9, 1),
                              "GBps_4branch": round(nb / tpm / 1e9, 1),
                              "parity_vs_packed": ok}), flush=True)


if __name__ == "__main__":
    main()
