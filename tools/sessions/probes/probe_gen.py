#!/usr/bin/env python3
"""Launch time vs batch size for the variable-length kernels on Zipf lengths
(the first n of the §8c sequence): a jump where the grid outgrows one
resident generation of waves (8 per SIMD) shows a second generation."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tulips_amd import csum  # noqa: E402
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    timer = bench.Timer(torch, stream)
    lib = csum.lib
    NB = int(os.environ.get("PROBE_NB", "8"))  # 8 copies: past the 256 MB MALL
    NMAX = 98304
    lens_all = bench.zipf_lengths(NMAX)
    geoms = {"span8": ("span", 8, 2), "split6": ("span", 6), "s2_8h2": ("span", 8, 4), "s2_8h1": ("span", 8, 5),
             "s2_6h2": ("span", 6, 4), "s2_10h2": ("span", 10, 4),
             "s3_4": ("span", 4, 6), "s3_5": ("span", 5, 6), "s3_6": ("span", 6, 6),
             "s3_7": ("span", 7, 6), "s3_8": ("span", 8, 6),
             "s3_10": ("span", 10, 6),
             "s4_5": ("span", 5, 7), "s4_6": ("span", 6, 7), "s4_7": ("span", 7, 7),
             "s4_8": ("span", 8, 7), "s4_6t": ("span", 6, 7, 0), "s4_8t": ("span", 8, 7, 0),
             "packed8x4pf": csum.Tuning(kind=csum.KIND_PACKED, group=8, unroll=4, nontemporal=1,
                                        block=256, sps=2),
             }
    if os.environ.get("PROBE_UNIFORM"):
        lens_all = np.full(NMAX, int(os.environ["PROBE_UNIFORM"]), np.uint16)
    out = torch.empty(NB * NMAX, dtype=torch.uint16, device=dev)
    sizes = [int(x) for x in os.environ.get("PROBE_SIZES", "1024,8192,32768,65536,98304").split(",")]
    for n in sizes:
        lens = lens_all[:n]
        offs = np.zeros(n, np.uint64)
        np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
        nb = int(lens.astype(np.int64).sum())
        arena = torch.empty(NB * nb + 256, dtype=torch.uint8, device=dev)
        csum.fill_splitmix(arena, NB * nb)
        doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
        dlens = torch.from_numpy(lens.view(np.int16)).to(dev)
        row = {"n": n, "bytes": nb}
        only = os.environ.get("PROBE_GEOMS")
        for gname, t in geoms.items():
            if only and gname not in only.split(","):
                continue
            if isinstance(t, tuple):
                t = csum.Tuning(kind=csum.KIND_SPAN, unroll=t[1],
                                group=t[2] if len(t) > 2 else 0,
                                nontemporal=t[3] if len(t) > 3 else 1)

                def fn(i, sh, t=t):
                    b = i % NB
                    assert lib.tulips_csum_batch_arena_tuned(
                        arena.data_ptr() + b * nb, nb, doffs.data_ptr(), dlens.data_ptr(),
                        None, None, None, out.data_ptr() + b * n * 2, n, 0, t, sh) == 0
            else:
                def fn(i, sh, t=t):
                    b = i % NB
                    assert lib.tulips_csum_batch_tuned(
                        arena.data_ptr() + b * nb, doffs.data_ptr(), dlens.data_ptr(), None,
                        None, None, out.data_ptr() + b * n * 2, n, 0, t, sh) == 0
            for i in range(NB):
                fn(i, stream.cuda_stream)
            tm = float(np.median([timer(fn, 64) for _ in range(3)]))
            row[gname] = round(tm * 1e6, 2)
            if os.environ.get("PROBE_PIPE"):
                tp = float(np.median([timer(fn, 64, branches=4) for _ in range(3)]))
                row[gname + "_pipe4"] = round(tp * 1e6, 2)
        print(json.dumps(row), flush=True)
        del arena


if __name__ == "__main__":
    main()
