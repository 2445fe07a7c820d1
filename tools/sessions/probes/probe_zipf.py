#!/usr/bin/env python3
"""Where does the ZIPF batch's time go? (tuning tool)

Same byte volume, different shapes:
  fixed668   fixed kernel, 65,536 x 668 B (Zipf mean), no metadata arrays
  var668     variable-length kernel on the same segments (offsets/lengths)
  zipf       the real Zipf batch
  zipf<=1K   Zipf lengths clipped to 1024 (no long tail)
  zipf x8    8 Zipf batches in ONE launch (524,288 segments): fixed vs per-byte
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

N = 65536


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    timer = bench.Timer(torch, stream)
    lib = csum.lib
    zl = bench.zipf_lengths(N)
    shapes = {
        "var668": np.full(N, 668, np.uint16),
        "zipf": zl,
        "zipf<=1K": np.minimum(zl, 1024).astype(np.uint16),
        "zipf x8": np.tile(zl, 8),
    }
    arena_bytes = 8 * int(zl.astype(np.int64).sum()) + 4096
    buf = torch.empty(arena_bytes, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(buf, arena_bytes)
    out = torch.empty(8 * N, dtype=torch.uint16, device=dev)
    B, O = buf.data_ptr(), out.data_ptr()
    work = []
    for g, u in ((16, 4), (8, 4)):
        if g == 16:
            t = csum.Tuning(group=16, unroll=4, nontemporal=1, max_blocks=0)

            def ff(i, sh, t=t):
                lib.tulips_csum_batch_fixed_tuned(B, 668, 668, None, None, None, O, N, 0, t, sh)
            work.append(("fixed668 g16u4", ff, N * 668))
    for name, lens in shapes.items():
        offs = np.zeros(len(lens), np.uint64)
        np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
        total = int(lens.astype(np.int64).sum())
        assert total + 16 <= arena_bytes
        doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
        dlens = torch.from_numpy(lens).to(dev)
        for g, u in ((-16, 4), (-8, 8), (16, 4), (64, 4)):
            t = csum.Tuning(group=g, unroll=u, nontemporal=1, max_blocks=0)

            def fv(i, sh, t=t, doffs=doffs, dlens=dlens, n=len(lens)):
                lib.tulips_csum_batch_tuned(B, doffs.data_ptr(), dlens.data_ptr(), None, None,
                                            None, O, n, 0, t, sh)
            work.append((f"{name} g{g}u{u}", fv, total))
    for _, fn, _ in work:
        fn(0, stream.cuda_stream)
    torch.cuda.synchronize()
    res = {}
    for r in range(5):
        for key, fn, nbytes in work:
            res.setdefault(key, []).append(timer(fn, 16))
    for key, fn, nbytes in work:
        t = float(np.median(res[key]))
        print(json.dumps({"probe": key, "us": round(t * 1e6, 2),
                          "GBps": round(nbytes / t / 1e9, 1)}))


if __name__ == "__main__":
    main()
