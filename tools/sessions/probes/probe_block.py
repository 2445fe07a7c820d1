#!/usr/bin/env python3
"""Workgroup size vs dispatch-rate limit (tuning tool).

The per-wave stamps (tools/probe_stamps.py) showed F1500 waves living ~2.3 us
while the dispatcher refills at ~1.6 waves/ns, so only 3-4K of 8K wave slots
are busy. Larger workgroups mean fewer dispatches for the same waves.
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
    total = 16 * NSEG * 1500 + 4096
    assert total >= 2 * NSEG * 9000 + 16
    buf = torch.empty(total, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(buf, total)
    out = torch.empty(NSEG, dtype=torch.uint16, device=dev)
    B, O = buf.data_ptr(), out.data_ptr()
    lens = bench.zipf_lengths(NSEG)
    offs = np.zeros(NSEG, np.uint64)
    np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    zb = int(lens.astype(np.int64).sum())
    doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
    dlens = torch.from_numpy(lens).to(dev)
    work = []
    for blk in (256, 512, 1024):
        for name, L, nb, g, u in (("F1500", 1500, 16, 32, 4), ("F1500", 1500, 16, 16, 8),
                                  ("F1500", 1500, 16, 64, 2), ("F9000", 9000, 2, 64, 8)):
            t = csum.Tuning(group=g, unroll=u, nontemporal=1, max_blocks=0, block=blk)

            def ff(i, sh, t=t, L=L, nb=nb):
                lib.tulips_csum_batch_fixed_tuned(B + (i % nb) * NSEG * L, L, L, None, None,
                                                  None, O, NSEG, 0, t, sh)
            work.append((f"{name} g{g}u{u} blk{blk}", ff, NSEG * L))
        for g, u in ((-16, 4), (16, 4)):
            t = csum.Tuning(group=g, unroll=u, nontemporal=1, max_blocks=0, block=blk)

            def fz(i, sh, t=t):
                lib.tulips_csum_batch_tuned(B + (i % 8) * zb, doffs.data_ptr(), dlens.data_ptr(),
                                            None, None, None, O, NSEG, 0, t, sh)
            work.append((f"ZIPF g{g}u{u} blk{blk}", fz, zb))
    for _, fn, _ in work:
        fn(0, stream.cuda_stream)
    torch.cuda.synchronize()
    res = {}
    for r in range(5):
        for key, fn, nbytes in work:
            res.setdefault(key, []).append(timer(fn, 32))
    for key, fn, nbytes in work:
        t = float(np.median(res[key]))
        print(json.dumps({"probe": key, "us": round(t * 1e6, 2),
                          "GBps": round(nbytes / t / 1e9, 1)}))


if __name__ == "__main__":
    main()
