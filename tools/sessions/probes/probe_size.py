#!/usr/bin/env python3
"""Fixed-overhead probe (tuning tool): kernel time vs batch size.

For the checksum kernel and the plain streaming read, time one launch per
batch over batch sizes 8K..512K segments (x1500 B) with rotating buffers, and
fit t = a + B/bw. `a` is the per-launch fixed cost, `bw` the streaming rate.
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


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    timer = bench.Timer(torch, stream)
    lib = csum.lib
    total = 1 << 31
    buf = torch.empty(total, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(buf, total)
    out = torch.empty(1 << 20, dtype=torch.uint16, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    B = buf.data_ptr()
    variants = {
        "csum g16u2": csum.Tuning(group=16, unroll=2, nontemporal=0, max_blocks=0),
        "csum g16u4nt": csum.Tuning(group=16, unroll=4, nontemporal=1, max_blocks=0),
        "csum g64u4nt": csum.Tuning(group=64, unroll=4, nontemporal=1, max_blocks=0),
    }
    sizes = [8192, 16384, 32768, 65536, 131072, 262144, 524288]
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
    rows = []
    for n in sizes:
        nbytes = n * L
        nb = min(16, total // nbytes - 1)
        if nb < 2:                      # never address past the buffer
            continue
        assert nb * nbytes + 16 <= total
        for name, t in variants.items():
            def fn(i, sh, t=t, n=n, nbytes=nbytes, nb=nb):
                lib.tulips_csum_batch_fixed_tuned(B + (i % nb) * nbytes, L, L, None, None,
                                                  None, out.data_ptr(), n, 0, t, sh)
            ts = [timer(fn, 32) for _ in range(3)]
            rows.append((name, n, nbytes, float(np.median(ts))))
        for mb in (2048, 8192):
            def fr(i, sh, nbytes=nbytes, nb=nb, mb=mb):
                lib.tulips_csum_stream_read(B + (i % nb) * nbytes, nbytes - nbytes % 16,
                                            sink.data_ptr(), mb, sh)
            ts = [timer(fr, 32) for _ in range(3)]
            rows.append((f"read mb{mb}", n, nbytes, float(np.median(ts))))
    by = {}
    for name, n, nbytes, t in rows:
        print(json.dumps({"v": name, "n": n, "MB": round(nbytes / 1e6, 1),
                          "us": round(t * 1e6, 2), "GBps": round(nbytes / t / 1e9, 1)}))
        by.setdefault(name, []).append((nbytes, t))
    for name, pts in by.items():
        x = np.array([p[0] for p in pts], dtype=np.float64)
        y = np.array([p[1] for p in pts], dtype=np.float64)
        slope, icpt = np.polyfit(x, y, 1)
        print(json.dumps({"fit": name, "fixed_us": round(icpt * 1e6, 2),
                          "stream_GBps": round(1 / slope / 1e9, 1)}))


if __name__ == "__main__":
    main()
