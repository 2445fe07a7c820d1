#!/usr/bin/env python3
"""Where the arena-span kernel's time goes on the §8c ZIPF batch: the product
kernel vs diagnostic builds that stop after staging the chunks in LDS
(tools/libcsum_spandiag1.so: no offsets window; 2, 3: with it), before the
segment pass (4; the boundary-slot form: once its slots are filled) or that
skip the result stores (5) or store each workgroup's results to a 256-byte
block of its own (6, v5 only), and the plain streaming read of the same bytes;
serial and 4-branch pipelined. `g` = tuning group: 2 = v5 (product), 4 =
boundary-slot form."""
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


def load(path):
    lib = C.CDLL(path)
    for name, (res, argt) in csum._SIGNATURES.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, argt
    return lib


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    timer = bench.Timer(torch, stream)
    n = 65536
    lens = bench.zipf_lengths(n)
    offs = np.zeros(n, np.uint64)
    np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    nb = int(lens.astype(np.int64).sum())
    NB = int(os.environ.get("PROBE_NB", "8"))  # 8 copies: past the 256 MB MALL
    arena = torch.empty(NB * nb + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(arena, NB * nb)
    doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
    dlens = torch.from_numpy(lens.view(np.int16)).to(dev)
    out = torch.empty(NB * n, dtype=torch.uint16, device=dev)
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)
    libs = {"product": csum.lib,
            "diag1": load(os.path.join(ROOT, "tools", "libcsum_spandiag1.so")),
            "diag2": load(os.path.join(ROOT, "tools", "libcsum_spandiag2.so")),
            "diag3": load(os.path.join(ROOT, "tools", "libcsum_spandiag3.so")),
            "diag4": load(os.path.join(ROOT, "tools", "libcsum_spandiag4.so")),
            "diag5": load(os.path.join(ROOT, "tools", "libcsum_spandiag5.so")),
            "diag6": load(os.path.join(ROOT, "tools", "libcsum_spandiag6.so"))}
    row = {"n": n, "bytes": nb}
    geoms = [tuple(int(x) for x in g.split(":"))
             for g in os.environ.get("PROBE_SPAN", "8:2,8:4").split(",")]
    for u, hr in geoms:
        t = csum.Tuning(kind=csum.KIND_SPAN, unroll=u, group=hr, nontemporal=1)
        for lname, lib in list(libs.items()) + [("product_ntstore", csum.lib)]:
            if lname == "product_ntstore":
                t = csum.Tuning(kind=csum.KIND_SPAN, unroll=u, group=hr, nontemporal=3)
            def fn(i, sh, lib=lib, t=t):
                b = i % NB
                assert lib.tulips_csum_batch_arena_tuned(
                    arena.data_ptr() + b * nb, nb, doffs.data_ptr(), dlens.data_ptr(), None,
                    None, None, out.data_ptr() + b * n * 2, n, 0, t, sh) == 0
            for i in range(NB):
                fn(i, stream.cuda_stream)
            ts = float(np.median([timer(fn, 64) for _ in range(3)]))
            tp = float(np.median([timer(fn, 64, branches=4) for _ in range(3)]))
            row[f"span{u}g{hr}_{lname}"] = [round(ts * 1e6, 2), round(tp * 1e6, 2)]

    def fr(i, sh):
        b = i % NB
        assert csum.lib.tulips_csum_stream_read(arena.data_ptr() + b * (nb & ~15), nb & ~15,
                                                sink.data_ptr(), 0, sh) == 0
    ts = float(np.median([timer(fr, 64) for _ in range(3)]))
    tp = float(np.median([timer(fr, 64, branches=4) for _ in range(3)]))
    row["stream_read"] = [round(ts * 1e6, 2), round(tp * 1e6, 2)]
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
