#!/usr/bin/env python3
"""Per-wave life times of the variable-length kernels on the ZIPF batch
(diagnostic; tools/libcsum_stamps.so). For the PACKED kernel every wave owns
`group` consecutive segments, so its bytes are known: reports how wave life
grows with wave bytes and what the slowest waves carry."""
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

N, NB = 65536, 8


def main():
    lib = C.CDLL(os.path.join(ROOT, "tools", "libcsum_stamps.so"))
    for name, (res, argt) in csum._SIGNATURES.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, argt
    lib.tulips_csum_stamps_arm.restype = C.c_int
    lib.tulips_csum_stamps_arm.argtypes = [C.c_void_p]
    lib.tulips_csum_stamps_count.restype = C.c_uint32
    dev = torch.device("cuda", 0)
    lens = bench.zipf_lengths(N)
    if os.environ.get("PROBE_LENS") == "v668":
        lens = np.full(N, 668, np.uint16)
    offs = np.zeros(N, np.uint64)
    np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    nb = int(lens.astype(np.int64).sum())
    buf = torch.empty(NB * nb + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(buf, NB * nb)
    doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
    dlens = torch.from_numpy(lens).to(dev)
    out = torch.empty(N, dtype=torch.uint16, device=dev)
    stamps = torch.zeros(4 * 300000, dtype=torch.int64, device=dev)
    sh = torch.cuda.current_stream().cuda_stream
    chunks = ((offs % 16) + lens + 15) // 16 * (lens > 0)
    for s_, u_, sps, blk in ((8, 4, 1, 256), (8, 4, 2, 256), (8, 4, 2, 1024)):
        t = csum.Tuning(kind=csum.KIND_PACKED, group=s_, unroll=u_, nontemporal=1, sps=sps,
                        block=blk)
        for i in range(NB):
            lib.tulips_csum_batch_tuned(buf.data_ptr() + (i % NB) * nb, doffs.data_ptr(),
                                        dlens.data_ptr(), None, None, None, out.data_ptr(),
                                        N, 0, C.byref(t), sh)
        torch.cuda.synchronize()
        assert lib.tulips_csum_stamps_arm(stamps.data_ptr()) == 0
        lib.tulips_csum_batch_tuned(buf.data_ptr() + 3 * nb, doffs.data_ptr(),
                                    dlens.data_ptr(), None, None, None, out.data_ptr(), N, 0,
                                    C.byref(t), sh)
        torch.cuda.synchronize()
        n = lib.tulips_csum_stamps_count()
        st = stamps[: 4 * n].cpu().numpy().reshape(n, 4)
        t0 = (st[:, 0] - st[:, 0].min()) / 100.0
        t1 = (st[:, 1] - st[:, 0].min()) / 100.0
        life = t1 - t0
        wchunks = np.add.reduceat(chunks, np.arange(0, N, s_))[:n]
        order = np.argsort(wchunks)
        deciles = np.array_split(order, 10)
        grid = np.arange(0, t1.max() + 0.01, 0.01)
        alive = np.array([((t0 <= x) & (t1 > x)).sum() for x in grid])
        rep = {
            "geom": f"packed{s_}x{u_}b{blk}" + ("pf" if sps == 2 else ""), "waves": int(n), "span_us": round(float(t1.max()), 2),
            "alive_max": int(alive.max()),
            "started_by_us": [[x, int((t0 <= x).sum())] for x in (0.5, 1, 1.5, 2, 4, 6, 8, 10)],
            "xcc_waves": np.bincount(st[:, 2].astype(np.int64) & 15, minlength=8).tolist(),
            "cu_ids": int(len(np.unique(st[:, 3] >> 8))),
            "start_p50_p99_max": [round(float(np.percentile(t0, q)), 2) for q in (50, 99, 100)],
            "end_p50_p99_max": [round(float(np.percentile(t1, q)), 2) for q in (50, 99, 100)],
            "life_p10_p50_p90_p99_max": [round(float(np.percentile(life, q)), 2)
                                         for q in (10, 50, 90, 99, 100)],
            "life_by_bytes_decile": [[int(wchunks[d].mean() * 16), round(float(life[d].mean()), 2)]
                                     for d in deciles],
            "slowest10": [[int(wchunks[i] * 16), round(float(life[i]), 2), round(float(t0[i]), 2)]
                          for i in np.argsort(-t1)[:10]],
        }
        print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
