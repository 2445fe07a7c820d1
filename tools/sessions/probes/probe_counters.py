#!/usr/bin/env python3
"""Frame validation with and without the optional counters (4 x u32 device
words every frame's verdict is added to), 8 rotated bursts of 65,536 x 1514 B
frames in 2 KiB slots (bench.py's frame workload). Prints us per launch,
one launch at a time and on 4 graph branches, per variant. Then
tulips_csum_verify on an all-bad burst against the plain batch."""
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
    nf, slot, flen, nb = bench.NSEG, 2048, bench.SEG + 14, 8
    ar = torch.empty(nb * nf * slot, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(ar, seed=0xF4A3E5)
    v = ar.view(nb * nf, slot)
    for off, val in ((12, 0x08), (13, 0), (14, 0x45), (15, 0), (16, bench.SEG >> 8),
                     (17, bench.SEG & 0xFF), (20, 0x40), (21, 0), (23, 6), (46, 0x50)):
        v[:, off] = val
    offs = torch.arange(nf, dtype=torch.int64, device=dev) * slot
    lens = torch.full((nf,), flen, dtype=torch.int16, device=dev)
    flags = torch.empty(nb * nf, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(nb * 4, dtype=torch.int32, device=dev)
    burst = nf * slot
    for i in range(nb):
        lib.tulips_csum_generate_frames(ar.data_ptr() + i * burst, offs.data_ptr(),
                                        lens.data_ptr(), nf, None, stream.cuda_stream)
    for name, use in (("no_counters", False), ("counters", True), ("no_counters", False),
                      ("counters", True)):
        def fn(i, st, use=use):
            b = i % nb
            rc = lib.tulips_csum_validate_frames(
                ar.data_ptr() + b * burst, offs.data_ptr(), lens.data_ptr(), nf,
                flags.data_ptr() + b * nf, cnt.data_ptr() + 16 * b if use else None, st)
            assert rc == 0, rc
        ts = float(np.median([timer(fn, 64) for _ in range(3)]))
        tp = float(np.median([timer(fn, 64, branches=4) for _ in range(3)]))
        ok = bool((flags == 0x0F).all().item())
        c = cnt.view(nb, 4).cpu().numpy().tolist()[0]
        print(json.dumps({"variant": name, "us": round(ts * 1e6, 2), "pipe4_us": round(tp * 1e6, 2),
                          "flags_ok": ok, "counters_burst0": c if use else None}), flush=True)

    # verify (results != 0xffff counted) on an all-bad burst: 65,536 random
    # 1500 B segments through offsets, against the same batch uncounted
    n, L = bench.NSEG, bench.SEG
    arena = torch.empty(4 * n * L, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(arena, seed=0x5EED)
    voffs = torch.arange(n, dtype=torch.int64, device=dev) * L
    vlens = torch.full((n,), L, dtype=torch.int16, device=dev)
    out = torch.empty(4 * n, dtype=torch.uint16, device=dev)
    bad = torch.zeros(4, dtype=torch.int32, device=dev)
    for name in ("batch", "verify", "batch", "verify"):
        def fv(i, st, name=name):
            b = i % 4
            if name == "batch":
                rc = lib.tulips_csum_batch(arena.data_ptr() + b * n * L, voffs.data_ptr(),
                                           vlens.data_ptr(), None, None, None,
                                           out.data_ptr() + 2 * b * n, n, 1, st)
            else:
                rc = lib.tulips_csum_verify(arena.data_ptr() + b * n * L, voffs.data_ptr(),
                                            vlens.data_ptr(), None, None,
                                            out.data_ptr() + 2 * b * n, bad.data_ptr() + 4 * b,
                                            n, 1, st)
            assert rc == 0, rc
        ts = float(np.median([timer(fv, 32) for _ in range(3)]))
        print(json.dumps({"variant": f"{name}_all_bad_F1500_offsets", "us": round(ts * 1e6, 2),
                          "bad_counts": bad.cpu().numpy().tolist() if name == "verify" else None}),
              flush=True)


if __name__ == "__main__":
    main()
