#!/usr/bin/env python3
"""Geometry sweep of the checksum kernels on one MI355X (tuning tool).

Times every (group, unroll, nontemporal, max_blocks) variant on the F1500,
F9000 and ZIPF workloads with HIP events on the launch stream, interleaving
variants over several rounds in one process (methodology rule: perf deltas
come from interleaved rounds), and prints one JSON line per variant with the
median and min over rounds.
"""
import argparse
import itertools
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

NSEG = 65536


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--reps", type=int, default=48)
    p.add_argument("--only", default="F1500,F9000,ZIPF,READ")
    a = p.parse_args()
    only = set(a.only.split(","))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    timer = bench.Timer(torch, stream)
    lib = csum.lib
    results = {}

    def record(key, t, nbytes):
        results.setdefault(key, []).append(nbytes / t / 1e9)

    work = []
    if "F1500" in only or "F9000" in only:
        for L, nb in ((1500, 16), (9000, 3)):
            if f"F{L}" not in only:
                continue
            bb = NSEG * L
            buf = torch.empty(nb * bb + 256, dtype=torch.uint8, device=dev)
            csum.fill_splitmix(buf, nb * bb)
            out = torch.empty(nb * NSEG, dtype=torch.uint16, device=dev)
            for g, u, nt, mb in itertools.product((16, 32, 64), (2, 4, 8), (0, 1),
                                                  (0, 1024, 2048)):
                t = csum.Tuning(group=g, unroll=u, nontemporal=nt, max_blocks=mb)

                def fn(i, sh, buf=buf, out=out, t=t, L=L, bb=bb, nb=nb):
                    b = i % nb
                    lib.tulips_csum_batch_fixed_tuned(buf.data_ptr() + b * bb, L, L, None,
                                                      None, None, out.data_ptr() + b * NSEG * 2,
                                                      NSEG, 0, t, sh)
                work.append((f"F{L} g{g} u{u} nt{nt} mb{mb}", fn, bb))
    if "ZIPF" in only:
        lens = bench.zipf_lengths(NSEG)
        offs = np.zeros(NSEG, dtype=np.uint64)
        np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
        zb = int(lens.astype(np.int64).sum())
        nz = 8
        zbuf = torch.empty(nz * zb + 256, dtype=torch.uint8, device=dev)
        csum.fill_splitmix(zbuf, nz * zb)
        doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
        dlens = torch.from_numpy(lens).to(dev)
        zout = torch.empty(nz * NSEG, dtype=torch.uint16, device=dev)
        S, H = csum.KIND_SUBGROUP, KIND_HYBRID
        geoms = [(S, g, u, 1) for g in (16, 32, 64) for u in (4, 8)]
        geoms += [(H, 8, 4, 1), (H, 8, 4, 2), (H, 8, 4, 4), (H, 8, 8, 1), (H, 16, 2, 1),
                  (H, 16, 2, 2), (H, 16, 2, 4), (H, 16, 4, 1), (H, 16, 4, 2), (H, 16, 8, 1),
                  (H, 32, 4, 1)]
        for (k, g, u, sps), nt in itertools.product(geoms, (0, 1)):
            t = csum.Tuning(kind=k, group=g, unroll=u, nontemporal=nt, sps=sps)

            def fz(i, sh, t=t):
                b = i % nz
                lib.tulips_csum_batch_tuned(zbuf.data_ptr() + b * zb, doffs.data_ptr(),
                                            dlens.data_ptr(), None, None, None,
                                            zout.data_ptr() + b * NSEG * 2, NSEG, 0, t, sh)
            work.append((f"ZIPF k{k} g{g} u{u} s{sps} nt{nt}", fz, zb))
    if "READ" in only:
        rb = 16 * NSEG * 1500
        rbuf = torch.empty(rb, dtype=torch.uint8, device=dev)
        csum.fill_splitmix(rbuf, rb)
        sink = torch.zeros(4, dtype=torch.int32, device=dev)
        for mb in (1024, 2048, 4096, 8192, 16384):
            def fr(i, sh, mb=mb):
                lib.tulips_csum_stream_read(rbuf.data_ptr(), rb, sink.data_ptr(), mb, sh)
            work.append((f"READ mb{mb}", fr, rb))

    for key, fn, nbytes in work:     # warm every variant once
        for i in range(4):
            fn(i, sh)
    torch.cuda.synchronize()
    for r in range(a.rounds):
        for key, fn, nbytes in work:
            reps = a.reps if not key.startswith("READ") else max(4, a.reps // 8)
            record(key, timer(fn, reps), nbytes)
        print(f"round {r} done", file=sys.stderr, flush=True)
    rows = []
    for key, v in results.items():
        rows.append({"variant": key, "GBps_median": round(float(np.median(v)), 1),
                     "GBps_max": round(float(np.max(v)), 1)})
    rows.sort(key=lambda x: (x["variant"].split()[0], -x["GBps_median"]))
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
