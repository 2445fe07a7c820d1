#!/usr/bin/env python3
"""Fixed-length geometry probe (F1500 and F9000, rotated HBM-resident
batches): subgroup size x chunks per lane x block size (x nontemporal mode,
PROBE_NT: bit 0 loads, bit 1 stores), interleaved over rounds; every
geometry's results are checked against the default's."""
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
    geoms = [(32, 4, 256), (16, 6, 256), (32, 3, 256), (16, 8, 256), (16, 6, 512),
             (32, 3, 512), (16, 6, 1024), (64, 2, 256)]
    nts = [int(x) for x in os.environ.get("PROBE_NT", "1").split(",")]
    lens = [int(x) for x in os.environ.get("PROBE_LENS", "1500,9000").split(",")]
    if os.environ.get("PROBE_GEOMS"):
        geoms = [tuple(int(v) for v in g.split(":")) for g in os.environ["PROBE_GEOMS"].split(",")]
    for L, nb in ((1500, 16), (9000, 3)):
        if L not in lens:
            continue
        if L == 9000 and not os.environ.get("PROBE_GEOMS"):
            geoms = [(64, 8, 256), (64, 9, 256), (64, 12, 256), (64, 4, 256), (64, 9, 512)]
        bb = N * L
        buf = torch.empty(nb * bb + 256, dtype=torch.uint8, device=dev)
        csum.fill_splitmix(buf, nb * bb)
        out = torch.empty(nb * N, dtype=torch.uint16, device=dev)
        res, ref = {}, None
        for rnd in range(int(os.environ.get("ROUNDS", "3"))):
            for gm, nt in [(gm, nt) for gm in geoms for nt in nts]:
                g, u, blk = gm[:3]
                cap = gm[3] if len(gm) > 3 else 0    # g:u:block[:max_blocks]
                t = csum.Tuning(group=g, unroll=u, nontemporal=nt, block=blk, max_blocks=cap)

                def fn(i, sh, t=t):
                    b = i % nb
                    rc = lib.tulips_csum_batch_fixed_tuned(buf.data_ptr() + b * bb, L, L, None,
                                                           None, None,
                                                           out.data_ptr() + b * N * 2, N, 0,
                                                           t, sh)
                    assert rc == 0, rc
                for i in range(nb):
                    fn(i, stream.cuda_stream)
                torch.cuda.synchronize()
                o = out.cpu().numpy()
                if ref is None:
                    ref = o
                assert np.array_equal(o, ref), (g, u, blk, cap, nt)
                res.setdefault((g, u, blk, cap, nt), []).append(
                    timer(fn, bench.SERIAL_LAUNCHES, replays=3))
        for (g, u, blk, cap, nt), ts in res.items():
            tm = float(np.median(ts))
            print(json.dumps({"L": L, "geom": f"g{g}u{u}b{blk}c{cap}nt{nt}", "us": round(tm * 1e6, 2),
                              "GBps": round(bb / tm / 1e9, 1)}), flush=True)
        del buf


if __name__ == "__main__":
    main()
