#!/usr/bin/env python3
"""Per-wave life times inside one checksum launch (diagnostic tool).

Loads tools/libcsum_stamps.so (the product sources built with
-DTULIPS_CSUM_STAMPS; every wave records its start/end in 100 MHz ticks) and
reports, for one F1500 launch per geometry: kernel span, first-wave start
spread, last-wave end spread, wave life percentiles, and how many waves were
alive over time (ramp-up / drain).
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tulips_amd import csum  # noqa: E402  (torch first: one HIP runtime)

NSEG, L, NB = 65536, 1500, 16


def main():
    lib = C.CDLL(os.path.join(ROOT, "tools", "libcsum_stamps.so"))
    for name, (res, argt) in csum._SIGNATURES.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, argt
    lib.tulips_csum_stamps_arm.restype = C.c_int
    lib.tulips_csum_stamps_arm.argtypes = [C.c_void_p]
    lib.tulips_csum_stamps_count.restype = C.c_uint32
    dev = torch.device("cuda", 0)
    bb = NSEG * L
    buf = torch.empty(NB * bb + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(buf, NB * bb)
    out = torch.empty(NSEG, dtype=torch.uint16, device=dev)
    stamps = torch.zeros(4 * 300000, dtype=torch.int64, device=dev)
    sh = torch.cuda.current_stream().cuda_stream
    for g, u in ((32, 4), (16, 8), (64, 8)):
        t = csum.Tuning(group=g, unroll=u, nontemporal=1, max_blocks=0)
        for i in range(8):   # warm: clocks up, code resident
            lib.tulips_csum_batch_fixed_tuned(buf.data_ptr() + (i % NB) * bb, L, L, None,
                                              None, None, out.data_ptr(), NSEG, 0,
                                              C.byref(t), sh)
        torch.cuda.synchronize()
        assert lib.tulips_csum_stamps_arm(stamps.data_ptr()) == 0
        lib.tulips_csum_batch_fixed_tuned(buf.data_ptr() + 9 * bb, L, L, None, None, None,
                                          out.data_ptr(), NSEG, 0, C.byref(t), sh)
        torch.cuda.synchronize()
        n = lib.tulips_csum_stamps_count()
        s = stamps[: 4 * n].cpu().numpy().reshape(n, 4)
        t0 = s[:, 0] - s[:, 0].min()
        t1 = s[:, 1] - s[:, 0].min()
        us = 1 / 100.0   # 100 MHz ticks -> us
        span = t1.max() * us
        life = (t1 - t0) * us
        grid = np.arange(0, t1.max() + 1)
        alive = np.array([((t0 <= x) & (t1 > x)).sum() for x in grid])
        rep = {
            "geometry": f"g{g}u{u}", "waves": int(n), "span_us": round(float(span), 2),
            "GBps_span": round(bb / (span * 1e-6) / 1e9, 1),
            "start_p50_us": round(float(np.percentile(t0, 50) * us), 2),
            "start_p99_us": round(float(np.percentile(t0, 99) * us), 2),
            "last_start_us": round(float(t0.max() * us), 2),
            "end_p1_us": round(float(np.percentile(t1, 1) * us), 2),
            "end_p50_us": round(float(np.percentile(t1, 50) * us), 2),
            "life_p10_p50_p90_us": [round(float(np.percentile(life, q)), 2) for q in (10, 50, 90)],
            "alive_per_10ns_tick_max": int(alive.max()),
            "alive_profile": [int(alive[int(len(alive) * f)]) for f in
                              (0.0, 0.02, 0.05, 0.1, 0.25, 0.5, 0.75, 0.9, 0.95, 0.98)],
            "xcc_waves": np.bincount(s[:, 2].astype(np.int64) & 15, minlength=8).tolist(),
        }
        print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
