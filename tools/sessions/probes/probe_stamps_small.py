#!/usr/bin/env python3
"""Per-wave life of the variable-length kernels on a SMALL Zipf batch (the
first n of the §8c sequence; diagnostic build tools/libcsum_stamps.so): which
waves end last, when they started, and how many bytes their segments hold."""
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


def main():
    lib = C.CDLL(os.path.join(ROOT, "tools", "libcsum_stamps.so"))
    for name, (res, argt) in csum._SIGNATURES.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, argt
    lib.tulips_csum_stamps_arm.restype = C.c_int
    lib.tulips_csum_stamps_arm.argtypes = [C.c_void_p]
    lib.tulips_csum_stamps_count.restype = C.c_uint32
    dev = torch.device("cuda", 0)
    n = int(os.environ.get("PROBE_N", "1024"))
    lens = bench.zipf_lengths(n)
    if os.environ.get("PROBE_UNIFORM"):
        lens = np.full(n, int(os.environ["PROBE_UNIFORM"]), np.uint16)
    offs = np.zeros(n, np.uint64)
    np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    nb = int(lens.astype(np.int64).sum())
    NB = 4
    buf = torch.empty(NB * nb + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(buf, NB * nb)
    doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
    dlens = torch.from_numpy(lens.view(np.int16)).to(dev)
    out = torch.empty(n, dtype=torch.uint16, device=dev)
    stamps = torch.zeros(4 * 300000, dtype=torch.int64, device=dev)
    sh = torch.cuda.current_stream().cuda_stream
    geoms = {"packed8x4pf": (csum.KIND_PACKED, 8, 4, 2, 256),
             "span8": (csum.KIND_SPAN, 2, 8, 0, 0),
             "s2_8h2": (csum.KIND_SPAN, 4, 8, 0, 0)}
    only = os.environ.get("PROBE_GEOMS")
    if only:
        geoms = {k: v for k, v in geoms.items() if k in only.split(",")}

    def run(t, i):
        if t.kind == csum.KIND_SPAN:
            return lib.tulips_csum_batch_arena_tuned(
                buf.data_ptr() + (i % NB) * nb, nb, doffs.data_ptr(), dlens.data_ptr(), None,
                None, None, out.data_ptr(), n, 0, C.byref(t), sh)
        return lib.tulips_csum_batch_tuned(buf.data_ptr() + (i % NB) * nb, doffs.data_ptr(),
                                           dlens.data_ptr(), None, None, None, out.data_ptr(),
                                           n, 0, C.byref(t), sh)
    for gname, (kind, g, u, sps, blk) in geoms.items():
        t = csum.Tuning(kind=kind, group=g, unroll=u, nontemporal=1, sps=sps, block=blk)
        for i in range(8):
            assert run(t, i) == 0
        torch.cuda.synchronize()
        assert lib.tulips_csum_stamps_arm(stamps.data_ptr()) == 0
        assert run(t, 3) == 0
        torch.cuda.synchronize()
        m = lib.tulips_csum_stamps_count()
        st = stamps[: 4 * m].cpu().numpy().reshape(m, 4)
        base = st[:, 0].min()
        t0 = (st[:, 0] - base) / 100.0
        t1 = (st[:, 1] - base) / 100.0
        life = t1 - t0
        # bytes per wave (packed kinds: 8 consecutive segments per wave)
        wb = np.add.reduceat(lens.astype(np.int64), np.arange(0, n, 8))[:m] \
            if kind == csum.KIND_PACKED else np.zeros(m)
        rep = {"geom": gname, "n": n, "waves": int(m), "span_us": round(float(t1.max()), 2),
               "start_p50_max": [round(float(np.percentile(t0, 50)), 2), round(float(t0.max()), 2)],
               "life_p10_p50_p90_max": [round(float(np.percentile(life, q)), 2)
                                        for q in (10, 50, 90, 100)],
               "last10_end_life_start_bytes": [[round(float(t1[i]), 2), round(float(life[i]), 2),
                                                round(float(t0[i]), 2), int(wb[i])]
                                               for i in np.argsort(-t1)[:10]]}
        if kind == csum.KIND_SPAN:
            # field 2 = the stamp after the first barrier (window counted,
            # every wave's chunks staged and scanned)
            tm = (st[:, 2] - base) / 100.0
            w0 = np.arange(m) % 4 == 0
            rep["to_staged_p50_p90_max"] = [round(float(np.percentile(tm - t0, q)), 2)
                                            for q in (50, 90, 100)]
            rep["after_staged_p50_p90_max"] = [round(float(np.percentile(t1 - tm, q)), 2)
                                               for q in (50, 90, 100)]
            rep["wg_start_p10_p50_p90_max"] = [round(float(np.percentile(t0[w0], q)), 2)
                                               for q in (10, 50, 90, 100)]
        print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
