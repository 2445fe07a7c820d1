#!/usr/bin/env python3
"""Graph branches for the overlapped ("pipeline") figures: 4 (one per
hardware queue the box gives a process) against 8, on F1500, ZIPF (arena
entry) and frame validation, as bench.py times them (rotated batches, HIP
events around a graph replay). Measurement only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from tulips_amd import csum  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    timer = bench.Timer(torch, stream)
    lib = csum.lib
    NSEG, SEG = bench.NSEG, bench.SEG
    bb = NSEG * SEG
    a15 = torch.empty(16 * bb + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(a15, 16 * bb)
    o15 = torch.empty(16 * NSEG, dtype=torch.int16, device=dev)

    def f1500(i, st):
        b = i % 16
        lib.tulips_csum_batch_fixed(a15.data_ptr() + b * bb, SEG, SEG, None, None, None,
                                    o15.data_ptr() + 2 * b * NSEG, NSEG, 0, st)
    lens = bench.zipf_lengths(NSEG)
    offs = np.zeros(NSEG, dtype=np.uint64)
    np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    zb = int(lens.astype(np.int64).sum())
    az = torch.empty(8 * zb + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(az, 8 * zb)
    zo = torch.from_numpy(offs.view(np.int64)).to(dev)
    zl = torch.from_numpy(lens.view(np.int16).copy()).to(dev)
    oz = torch.empty(8 * NSEG, dtype=torch.int16, device=dev)

    def zipf(i, st):
        b = i % 8
        lib.tulips_csum_batch_arena(az.data_ptr() + b * zb, zb, zo.data_ptr(), zl.data_ptr(),
                                    None, None, None, oz.data_ptr() + 2 * b * NSEG, NSEG, 0, st)
    nf, slot, flen, nb = NSEG, 2048, SEG + 14, 8
    ar = torch.empty(nb * nf * slot, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(ar, seed=0xF4A3E5)
    fo = torch.arange(nf, dtype=torch.int64, device=dev) * slot
    fl = torch.full((nf,), flen, dtype=torch.int16, device=dev)
    flags = torch.empty(nb * nf, dtype=torch.uint8, device=dev)

    def fval(i, st):
        b = i % nb
        lib.tulips_csum_validate_frames(ar.data_ptr() + b * nf * slot, fo.data_ptr(),
                                        fl.data_ptr(), nf, flags.data_ptr() + b * nf, None, st)
    work = {"F1500": (f1500, bb, 256), "ZIPF": (zipf, zb, 160), "frames_validate": (fval,
                                                                                   nf * flen, 128)}
    # PROBE_REPS_SCALE="1,2,4": also time each pipeline over 2x / 4x the
    # launches (the graph's fork and join are then spread over more launches)
    scales = [int(x) for x in os.environ.get("PROBE_REPS_SCALE", "1").split(",")]
    only = os.environ.get("PROBE_ONLY")
    res = {}
    for rnd in range(3):
        for name, (fn, nbytes, reps0) in work.items():
            if only and name != only:
                continue
            for sc in scales:
                reps = reps0 * sc
                for br in (4, 8):
                    t = timer(fn, reps, branches=br)
                    res.setdefault((name, br, reps), []).append(t * 1e6)
                    print(f"round {rnd} {name:16s} {reps:4d} launches {br} branches: "
                          f"{t * 1e6:6.2f} us per launch ({nbytes / t / 8e12:.3f})", flush=True)
    for (name, br, reps), v in res.items():
        print(f"{name:16s} {reps:4d} launches {br} branches: median {np.median(v):6.2f} us "
              f"({work[name][1] / np.median(v) / 8e6:.3f})")


if __name__ == "__main__":
    main()
