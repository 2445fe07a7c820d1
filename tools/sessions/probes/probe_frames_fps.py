#!/usr/bin/env python3
"""A/B of frame validation geometries on one box, one process: the product
default (16 lanes x 6 chunks, one frame per subgroup) against two frames per
subgroup in flight (tuning.sps = 2), and the slot-read ceiling, over bench.py's
8 rotated bursts of 65,536 x 1514 B in 2 KiB slots. Serial and 4-branch
figures, ROUNDS alternations; flags poisoned before each timed replay and
checked (== 0x0F) after. Measurement only; prints JSON lines."""
import ctypes as C
import json
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
    nf, slot, flen, nb = 65536, 2048, 1514, 8
    ar = torch.empty(nb * nf * slot, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(ar, seed=0xF4A3E5)
    v = ar.view(nb * nf, slot)
    for off, val in ((12, 0x08), (13, 0), (14, 0x45), (15, 0), (16, 1500 >> 8),
                     (17, 1500 & 0xFF), (20, 0x40), (21, 0), (23, 6), (46, 0x50)):
        v[:, off] = val
    offs = torch.arange(nf, dtype=torch.int64, device=dev) * slot
    lens = torch.full((nf,), flen, dtype=torch.int16, device=dev)
    flags = torch.empty(nb * nf, dtype=torch.uint8, device=dev)
    burst = nf * slot
    for b in range(nb):
        lib.tulips_csum_generate_frames(ar.data_ptr() + b * burst, offs.data_ptr(),
                                        lens.data_ptr(), nf, None, stream.cuda_stream)
    torch.cuda.synchronize()
    alg = nf * flen
    if os.environ.get("BLOCKS"):
        # BLOCKS="256 512 1024": the default geometry at each workgroup size
        tunings = {f"b{b}": csum.Tuning(group=16, unroll=6, nontemporal=1, sps=1, block=int(b))
                   for b in os.environ["BLOCKS"].split()}
    elif os.environ.get("GEOMS"):
        # GEOMS="16x6 32x4 64x2": one frame per subgroup at each geometry
        tunings = {}
        for gu in os.environ["GEOMS"].split():
            g, u = (int(x) for x in gu.split("x"))
            tunings[gu] = csum.Tuning(group=g, unroll=u, nontemporal=1, sps=1)
    else:
        tunings = {"fps1": csum.Tuning(group=16, unroll=6, nontemporal=1, sps=1),
                   "fps2": csum.Tuning(group=16, unroll=6, nontemporal=1, sps=2),
                   "pipelined": csum.Tuning(group=16, unroll=6, nontemporal=1, sps=3)}

    def fval(t):
        def f(i, st):
            b = i % nb
            rc = lib.tulips_csum_frames_tuned(0, ar.data_ptr() + b * burst, offs.data_ptr(),
                                              lens.data_ptr(), nf, flags.data_ptr() + b * nf,
                                              None, C.byref(t), st)
            assert rc == 0
        return f
    sink = torch.zeros(4, dtype=torch.int32, device=dev)

    def frd(i, st):
        b = i % nb
        lib.tulips_csum_stream_read_slots(ar.data_ptr() + b * burst, slot, flen, nf,
                                          sink.data_ptr(), st)
    rounds = int(os.environ.get("ROUNDS", "3"))
    res = {k: [] for k in list(tunings) + ["read_slots"]}
    pipe = {k: [] for k in res}
    pz = bench.poisoner(flags)
    for r in range(rounds):
        for k, t in tunings.items():
            s = timer(fval(t), 64, poison=pz)
            ok = bool((flags == 0x0F).all().item())
            p = timer(fval(t), 4 * 64, branches=4, replays=3, poison=pz)
            ok = ok and bool((flags == 0x0F).all().item())
            res[k].append(round(alg / s / 1e9 / 8000, 4))
            pipe[k].append(round(alg / p / 1e9 / 8000, 4))
            if not ok:
                print(json.dumps({"parity": "MISMATCH", "tuning": k}), flush=True)
                sys.exit(1)
        s = timer(frd, 64)
        p = timer(frd, 4 * 64, branches=4, replays=3)
        res["read_slots"].append(round(alg / s / 1e9 / 8000, 4))
        pipe["read_slots"].append(round(alg / p / 1e9 / 8000, 4))
        print(json.dumps({"round": r, "serial_frac": {k: x[-1] for k, x in res.items()},
                          "pipe4_frac": {k: x[-1] for k, x in pipe.items()}}), flush=True)
    print(json.dumps({"what": "frame validation 65,536 x 1514 B, frac of 8 TB/s",
                      "serial_median": {k: float(np.median(x)) for k, x in res.items()},
                      "pipe4_median": {k: float(np.median(x)) for k, x in pipe.items()},
                      "parity": "ok"}), flush=True)


if __name__ == "__main__":
    main()
