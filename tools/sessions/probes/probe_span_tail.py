#!/usr/bin/env python3
"""A/B of the ZIPF arena cut: the uniform 28 KiB ranges of
the product against the tail-shaped cut (tulips_csum_batch_arena_tuned, group
9: the last `pct` % of the arena in half-size ranges, dispatched last), over
bench.py's 24 rotated ZIPF copies (1.05 GB, HBM-resident). Serial and
4-branch per launch, ROUNDS alternations in one process; outputs poisoned
before each timed replay and every copy's digest checked after. Measurement
only; prints JSON lines."""
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
    NSEG = bench.NSEG
    lens = bench.zipf_lengths(NSEG)
    offs = np.zeros(NSEG, dtype=np.uint64)
    np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    zb = int(lens.astype(np.int64).sum())
    nz = 24
    az = torch.empty(nz * zb + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(az, nz * zb)
    doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
    dlens = torch.from_numpy(lens).to(dev)
    oz = torch.empty(nz * NSEG, dtype=torch.uint16, device=dev)
    want = bench.golden_rotations()["ZIPF"][:nz]
    forms = {"uniform_u7": csum.Tuning(kind=csum.KIND_SPAN, unroll=7, group=0, nontemporal=1)}
    for u, pct in ((7, 8), (7, 12), (7, 20), (8, 12), (6, 12)):
        forms[f"tail_u{u}_{pct}pct"] = csum.Tuning(kind=csum.KIND_SPAN, unroll=u, group=9,
                                                   nontemporal=1, sps=pct)

    def f_of(t):
        def f(i, st):
            b = i % nz
            rc = lib.tulips_csum_batch_arena_tuned(
                az.data_ptr() + b * zb, zb, doffs.data_ptr(), dlens.data_ptr(), None, None,
                None, oz.data_ptr() + b * NSEG * 2, NSEG, 0, C.byref(t), st)
            assert rc == 0, rc
        return f
    pz = bench.poisoner(oz)
    rounds = int(os.environ.get("ROUNDS", "3"))
    ser = {k: [] for k in forms}
    pip = {k: [] for k in forms}
    for r in range(rounds):
        for k, t in forms.items():
            f = f_of(t)
            for i in range(nz):
                f(i, stream.cuda_stream)
            s = timer(f, 96, poison=pz)
            ok = bench.row_digests(oz, nz, NSEG) == want
            p = timer(f, 4 * 96, branches=4, replays=3, poison=pz)
            ok = ok and bench.row_digests(oz, nz, NSEG) == want
            if not ok:
                print(json.dumps({"form": k, "parity": "MISMATCH"}), flush=True)
                sys.exit(1)
            ser[k].append(round(s * 1e6, 3))
            pip[k].append(round(p * 1e6, 3))
        print(json.dumps({"round": r, "serial_us": {k: v[-1] for k, v in ser.items()},
                          "branch4_us": {k: v[-1] for k, v in pip.items()}}), flush=True)
    print(json.dumps({"what": "ZIPF arena, 24 copies rotated, us per launch (median of rounds)",
                      "serial_us": {k: float(np.median(v)) for k, v in ser.items()},
                      "branch4_us": {k: float(np.median(v)) for k, v in pip.items()},
                      "parity": "ok"}), flush=True)


if __name__ == "__main__":
    main()
