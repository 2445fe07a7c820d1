#!/usr/bin/env python3
"""Toeplitz RSS A/B, bench.py's workload (16.8 M tuples, 12 B in + 4 B out
each, the same batch every call): serial (HIP events around a captured chain
of 32 calls, median of 3 replays) and on 4 graph branches, ROUNDS
alternations, for the tree's library and the builds named in LIB_B
(comma-separated paths); every build's hashes must equal the tree's.
Measurement only; prints JSON lines."""
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


def load(path):
    lib = C.CDLL(path)
    for name, (res, args) in csum._SIGNATURES.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args
    return lib


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    timer = bench.Timer(torch, stream)
    nt = 1 << 24
    g = torch.Generator(device="cpu").manual_seed(5)
    tup = torch.randint(0, 2**31 - 1, (4, nt), generator=g, dtype=torch.int64)
    sa, da = tup[0].to(torch.int32).to(dev), tup[1].to(torch.int32).to(dev)
    sp, dp = tup[2].to(torch.int16).to(dev), tup[3].to(torch.int16).to(dev)
    key = np.frombuffer(bytes(range(1, 41)), dtype=np.uint8).copy()
    kp = key.ctypes.data_as(C.POINTER(C.c_uint8))
    libs = {"P": csum.lib}
    for i, path in enumerate(filter(None, os.environ.get("LIB_B", "").split(","))):
        libs[f"Q{i}"] = load(os.path.join(ROOT, path))
    outs = {k: torch.empty(nt, dtype=torch.int32, device=dev) for k in libs}

    def form(k):
        lib, o = libs[k], outs[k]

        def f(i, st):
            assert lib.tulips_rss_toeplitz_batch(sa.data_ptr(), da.data_ptr(), sp.data_ptr(),
                                                 dp.data_ptr(), nt, kp, 40, 0, o.data_ptr(),
                                                 st) == 0
        return f
    forms = {k: form(k) for k in libs}
    rounds = int(os.environ.get("ROUNDS", "3"))
    ser = {k: [] for k in forms}
    pip = {k: [] for k in forms}
    for r in range(rounds):
        for k, f in forms.items():
            pz = bench.poisoner(outs[k])
            ser[k].append(round(timer(f, 32, replays=3, poison=pz) * 1e6, 3))
            pip[k].append(round(timer(f, 128, branches=4, replays=3, poison=pz) * 1e6, 3))
            if not torch.equal(outs[k], outs["P"]):
                print(json.dumps({"form": k, "parity": "MISMATCH"}), flush=True)
                sys.exit(1)
        print(json.dumps({"round": r, "serial_us": {k: v[-1] for k, v in ser.items()},
                          "branch4_us": {k: v[-1] for k, v in pip.items()}}), flush=True)
    med = {k: float(np.median(v)) for k, v in ser.items()}
    print(json.dumps({"what": "RSS 16.8 M tuples, us per call (median of rounds)",
                      "serial_us": med,
                      "serial_frac": {k: round(nt * 16 / (v * 1e-6) / 8e12, 4)
                                      for k, v in med.items()},
                      "branch4_us": {k: float(np.median(v)) for k, v in pip.items()},
                      "parity": "ok"}), flush=True)


if __name__ == "__main__":
    main()
