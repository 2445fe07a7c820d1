#!/usr/bin/env python3
"""Fixed-length checksum A/B between library builds: F1500 (16 rotated
98.3 MB batches) and F9000 (4 rotated 590 MB batches) through
tulips_csum_batch_fixed with the default geometry, for the tree's library and
the builds named in LIB_B (comma-separated paths), and the kernel's own load
pattern without arithmetic ("read": tulips_csum_stream_read_slots_geom 32 x 3,
tulips_csum_stream_read_tiles 64 x 12), interleaved over ROUNDS;
serial (HIP events around a captured chain of 256 launches, median of 3
replays) and on 4 graph branches. Every build's results must equal the
tree's (NO_PARITY=1: skipped, for diagnostic builds that drop work).
Measurement only; prints JSON lines."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from tulips_amd import csum  # noqa: E402
import benchlib  # noqa: E402

N = 65536


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
    libs = {"P": csum.lib}
    for i, path in enumerate(filter(None, os.environ.get("LIB_B", "").split(","))):
        libs[f"Q{i}"] = load(os.path.join(ROOT, path))
    rounds = int(os.environ.get("ROUNDS", "3"))
    lens = [int(x) for x in os.environ.get("PROBE_LENS", "1500,9000").split(",")]
    for L, nb, chain in ((1500, 16, 256), (9000, 4, 64)):
        if L not in lens:
            continue
        bb = N * L
        buf = torch.empty(nb * bb + 256, dtype=torch.uint8, device=dev)
        benchlib.fill_splitmix(buf, nb * bb)
        outs = {k: torch.empty(nb * N, dtype=torch.uint16, device=dev) for k in libs}

        def form(k):
            lib, o = libs[k], outs[k]

            def f(i, st):
                b = i % nb
                assert lib.tulips_csum_batch_fixed(buf.data_ptr() + b * bb, L, L, None, None,
                                                   None, o.data_ptr() + b * N * 2, N, 0,
                                                   st) == 0
            return f
        forms = {k: form(k) for k in libs}
        sink = torch.zeros(4, dtype=torch.int32, device=dev)

        def read(i, st):   # the kernel's own load pattern, no arithmetic
            b = i % nb
            if L == 1500:
                benchlib.lib.tulips_csum_stream_read_slots_geom(buf.data_ptr() + b * bb, L, L, N, 32,
                                                            3, sink.data_ptr(), st)
            else:
                benchlib.lib.tulips_csum_stream_read_tiles(buf.data_ptr() + b * bb, L, N,
                                                       sink.data_ptr(), st)
        forms["read"] = read
        outs["read"] = outs["P"]
        ser = {k: [] for k in forms}
        pip = {k: [] for k in forms}
        for r in range(rounds):
            for k, f in forms.items():
                pz = bench.poisoner(outs[k]) if k != "read" else None
                ser[k].append(round(timer(f, chain, replays=3, poison=pz) * 1e6, 3))
                pip[k].append(round(timer(f, chain, branches=4, replays=3, poison=pz) * 1e6, 3))
                if k != "read" and not os.environ.get("NO_PARITY") and \
                        not torch.equal(outs[k], outs["P"]):
                    print(json.dumps({"L": L, "form": k, "parity": "MISMATCH"}), flush=True)
                    sys.exit(1)
            print(json.dumps({"L": L, "round": r, "serial_us": {k: v[-1] for k, v in ser.items()},
                              "branch4_us": {k: v[-1] for k, v in pip.items()}}), flush=True)
        med = {k: float(np.median(v)) for k, v in ser.items()}
        print(json.dumps({"L": L, "serial_us": med,
                          "serial_frac": {k: round(bb / (v * 1e-6) / 8e12, 4)
                                          for k, v in med.items()},
                          "branch4_us": {k: float(np.median(v)) for k, v in pip.items()},
                          "parity": "ok"}), flush=True)
        del buf, outs


if __name__ == "__main__":
    main()
