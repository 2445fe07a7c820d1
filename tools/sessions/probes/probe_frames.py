#!/usr/bin/env python3
"""Geometry / grid sweep of the frame kernels (validate, generate) on the
bench's frame workload: 8 bursts x 65,536 TCP frames of 1514 B in 2 KiB
slots. Writes gpurun_out/probe_frames.json; every configuration's validate
flags are checked (all frames verify after generation)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import Timer  # noqa: E402
from tulips_amd import csum  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    timer = Timer(torch, stream)
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
    alg = nf * flen
    lib = csum.lib
    if os.environ.get("PROBE_LIB"):
        # a diagnostic build (e.g. tools/libcsum_nostore.so); the frames are
        # sealed by the product library first so validation still checks
        import ctypes as C
        for i in range(nb):
            assert csum.lib.tulips_csum_generate_frames(ar.data_ptr() + i * burst,
                                                         offs.data_ptr(), lens.data_ptr(), nf,
                                                         None, stream.cuda_stream) == 0
        torch.cuda.synchronize()
        lib = C.CDLL(os.path.join(ROOT, os.environ["PROBE_LIB"]))
        for name, (res, argt) in csum._SIGNATURES.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, argt
    ft = lib.tulips_csum_frames_tuned
    results = []
    geos = [(16, 4), (16, 6), (16, 8), (8, 8), (8, 16), (32, 4), (64, 2)]
    if os.environ.get("PROBE_GEOS"):
        geos = [tuple(int(v) for v in g.split("x")) for g in os.environ["PROBE_GEOS"].split(",")]
    caps = [int(x) for x in os.environ.get("PROBE_CAPS", "0").split(",")]
    blocks = [int(x) for x in os.environ.get("PROBE_BLOCKS", "256").split(",")]
    nts = [int(x) for x in os.environ.get("PROBE_NT", "1,0").split(",")]
    configs = [(gu, c, b, nt) for gu in geos for c in caps for b in blocks for nt in nts]
    fields = torch.empty(nb * nf, dtype=torch.int32, device=dev)
    rounds = int(os.environ.get("ROUNDS", "1"))
    ops = ((1, "generate"), (0, "validate"), (2, "fields"))
    times = {}
    ref_fields = None
    for rnd in range(rounds):
        for (g, u), cap, blk, nt in configs:
            t = csum.Tuning(group=g, unroll=u, max_blocks=cap, block=blk, nontemporal=nt)
            for op, name in ops:
                def fn(i, st, op=op):
                    b = i % nb
                    rc = ft(op, ar.data_ptr() + b * burst, offs.data_ptr(), lens.data_ptr(), nf,
                            flags.data_ptr() + b * nf if op != 2 else None,
                            fields.data_ptr() + b * nf * 4 if op == 2 else None, t, st)
                    assert rc == 0, rc
                for i in range(nb):
                    fn(i, stream.cuda_stream)
                torch.cuda.synchronize()
                s = timer(fn, 128, replays=3)
                times.setdefault(((g, u), cap, blk, nt, name), []).append(s)
                if op == 0:
                    assert bool((flags == 0x0F).all().item()), (g, u, blk, nt)
                if op == 2:
                    if ref_fields is None:
                        ref_fields = fields.clone()
                    assert torch.equal(fields, ref_fields), (g, u, blk, nt)
    import numpy as np
    for (g, u), cap, blk, nt in configs:
        row = {"group": g, "unroll": u, "max_blocks": cap, "block": blk, "nt": nt}
        for op, name in ops:
            s = float(np.median(times[((g, u), cap, blk, nt, name)]))
            row[name + "_us"] = round(s * 1e6, 2)
            row[name + "_GBps"] = round(alg / s / 1e9, 1)
        row["parity"] = "ok"
        results.append(row)
        print(json.dumps(row), flush=True)
    best = {k: max(results, key=lambda r: r[k + "_GBps"]) for k in ("validate", "generate", "fields")}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "probe_frames.json"), "w") as f:
        json.dump({"workload": "8 x 65,536 x 1514 B TCP frames, 2 KiB slots",
                   "results": results, "best": best}, f, indent=1)
    print("best", json.dumps(best))


if __name__ == "__main__":
    main()
