#!/usr/bin/env python3
"""Segmentation A/B, bench.py's workload (4 rotated batches of 1024
super-frames of 64,294 B, MSS 1460, 1536 B slots): the prologue form
(tulips_csum_segment_frames), the planned form
(tulips_csum_segment_frames_planned, plan from the host) and, for the
planned kernel's ceiling, the prologue form's segment kernel alone is not
separable here - use rocprofv3 for that. Serial (HIP events around a captured
chain of 32 calls, median of 3 replays) and on 4 graph branches, ROUNDS
alternations; the planned outputs are compared with the prologue form's byte
for byte after every timed replay. Measurement only; prints JSON lines.
Optional env LIB_B: other builds of the library (comma-separated paths) whose
planned entries are timed beside the in-tree one (A/B of planned-kernel
variants)."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import benchlib  # noqa: E402
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
    nsf, pay, mss = 1024, 44 * 1460, 1460
    sflen, sslot, sb = 54 + pay, 65536, 4
    sa = torch.empty(sb * nsf * sslot, dtype=torch.uint8, device=dev)
    benchlib.fill_splitmix(sa, seed=0x7505)
    sv = sa.view(sb * nsf, sslot)
    tot = sflen - 14
    for off, val in ((12, 0x08), (13, 0), (14, 0x45), (15, 0), (16, tot >> 8),
                     (17, tot & 0xFF), (20, 0x40), (21, 0), (23, 6), (46, 0x50)):
        sv[:, off] = val
    soffs = torch.arange(nsf, dtype=torch.int64, device=dev) * sslot
    slens = torch.full((nsf,), sflen - 65536, dtype=torch.int16, device=dev)
    nseg, ost = nsf * 44, 1536
    libs = {"P": csum.lib}
    for i, path in enumerate(filter(None, os.environ.get("LIB_B", "").split(","))):
        libs[f"Q{i}"] = load(os.path.join(ROOT, path))
    keys = list(libs) + ["R"]
    outs = {k: torch.empty(sb * nseg * ost, dtype=torch.uint8, device=dev) for k in keys}
    olen = {k: torch.zeros(sb * nseg, dtype=torch.int16, device=dev) for k in keys}
    sfirst = torch.empty(sb * (nsf + 1), dtype=torch.int32, device=dev)
    hdr = sv[:nsf, :64].cpu().numpy().reshape(-1)
    plan = csum.segment_plan(hdr, np.arange(nsf, dtype=np.uint64) * np.uint64(64),
                             np.full(nsf, sflen, dtype=np.uint16), mss)
    dplan = torch.from_numpy(plan.view(np.int32).copy()).to(dev)

    def prologue(i, st):
        b = i % sb
        assert csum.lib.tulips_csum_segment_frames(
            sa.data_ptr() + b * nsf * sslot, soffs.data_ptr(), slens.data_ptr(), nsf, mss,
            outs["R"].data_ptr() + b * nseg * ost, ost, nseg,
            olen["R"].data_ptr() + b * nseg * 2, sfirst.data_ptr() + b * (nsf + 1) * 4,
            st) == 0

    def planned(k):
        lib = libs[k]

        def f(i, st):
            b = i % sb
            assert lib.tulips_csum_segment_frames_planned(
                sa.data_ptr() + b * nsf * sslot, soffs.data_ptr(), slens.data_ptr(), nsf, mss,
                dplan.data_ptr(), outs[k].data_ptr() + b * nseg * ost, ost, nseg,
                olen[k].data_ptr() + b * nseg * 2, st) == 0
        return f
    forms = {"prologue": (prologue, "R")}
    for k in libs:
        forms[f"planned_{k}"] = (planned(k), k)
    # (slot bytes past a segment's length are never written: the reference
    # copy carries the same poison byte there as every timed replay's)
    bench.poisoner(outs["R"], olen["R"])()
    for i in range(sb):
        prologue(i, stream.cuda_stream)
    torch.cuda.synchronize()
    ref_o, ref_l = outs["R"].clone(), olen["R"].clone()
    rounds = int(os.environ.get("ROUNDS", "3"))
    ser = {k: [] for k in forms}
    pip = {k: [] for k in forms}
    for r in range(rounds):
        for name, (f, k) in forms.items():
            pz = bench.poisoner(outs[k], olen[k])
            s = timer(f, 32, replays=3, poison=pz)
            ok = torch.equal(outs[k], ref_o) and torch.equal(olen[k], ref_l)
            p = timer(f, 128, branches=4, replays=3, poison=pz)
            ok = ok and torch.equal(outs[k], ref_o) and torch.equal(olen[k], ref_l)
            if not ok:
                print(json.dumps({"form": name, "parity": "MISMATCH"}), flush=True)
                sys.exit(1)
            ser[name].append(round(s * 1e6, 3))
            pip[name].append(round(p * 1e6, 3))
        print(json.dumps({"round": r, "serial_us": {k: v[-1] for k, v in ser.items()},
                          "branch4_us": {k: v[-1] for k, v in pip.items()}}), flush=True)
    moved = nsf * sflen + nseg * (54 + mss)
    med = {k: float(np.median(v)) for k, v in ser.items()}
    print(json.dumps({"what": "segmentation, 4 rotated batches of 1024 x 64,294 B super-frames, "
                              "us per call (median of rounds)",
                      "serial_us": med,
                      "serial_frac": {k: round(moved / (v * 1e-6) / 8e12, 4)
                                      for k, v in med.items()},
                      "branch4_us": {k: float(np.median(v)) for k, v in pip.items()},
                      "parity": "ok"}), flush=True)


if __name__ == "__main__":
    main()
