#!/usr/bin/env python3
"""(r06: probe_frames_ops.py with benchlib, and a regeneration check: every
frame's fields cleared and regenerated must give the arena back.)
The three frame entry points at their product defaults, timed in one
process: validation (`tulips_csum_validate_frames`), in-place generation
(`tulips_csum_generate_frames`) and compact fields
(`tulips_csum_generate_fields`), over bench.py's 8 rotated bursts of
65,536 x 1514 B TCP frames in 2 KiB slots; serial and 4-branch figures as
fractions of 8 TB/s. Outputs are poisoned before each timed replay and
checked after (flags == 0x0F; generation leaves the arena's digest as it was,
since the frames already carry correct fields, and the compact fields equal
the stored ones; a digest of the first 4,096 fields is printed so two builds
can be compared). Run it once per library build to A/B them.
Measurement only; prints JSON lines."""
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


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    timer = bench.Timer(torch, stream)
    lib = csum.lib
    nf, slot, flen, nb = 65536, 2048, 1514, 8
    ar = torch.empty(nb * nf * slot, dtype=torch.uint8, device=dev)
    benchlib.fill_splitmix(ar, seed=0xF4A3E5)
    v = ar.view(nb * nf, slot)
    for off, val in ((12, 0x08), (13, 0), (14, 0x45), (15, 0), (16, 1500 >> 8),
                     (17, 1500 & 0xFF), (20, 0x40), (21, 0), (23, 6), (46, 0x50)):
        v[:, off] = val
    offs = torch.arange(nf, dtype=torch.int64, device=dev) * slot
    lens = torch.full((nf,), flen, dtype=torch.int16, device=dev)
    flags = torch.empty(nb * nf, dtype=torch.uint8, device=dev)
    fields = torch.empty(nb * nf, dtype=torch.int32, device=dev)
    burst = nf * slot
    for b in range(nb):
        lib.tulips_csum_generate_frames(ar.data_ptr() + b * burst, offs.data_ptr(),
                                        lens.data_ptr(), nf, None, stream.cuda_stream)
    torch.cuda.synchronize()
    arena0 = ar.clone()   # generation must leave every byte as it is

    def regenerate_check(tag):
        # every frame's two fields cleared, regenerated: the arena as it was
        hv = ar.view(nb * nf, slot)
        for c in (24, 25, 50, 51):
            hv[:, c] = 0
        for b in range(nb):
            assert lib.tulips_csum_generate_frames(ar.data_ptr() + b * burst, offs.data_ptr(),
                                                   lens.data_ptr(), nf, None,
                                                   stream.cuda_stream) == 0
        torch.cuda.synchronize()
        if not torch.equal(ar, arena0):
            print(json.dumps({"parity": "MISMATCH", "op": "regenerate", "when": tag}),
                  flush=True)
            sys.exit(1)

    diag = os.environ.get("GEN_DIAG") == "1"   # a diagnostic build: stores elsewhere
    if not diag:
        regenerate_check("before")
    alg = nf * flen

    def fval(i, st):
        b = i % nb
        rc = lib.tulips_csum_validate_frames(ar.data_ptr() + b * burst, offs.data_ptr(),
                                             lens.data_ptr(), nf, flags.data_ptr() + b * nf,
                                             None, st)
        assert rc == 0

    def fgen(i, st):
        b = i % nb
        rc = lib.tulips_csum_generate_frames(ar.data_ptr() + b * burst, offs.data_ptr(),
                                             lens.data_ptr(), nf, None, st)
        assert rc == 0

    def ffld(i, st):
        b = i % nb
        rc = lib.tulips_csum_generate_fields(ar.data_ptr() + b * burst, offs.data_ptr(),
                                             lens.data_ptr(), nf,
                                             fields.data_ptr() + b * nf * 4, None, st)
        assert rc == 0

    ops = {"validate": (fval, bench.poisoner(flags)),
           "generate": (fgen, None),
           "fields": (ffld, bench.poisoner(fields))}
    if os.environ.get("PROBE_OPS"):
        ops = {k: ops[k] for k in os.environ["PROBE_OPS"].split()}
    # NOCHECK=1: a diagnostic build that does not write flags (timing only)
    nocheck = os.environ.get("NOCHECK") == "1"
    rounds = int(os.environ.get("ROUNDS", "2"))
    res = {k: [] for k in ops}
    pipe = {k: [] for k in ops}
    fld_digest = None
    for r in range(rounds):
        for k, (fn, pz) in ops.items():
            s = timer(fn, 64, poison=pz)
            p = timer(fn, 4 * 64, branches=4, replays=3, poison=pz)
            res[k].append(round(alg / s / 1e9 / 8000, 4))
            pipe[k].append(round(alg / p / 1e9 / 8000, 4))
            if k == "validate":
                ok = nocheck or bool((flags == 0x0F).all().item())
            elif k == "generate":
                ok = diag or bool(torch.equal(ar, arena0))
            else:
                d = bench.fnv1a_u16(fields[:4096].cpu().numpy().view(np.uint16))
                ok = fld_digest is None or d == fld_digest
                fld_digest = d
                # the fields of frames that already carry correct checksums
                # are their own header words 24..25 and 50..51
                hv = ar.view(nb * nf, slot)
                want = (hv[:, 24].int() | (hv[:, 25].int() << 8) | (hv[:, 50].int() << 16)
                        | (hv[:, 51].int() << 24))
                ok = ok and bool(torch.equal(fields, want))
            if not ok:
                print(json.dumps({"parity": "MISMATCH", "op": k}), flush=True)
                sys.exit(1)
        print(json.dumps({"round": r, "serial_frac": {k: x[-1] for k, x in res.items()},
                          "pipe4_frac": {k: x[-1] for k, x in pipe.items()}}), flush=True)
    if not diag:
        regenerate_check("after")
    print(json.dumps({"what": "frame ops 65,536 x 1514 B, frac of 8 TB/s",
                      "lib": os.path.basename(os.path.realpath(csum.LIB_PATH)),
                      "serial_median": {k: float(np.median(x)) for k, x in res.items()},
                      "pipe4_median": {k: float(np.median(x)) for k, x in pipe.items()},
                      "fields_digest": fld_digest,
                      "parity": "unchecked" if nocheck else "ok"}), flush=True)


if __name__ == "__main__":
    main()
