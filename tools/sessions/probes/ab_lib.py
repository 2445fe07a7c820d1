#!/usr/bin/env python3
"""A/B of two builds of the product library on one box, in one process:
AB_A (default tools/abx_old.so, a copy of the previous build) against AB_B
(default the in-tree tulips_amd/libtulips_csum.so). Workloads as bench.py's
serial and 4-branch figures: F1500 (16 rotated batches of the M8 shard
layout), F9000 (2 rotated batches), ZIPF through the any-layout entry
(8 rotated copies), frame validation / in-place generation / compact fields
(8 bursts of 65,536 x 1514 B in 2 KiB slots), segmentation (4 x 1024
super-frames). Each workload's outputs are compared between the two builds
(bit-exact) before timing; ROUNDS alternations. Measurement only; writes
gpurun_out/ab_lib.json."""
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
    sh = stream.cuda_stream
    timer = bench.Timer(torch, stream)
    libs = {"A": load(os.path.join(ROOT, os.environ.get("AB_A", "tools/abx_old.so"))),
            "B": load(os.path.join(ROOT, os.environ.get("AB_B", "tulips_amd/libtulips_csum.so")))}
    NSEG, SEG = bench.NSEG, bench.SEG
    work = {}

    # F1500: 16 batches of 65,536 x 1500 B (1.57 GB)
    bb = NSEG * SEG
    a15 = torch.empty(16 * bb + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(a15, 16 * bb)
    o15 = torch.empty(16 * NSEG, dtype=torch.int16, device=dev)

    def f1500(lib, i, st):
        b = i % 16
        assert lib.tulips_csum_batch_fixed(a15.data_ptr() + b * bb, SEG, SEG, None, None, None,
                                           o15.data_ptr() + 2 * b * NSEG, NSEG, 0, st) == 0
    work["F1500"] = (f1500, bb, o15, 16)

    b9 = NSEG * 9000
    a9 = torch.empty(2 * b9 + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(a9, 2 * b9)
    o9 = torch.empty(2 * NSEG, dtype=torch.int16, device=dev)

    def f9000(lib, i, st):
        b = i % 2
        assert lib.tulips_csum_batch_fixed(a9.data_ptr() + b * b9, 9000, 9000, None, None, None,
                                           o9.data_ptr() + 2 * b * NSEG, NSEG, 0, st) == 0
    work["F9000"] = (f9000, b9, o9, 2)

    lens = bench.zipf_lengths(NSEG)
    offs = np.zeros(NSEG, dtype=np.uint64)
    np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    zb = int(lens.astype(np.int64).sum())
    az = torch.empty(8 * zb + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(az, 8 * zb)
    zo = torch.from_numpy(offs.view(np.int64)).to(dev)
    zl = torch.from_numpy(lens.view(np.int16).copy()).to(dev)
    oz = torch.empty(8 * NSEG, dtype=torch.int16, device=dev)

    def zipf_any(lib, i, st):
        b = i % 8
        assert lib.tulips_csum_batch(az.data_ptr() + b * zb, zo.data_ptr(), zl.data_ptr(), None,
                                     None, None, oz.data_ptr() + 2 * b * NSEG, NSEG, 0, st) == 0
    work["ZIPF_any_layout"] = (zipf_any, zb, oz, 8)

    nf, slot, flen, nb = NSEG, 2048, SEG + 14, 8
    ar = torch.empty(nb * nf * slot, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(ar, seed=0xF4A3E5)
    v = ar.view(nb * nf, slot)
    for off, val in ((12, 0x08), (13, 0), (14, 0x45), (15, 0), (16, SEG >> 8),
                     (17, SEG & 0xFF), (20, 0x40), (21, 0), (23, 6), (46, 0x50)):
        v[:, off] = val
    fo = torch.arange(nf, dtype=torch.int64, device=dev) * slot
    fl = torch.full((nf,), flen, dtype=torch.int16, device=dev)
    flags = torch.empty(nb * nf, dtype=torch.uint8, device=dev)
    fields = torch.empty(nb * nf, dtype=torch.int32, device=dev)
    burst = nf * slot
    for i in range(nb):
        assert csum.lib.tulips_csum_generate_frames(ar.data_ptr() + i * burst, fo.data_ptr(),
                                                    fl.data_ptr(), nf, None, sh) == 0

    def fval(lib, i, st):
        b = i % nb
        assert lib.tulips_csum_validate_frames(ar.data_ptr() + b * burst, fo.data_ptr(),
                                               fl.data_ptr(), nf, flags.data_ptr() + b * nf,
                                               None, st) == 0

    def fgen(lib, i, st):
        b = i % nb
        assert lib.tulips_csum_generate_frames(ar.data_ptr() + b * burst, fo.data_ptr(),
                                               fl.data_ptr(), nf, None, st) == 0

    def ffld(lib, i, st):
        b = i % nb
        assert lib.tulips_csum_generate_fields(ar.data_ptr() + b * burst, fo.data_ptr(),
                                               fl.data_ptr(), nf, fields.data_ptr() + 4 * b * nf,
                                               None, st) == 0
    work["frames_validate"] = (fval, nf * flen, flags, nb)
    work["frames_generate"] = (fgen, nf * flen, None, nb)
    work["frames_fields"] = (ffld, nf * flen, fields, nb)

    nsf, pay, mss = 1024, 44 * 1460, 1460
    sflen, sslot, sb = 54 + pay, 65536, 4
    sa = torch.empty(sb * nsf * sslot, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(sa, seed=0x7505)
    sv = sa.view(sb * nsf, sslot)
    tot = sflen - 14
    for off, val_ in ((12, 0x08), (13, 0), (14, 0x45), (15, 0), (16, tot >> 8),
                      (17, tot & 0xFF), (20, 0x40), (21, 0), (23, 6), (46, 0x50)):
        sv[:, off] = val_
    so_ = torch.arange(nsf, dtype=torch.int64, device=dev) * sslot
    sl_ = torch.full((nsf,), sflen - 65536 if sflen > 32767 else sflen, dtype=torch.int16,
                     device=dev)
    nseg, ostride = nsf * (pay // mss), 1536
    sout = torch.empty(sb * nseg * ostride, dtype=torch.uint8, device=dev)
    solen = torch.zeros(sb * nseg, dtype=torch.int16, device=dev)
    sfirst = torch.empty(sb * (nsf + 1), dtype=torch.int32, device=dev)

    def fseg(lib, i, st):
        b = i % sb
        assert lib.tulips_csum_segment_frames(sa.data_ptr() + b * nsf * sslot, so_.data_ptr(),
                                              sl_.data_ptr(), nsf, mss,
                                              sout.data_ptr() + b * nseg * ostride, ostride,
                                              nseg, solen.data_ptr() + b * nseg * 2,
                                              sfirst.data_ptr() + b * (nsf + 1) * 4, st) == 0
    work["segment"] = (fseg, nsf * sflen + nseg * (54 + mss), sout, sb)

    # parity: every workload's outputs from both builds, bit-exact
    parity = {}
    for name, (fn, _, out, rot) in work.items():
        got = {}
        for k, lib in libs.items():
            if name == "frames_generate":   # in place: check by validating after
                for i in range(rot):
                    fn(lib, i, sh)
                torch.cuda.synchronize()
                for i in range(rot):
                    fval(libs["B"], i, sh)
                torch.cuda.synchronize()
                got[k] = flags.clone()
                continue
            out.zero_()
            for i in range(rot):
                fn(lib, i, sh)
            torch.cuda.synchronize()
            got[k] = out.clone()
        same = bool(torch.equal(got["A"], got["B"]))
        if name in ("frames_validate", "frames_generate"):
            same = same and bool((got["B"] == 0x0F).all().item())
        parity[name] = "ok" if same else "MISMATCH"
    print(json.dumps({"parity": parity}), flush=True)

    res = {}
    for rnd in range(int(os.environ.get("ROUNDS", "3"))):
        for name, (fn, nbytes, _, rot) in work.items():
            for k, lib in libs.items():
                def f(i, st, fn=fn, lib=lib):
                    fn(lib, i, st)
                reps = 32 if name == "segment" else 64
                ts = timer(f, reps)
                tp = timer(f, reps, branches=4)
                r = res.setdefault(name, {}).setdefault(k, {"serial_us": [], "branch4_us": []})
                r["serial_us"].append(round(ts * 1e6, 3))
                r["branch4_us"].append(round(tp * 1e6, 3))
                print(f"round {rnd} {name:16s} {k}: serial {ts * 1e6:7.2f} us "
                      f"({nbytes / ts / 8e12:.3f})  4-branch {tp * 1e6:7.2f} us "
                      f"({nbytes / tp / 8e12:.3f})", flush=True)
    summ = {name: {k: {"serial_median_us": float(np.median(x["serial_us"])),
                       "branch4_median_us": float(np.median(x["branch4_us"]))}
                   for k, x in r.items()} for name, r in res.items()}
    for name, r in summ.items():
        print(f"{name:16s} A {r['A']['serial_median_us']:7.2f} / {r['A']['branch4_median_us']:7.2f}"
              f"   B {r['B']['serial_median_us']:7.2f} / {r['B']['branch4_median_us']:7.2f}")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "ab_lib.json"), "w") as f:
        json.dump({"A": os.environ.get("AB_A", "tools/abx_old.so"),
                   "B": os.environ.get("AB_B", "tulips_amd/libtulips_csum.so"),
                   "parity": parity, "runs": res, "summary": summ}, f, indent=1)


if __name__ == "__main__":
    main()
