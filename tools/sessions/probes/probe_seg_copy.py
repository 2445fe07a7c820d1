#!/usr/bin/env python3
"""Segmentation against its copy ceiling, bench.py's workload (4 rotated
batches of 1024 super-frames of 64,294 B, MSS 1460, 1536 B slots):
  planned   tulips_csum_segment_frames_planned (the bench's figure)
  copy      tulips_csum_stream_copy_slots over the same source bytes (slot k
            copies [frame + (k % 44) * 1460, + 1514) to its slot): the
            segment kernel's loads and stores without the header work
  flat      a plain device-to-device copy (torch copy_) of the same number of
            bytes read (65.8 MB) into a contiguous buffer
Serial (HIP events around a captured chain of 32 calls, median of 3 replays)
and on 4 graph branches, ROUNDS alternations. Parity: the copy's payload bytes
[54, 1514) of every slot equal the planned segmentation's. Measurement only;
prints JSON lines."""
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
    nsf, pay, mss = 1024, 44 * 1460, 1460
    sflen, sslot, sb = 54 + pay, 65536, 4
    sa = torch.empty(sb * nsf * sslot, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(sa, seed=0x7505)
    sv = sa.view(sb * nsf, sslot)
    tot = sflen - 14
    for off, val in ((12, 0x08), (13, 0), (14, 0x45), (15, 0), (16, tot >> 8),
                     (17, tot & 0xFF), (20, 0x40), (21, 0), (23, 6), (46, 0x50)):
        sv[:, off] = val
    soffs = torch.arange(nsf, dtype=torch.int64, device=dev) * sslot
    slens = torch.full((nsf,), sflen - 65536, dtype=torch.int16, device=dev)
    nseg, ost = nsf * 44, 1536
    out_p = torch.empty(sb * nseg * ost, dtype=torch.uint8, device=dev)
    out_c = torch.empty_like(out_p)
    olen = torch.zeros(sb * nseg, dtype=torch.int16, device=dev)
    hdr = sv[:nsf, :64].cpu().numpy().reshape(-1)
    plan = csum.segment_plan(hdr, np.arange(nsf, dtype=np.uint64) * np.uint64(64),
                             np.full(nsf, sflen, dtype=np.uint16), mss)
    dplan = torch.from_numpy(plan.view(np.int32).copy()).to(dev)
    flat_n = nsf * sflen
    flat_dst = torch.empty(sb * ((flat_n + 4095) // 4096 * 4096), dtype=torch.uint8, device=dev)
    fstride = flat_dst.numel() // sb
    lib = csum.lib

    def planned(i, st):
        b = i % sb
        assert lib.tulips_csum_segment_frames_planned(
            sa.data_ptr() + b * nsf * sslot, soffs.data_ptr(), slens.data_ptr(), nsf, mss,
            dplan.data_ptr(), out_p.data_ptr() + b * nseg * ost, ost, nseg,
            olen.data_ptr() + b * nseg * 2, st) == 0

    def copy(i, st):
        b = i % sb
        assert lib.tulips_csum_stream_copy_slots(
            sa.data_ptr() + b * nsf * sslot, sslot, 44, mss, 54 + mss, nseg,
            out_c.data_ptr() + b * nseg * ost, ost, st) == 0

    def flat(i, st):
        b = i % sb
        src = sa[b * nsf * sslot: b * nsf * sslot + flat_n]
        flat_dst[b * fstride: b * fstride + flat_n].copy_(src, non_blocking=True)

    forms = {"planned": planned, "copy": copy, "flat": flat}
    rounds = int(os.environ.get("ROUNDS", "3"))
    ser = {k: [] for k in forms}
    pip = {k: [] for k in forms}
    for r in range(rounds):
        for name, f in forms.items():
            s = timer(f, 32, replays=3)
            p = timer(f, 128, branches=4, replays=3)
            ser[name].append(round(s * 1e6, 3))
            pip[name].append(round(p * 1e6, 3))
        print(json.dumps({"round": r, "serial_us": {k: v[-1] for k, v in ser.items()},
                          "branch4_us": {k: v[-1] for k, v in pip.items()}}), flush=True)
    torch.cuda.synchronize()
    a = out_p.view(sb * nseg, ost)[:, 54:54 + mss]
    c = out_c.view(sb * nseg, ost)[:, 54:54 + mss]
    ok = bool(torch.equal(a, c))
    moved = nsf * sflen + nseg * (54 + mss)
    med = {k: float(np.median(v)) for k, v in ser.items()}
    pm = {k: float(np.median(v)) for k, v in pip.items()}
    for d in (med, pm):
        d["flat"] = round(d["flat"] * moved / (2 * flat_n), 3)   # per the same bytes moved
    print(json.dumps({"what": "segmentation vs its copy ceiling, 4 rotated batches of 1024 x "
                              "64,294 B super-frames, us per call (median of rounds; flat "
                              "scaled to the segmentation's bytes moved)",
                      "bytes_moved": moved,
                      "serial_us": med,
                      "serial_frac": {k: round(moved / (v * 1e-6) / 8e12, 4)
                                      for k, v in med.items()},
                      "branch4_us": pm,
                      "parity": "ok" if ok else "MISMATCH"}), flush=True)
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
