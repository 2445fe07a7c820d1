#!/usr/bin/env python3
"""Is frame validation (0.68 of 8 TB/s serial, against 0.75 for F1500) bound
by the 2 KiB receive-slot layout? On one box: the frame kernel over
65,536 x 1514 B TCP frames in 2 KiB slots, the plain checksum kernel over the
same slots (fixed length 1514, stride 2048), and the checksum kernel over the
same 65,536 x 1514 B packed end to end (stride 1514). 8 rotated bursts each,
serial chain and 4 graph branches. Measurement only; writes
gpurun_out/probe_slot_layout.json."""
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
    out = torch.empty(nb * nf, dtype=torch.int16, device=dev)
    burst = nf * slot
    packed = nf * flen
    alg = nf * flen
    lib = csum.lib
    for i in range(nb):
        assert lib.tulips_csum_generate_frames(ar.data_ptr() + i * burst, offs.data_ptr(),
                                               lens.data_ptr(), nf, None,
                                               stream.cuda_stream) == 0
    torch.cuda.synchronize()

    def frames(i, st):
        b = i % nb
        assert lib.tulips_csum_validate_frames(ar.data_ptr() + b * burst, offs.data_ptr(),
                                               lens.data_ptr(), nf, flags.data_ptr() + b * nf,
                                               None, st) == 0

    def fixed_slots(i, st):
        b = i % nb
        assert lib.tulips_csum_batch_fixed(ar.data_ptr() + b * burst, slot, flen, None, None,
                                           None, out.data_ptr() + 2 * b * nf, nf, 0, st) == 0

    def fixed_packed(i, st):
        b = i % nb
        assert lib.tulips_csum_batch_fixed(ar.data_ptr() + b * burst, flen, flen, None, None,
                                           None, out.data_ptr() + 2 * b * nf, nf, 0, st) == 0

    res = {}
    for rnd in range(int(os.environ.get("ROUNDS", "3"))):
        for name, fn in (("frames_validate_2k_slots", frames),
                         ("csum_fixed_1514_stride_2048", fixed_slots),
                         ("csum_fixed_1514_packed", fixed_packed)):
            for i in range(nb):
                fn(i, stream.cuda_stream)
            torch.cuda.synchronize()
            ts = timer(fn, 64)
            tp = timer(fn, 64, branches=4)
            r = res.setdefault(name, {"serial_us": [], "branch4_us": []})
            r["serial_us"].append(round(ts * 1e6, 3))
            r["branch4_us"].append(round(tp * 1e6, 3))
            print(f"round {rnd} {name}: serial {ts * 1e6:6.2f} us ({alg / ts / 8e12:.3f})  "
                  f"4-branch {tp * 1e6:6.2f} us ({alg / tp / 8e12:.3f})", flush=True)
    assert bool((flags == 0x0F).all().item())
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "probe_slot_layout.json"), "w") as f:
        json.dump({"alg_bytes_per_launch": alg, "results": res}, f, indent=1)


if __name__ == "__main__":
    main()
