#!/usr/bin/env python3
"""Segments per subgroup (tuning `sps` for SUBGROUP): F1500 (16 rotated
batches of 65,536 x 1500 B) and 1500 B at stride 2048 through
tulips_csum_batch_fixed_tuned, one subgroup per segment (sps 1) against two
segments per subgroup with both first batches in flight (sps 2). Every
geometry's results are compared with the default's. Serial chain and 4
graph branches, ROUNDS alternations. Measurement only; writes
gpurun_out/probe_spw.json. Needs tools/variants/csum_two_per_subgroup_r03.patch
applied (the library rejects sps 2 otherwise); measured slower, not kept
(profiles/probe_spw_r03.txt)."""
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
    NSEG, SEG = bench.NSEG, bench.SEG
    lib = csum.lib
    geos = [(32, 4, 1), (32, 3, 2), (32, 4, 2), (16, 4, 2), (16, 4, 1)]
    if os.environ.get("GEOS"):
        geos = [tuple(int(v) for v in g.split("x")) for g in os.environ["GEOS"].split(",")]
    res, parity = {}, {}
    for stride, nb in ((1500, 16), (2048, 12)):
        bb = NSEG * stride
        ar = torch.empty(nb * bb + 256, dtype=torch.uint8, device=dev)
        csum.fill_splitmix(ar, nb * bb)
        out = torch.empty(nb * NSEG, dtype=torch.int16, device=dev)
        ref = torch.empty_like(out)
        for b in range(nb):
            assert lib.tulips_csum_batch_fixed(ar.data_ptr() + b * bb, stride, SEG, None, None,
                                               None, ref.data_ptr() + 2 * b * NSEG, NSEG, 0,
                                               stream.cuda_stream) == 0
        torch.cuda.synchronize()
        for rnd in range(int(os.environ.get("ROUNDS", "3"))):
            for g, u, s in geos:
                t = csum.Tuning(kind=1, group=g, unroll=u, nontemporal=1, sps=s)

                def fn(i, st, t=t):
                    b = i % nb
                    rc = lib.tulips_csum_batch_fixed_tuned(ar.data_ptr() + b * bb, stride, SEG,
                                                           None, None, None,
                                                           out.data_ptr() + 2 * b * NSEG, NSEG,
                                                           0, C.byref(t), st)
                    assert rc == 0, rc
                key = f"s{stride}_{g}x{u}_sps{s}"
                if rnd == 0:
                    out.zero_()
                    for i in range(nb):
                        fn(i, stream.cuda_stream)
                    torch.cuda.synchronize()
                    parity[key] = "ok" if bool(torch.equal(out, ref)) else "MISMATCH"
                ts = timer(fn, 64)
                tp = timer(fn, 64, branches=4)
                r = res.setdefault(key, {"serial_us": [], "branch4_us": []})
                r["serial_us"].append(round(ts * 1e6, 3))
                r["branch4_us"].append(round(tp * 1e6, 3))
                print(f"round {rnd} {key:22s} serial {ts * 1e6:6.2f} us "
                      f"({NSEG * SEG / ts / 8e12:.3f})  4-branch {tp * 1e6:6.2f} us "
                      f"({NSEG * SEG / tp / 8e12:.3f})  {parity[key]}", flush=True)
        del ar
    for key, r in res.items():
        print(f"{key:22s} serial median {np.median(r['serial_us']):6.2f}  "
              f"4-branch median {np.median(r['branch4_us']):6.2f}  {parity[key]}")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "probe_spw.json"), "w") as f:
        json.dump({"parity": parity, "runs": res}, f, indent=1)


if __name__ == "__main__":
    main()
