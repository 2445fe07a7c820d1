#!/usr/bin/env python3
"""Launch the variable-length kernels on the §8c ZIPF batch and on fixed
64 B / 668 B segments (and the F1500 fixed-stride kernel for scale), a few
times each, for rocprofv3 --pmc instruction/cycle counters:

  rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
      SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS \
      --output-format csv -d OUT -o run -- python tools/pmc_var.py

Summarise with tools/pmc_var.py --summarise OUT/run_counter_collection.csv
(per kernel and workload: counters per dispatch, per wave, per segment).
"""
# archived kinds (round 3): only builds of tools/variants/ accept them; the
# product library rejects them (InvalidArgument)
KIND_HYBRID, KIND_BALANCED = 2, 4

import csv
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N = 65536
REPS = 4


def run():
    import torch
    from tulips_amd import csum
    import bench
    dev = torch.device("cuda", 0)
    lib = csum.lib
    sh = torch.cuda.current_stream().cuda_stream
    geoms = {"packed": csum.Tuning(kind=csum.KIND_PACKED, group=8, unroll=4, nontemporal=1,
                                   block=256, sps=2),
             "balanced": csum.Tuning(kind=KIND_BALANCED, group=8, unroll=2, nontemporal=1,
                                     block=256, sps=2),
             "vpacked": csum.Tuning(kind=csum.KIND_PACKED, group=8, unroll=2, nontemporal=1,
                                    block=256, sps=4),
             "span4": csum.Tuning(kind=csum.KIND_SPAN, unroll=4, nontemporal=1),
             "span8": csum.Tuning(kind=csum.KIND_SPAN, unroll=8, nontemporal=1),
             "span8t": csum.Tuning(kind=csum.KIND_SPAN, unroll=8, nontemporal=0)}
    only = os.environ.get("PMC_GEOMS")
    if only:
        geoms = {k: v for k, v in geoms.items() if k in only.split(",")}
    shapes = {"zipf": bench.zipf_lengths(N)}
    out = torch.empty(N, dtype=torch.uint16, device=dev)
    order = []
    for sname, lens in shapes.items():
        offs = np.zeros(N, np.uint64)
        np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
        nb = int(lens.astype(np.int64).sum())
        arena = torch.empty(nb + 256, dtype=torch.uint8, device=dev)
        csum.fill_splitmix(arena, nb)
        doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
        dlens = torch.from_numpy(lens.view(np.int16)).to(dev)
        for gname, t in geoms.items():
            for _ in range(REPS):
                if t.kind == csum.KIND_SPAN:
                    assert lib.tulips_csum_batch_arena_tuned(
                        arena.data_ptr(), nb, doffs.data_ptr(), dlens.data_ptr(), None, None,
                        None, out.data_ptr(), N, 0, t, sh) == 0
                else:
                    assert lib.tulips_csum_batch_tuned(arena.data_ptr(), doffs.data_ptr(),
                                                       dlens.data_ptr(), None, None, None,
                                                       out.data_ptr(), N, 0, t, sh) == 0
                order.append((gname, sname, nb))
            torch.cuda.synchronize()
    a = torch.empty(N * 1500 + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(a, N * 1500)
    for _ in range(REPS):
        assert lib.tulips_csum_batch_fixed(a.data_ptr(), 1500, 1500, None, None, None,
                                           out.data_ptr(), N, 0, sh) == 0
        order.append(("fixed", "F1500", N * 1500))
    torch.cuda.synchronize()
    print(json.dumps(order))


def summarise(path):
    rows = list(csv.DictReader(open(path)))
    per = {}
    for r in rows:
        k = (r.get("Kernel_Name") or r.get("Kernel-Name") or "")
        if "fill_splitmix" in k:
            continue
        disp = r.get("Dispatch_Id") or r.get("Dispatch-Id")
        per.setdefault((disp, k), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    out = {}
    for (disp, k), c in sorted(per.items(), key=lambda x: int(x[0][0])):
        kk = ("span" + k.split("csum_span_kernel")[1][:12] if "csum_span_kernel" in k else
              "balanced" if "balanced" in k else "vpacked" if "vpacked" in k else
              "packed" if "packed" in k else
              "fixed" if "csum_kernel" in k else k[:40])
        out.setdefault(kk, []).append(c)
    for kk, lst in out.items():
        print(kk, len(lst))
        for c in lst:
            w = c.get("SQ_WAVES", 1) or 1
            print("   ", {n: round(v) for n, v in sorted(c.items())},
                  "per wave VALU %.0f SALU %.0f" % (c.get("SQ_INSTS_VALU", 0) / w,
                                                   c.get("SQ_INSTS_SALU", 0) / w))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarise":
        summarise(sys.argv[2])
    else:
        run()
