"""Where a ZIPF arena launch spends its time: per-wave realtime stamps of the
product span kernel's own body (tools/probes/span_stamps.hip, marks in
tulips_amd/csrc/span_kernel.h), plus an A/B of the product library against a
second build (tools/probes/lib_span_before.so, when present).

Per launch (16 launches of a serial graph chain over 8 rotated copies of the
ZIPF batch, configs[3]) it reports, relative to the first wave's start:
workgroup start spread, window counted, data scanned, in-range stores issued
and end, as percentiles over workgroups, and the kernel's event-timed
duration for comparison. Parity: the stamped kernel's results against the
reference ZIPF digest. Measurement only."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from tulips_amd import csum  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
TICK_US = 0.01  # s_memrealtime runs at 100 MHz

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
stream = torch.cuda.current_stream()
timer = bench.Timer(torch, stream)
NSEG = 65536
lens = bench.zipf_lengths(NSEG)
offs = np.zeros(NSEG, dtype=np.uint64)
np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
zb = int(lens.astype(np.int64).sum())
nz = 8
az = torch.empty(nz * zb + 256, dtype=torch.uint8, device=dev)
csum.fill_splitmix(az, nz * zb)
doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
dlens = torch.from_numpy(lens).to(dev)
oz = torch.empty(nz * NSEG, dtype=torch.uint16, device=dev)
gold = bench.golden_digests()["ZIPF"]["fnv1a64"]
out = {"workload": "ZIPF batch (65,536 Zipf segments, 43.8 MB), 8 rotated copies"}

# 1. A/B: product library (this tree), the saved build, and the probe's own
#    instantiations of the same body with 8 (product), 16, 32, 64 ranges per
#    XCD run (no stamps)
sl = C.CDLL(os.path.join(HERE, "libspan_stamps.so"))
sl.span_probe_launch.restype = C.c_int
sl.span_probe_launch.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p,
                                 C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
sl.read_shape_launch.restype = C.c_int
sl.read_shape_launch.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32,
                                 C.c_uint32, C.c_void_p, C.c_void_p]
sl.span_diag_launch.restype = C.c_int
sl.span_diag_launch.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                C.c_void_p, C.c_void_p]
sink = torch.zeros(16, dtype=torch.int32, device=dev)
sl.span_stamps_ranges.restype = C.c_uint64
sl.span_stamps_ranges.argtypes = [C.c_void_p, C.c_uint64]
ranges = max(int(sl.span_stamps_ranges(az.data_ptr() + b * zb, zb)) for b in range(nz))
slots = torch.zeros(2 * ranges, dtype=torch.int64, device=dev)  # room for U >= 3
NL = 16
stamps = torch.zeros(NL, ranges * 4 * 8, dtype=torch.int64, device=dev)


def probe_fn(u, stamped, mh, nwin=1024, xc=8):
    def f(i, st):
        b = i % nz
        sp = stamps[i % NL].data_ptr() if stamped else None
        assert sl.span_probe_launch(az.data_ptr() + b * zb, zb, doffs.data_ptr(),
                                    dlens.data_ptr(), oz.data_ptr() + b * NSEG * 2, NSEG,
                                    slots.data_ptr(), 2 * ranges, 0x5eed, sp, u, xc, nwin, mh, st) == 0
    return f


def diag_fn(stop, mh):
    def f(i, st):
        b = i % nz
        assert sl.span_diag_launch(az.data_ptr() + b * zb, zb, doffs.data_ptr(),
                                   dlens.data_ptr(), oz.data_ptr() + b * NSEG * 2, NSEG,
                                   slots.data_ptr(), ranges, stop, mh, sink.data_ptr(), st) == 0
    return f


def read_fn(nwin):
    def f(i, st):
        b = i % nz
        assert sl.read_shape_launch(az.data_ptr() + b * zb, zb, doffs.data_ptr(),
                                    dlens.data_ptr(), NSEG, nwin, sink.data_ptr(), st) == 0
    return f


libs = [("product", csum.lib)]
before = os.path.join(HERE, "lib_span_before.so")
if os.path.exists(before):
    libs.append(("before", C.CDLL(before)))
cands = []
for name, lib in libs:
    lib.tulips_csum_batch_arena.restype = C.c_int
    lib.tulips_csum_batch_arena.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_uint32, C.c_uint32, C.c_void_p]

    def fz(i, st, lib=lib):
        b = i % nz
        assert lib.tulips_csum_batch_arena(az.data_ptr() + b * zb, zb, doffs.data_ptr(),
                                           dlens.data_ptr(), None, None, None,
                                           oz.data_ptr() + b * NSEG * 2, NSEG, 0, st) == 0
    cands.append((name, fz))
for u, mh, nwin, xc in ((6, 6, 1024, 8), (6, 3, 1024, 8), (6, 2, 1024, 8), (7, 2, 1024, 8),
                        (7, 3, 1024, 8), (7, 4, 1024, 8), (8, 3, 1024, 8), (8, 4, 1024, 8),
                        (7, 3, 768, 8)):
    cands.append((f"u{u}_mh{mh}_w{nwin}_xc{xc}", probe_fn(u, False, mh, nwin, xc)))
cands.append(("read_win1024", read_fn(1024)))
ab = {}
ROUNDS = int(os.environ.get("ROUNDS", "3"))
for rnd in range(ROUNDS):
    for name, fz in cands:
        oz.zero_()
        for i in range(nz):
            fz(i, stream.cuda_stream)
        ts = timer(fz, 80)
        tp = timer(fz, 80, branches=4)
        ok = name.startswith(("read_", "diag_")) or \
            bench.fnv1a_u16(oz[:NSEG].cpu().numpy().view(np.uint16)) == gold
        ab.setdefault(name, []).append((round(ts * 1e6, 3), round(tp * 1e6, 3), ok))
        print(f"round {rnd} {name:12s}: serial {ts * 1e6:6.2f} us  4-branch {tp * 1e6:6.2f} us "
              f"parity {'ok' if ok else 'MISMATCH'}", flush=True)
out["ab"] = ab
out["ab_median"] = {k: {"serial": float(np.median([x[0] for x in v])),
                        "branch4": float(np.median([x[1] for x in v])),
                        "parity": all(x[2] for x in v)} for k, v in ab.items()}

# 2. stamps (the product body, and with MH = 3)
STAMP_MH = int(os.environ.get("STAMP_MH", "3"))
fs = probe_fn(6, True, STAMP_MH)
oz.zero_()
stamps.zero_()

for i in range(nz):
    fs(i, stream.cuda_stream)
torch.cuda.synchronize()
ok = bench.fnv1a_u16(oz[:NSEG].cpu().numpy().view(np.uint16)) == gold
t_stamped = timer(fs, NL)
st = stamps.cpu().numpy().reshape(NL, -1, 4, 8)
launches = []
for li in range(NL):
    s = st[li]
    b = li % nz
    nr = int(sl.span_stamps_ranges(az.data_ptr() + b * zb, zb))
    s = s[:nr]
    t0 = s[:, :, 0].min()
    rel = (s[:, :, :6] - t0) * TICK_US                         # [wg, wave, mark]
    wg = {"start": rel[:, :, 0].min(1), "issued": rel[:, :, 1].max(1),
          "window": rel[:, :, 2].max(1), "scanned": rel[:, :, 3].max(1),
          "stored": rel[:, :, 4].max(1), "end": rel[:, :, 5].max(1)}
    pct = {k: [round(float(np.percentile(v, q)), 2) for q in (0, 50, 90, 99, 100)]
           for k, v in wg.items()}
    xcc = s[:, 0, 6] & 0xf
    per_xcc = {int(x): [round(float(np.percentile(wg["scanned"][xcc == x], q)), 2) for q in (50, 100)]
               for x in sorted(set(xcc.tolist()))}
    launches.append({"ranges": nr, "pct_0_50_90_99_100_us": pct,
                     "scanned_p50_max_by_xcc": per_xcc,
                     "wg_life_us_median": round(float(np.median(wg["end"] - wg["start"])), 2),
                     "post_scan_us_median": round(float(np.median(wg["end"] - wg["scanned"])), 2),
                     "post_scan_us_p99": round(float(np.percentile(wg["end"] - wg["scanned"], 99)), 2),
                     "rare_path_wgs": int((s[:, :, 7] != 0).any(1).sum()),
                     "end_minus_last_scan_us": round(float(wg["end"].max() - wg["scanned"].max()), 2)})
out["stamped"] = {"us_per_launch_serial_graph": round(t_stamped * 1e6, 3), "parity": ok,
                  "launches": launches[nz:]}
for L in launches[nz:nz + 3]:
    print(json.dumps(L), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", f"span_stamps_mh{STAMP_MH}.json"), "w") as f:
    json.dump(out, f, indent=1)
for k, v in out["ab_median"].items():
    print(f"median {k:22s} serial {v['serial']:6.2f}  4-branch {v['branch4']:6.2f}")
print(json.dumps({"ab": ab, "stamped_us": out["stamped"]["us_per_launch_serial_graph"],
                  "parity": ok}))
