"""A/B of the span kernel's word protocols on the ZIPF batch (configs[3]);
tools/probes/span_early.hip lists the variants. Parity first:
every variant against the reference ZIPF digest and against the product
library on random in-order layouts (gaps, odd bases, 0..65,535-byte segments,
TCP mode, a contract-breaking batch followed by valid ones on the same
words). Then timing: 8 rotated copies, serial chain and 4 graph branches,
ROUNDS alternations. Measurement only."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
import tulips_amd  # noqa: E402
from tulips_amd import csum  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
stream = torch.cuda.current_stream()
timer = bench.Timer(torch, stream)
sl = C.CDLL(os.path.join(HERE, os.environ.get("SPAN_LIB", "libspan_early.so")))
sl.span_early_launch.restype = C.c_int
sl.span_early_launch.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p,
                                 C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p]
VARIANTS = [int(x) for x in os.environ.get("VARIANTS", "0,1,2,3").split(",")]
NSLOTS = 1 << 18
slots = torch.zeros(NSLOTS, dtype=torch.int64, device=dev)
MODE_TCP = 2


def launch(var, arena_ptr, arena_bytes, doffs, dlens, out, n, mode=0, src=None, dst=None,
           st=None):
    rc = sl.span_early_launch(arena_ptr, arena_bytes, doffs.data_ptr(), dlens.data_ptr(),
                              src.data_ptr() if src is not None else None,
                              dst.data_ptr() if dst is not None else None, out.data_ptr(), n,
                              mode, slots.data_ptr(), NSLOTS, 0x5eed,
                              var, st if st is not None else stream.cuda_stream)
    assert rc == 0, rc


def d(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


# --- parity ----------------------------------------------------------------
rng = np.random.default_rng(7)
bad = []
cases = 0
for trial in range(24):
    n = int(rng.choice([1, 2, 17, 300, 5000, 65536]))
    kind = trial % 4
    if kind in (1, 3):
        n = min(n, 5000)
    if kind == 0:
        lens = bench.zipf_lengths(n) if n == 65536 else rng.integers(0, 9001, n)
    elif kind == 1:
        lens = rng.integers(0, 65536, n)
    elif kind == 2:
        lens = rng.integers(0, 16, n)
    else:
        lens = np.where(rng.random(n) < 0.05, rng.integers(20000, 65536, n),
                        rng.integers(0, 3000, n))
    lens = lens.astype(np.uint16)
    gaps = np.where(rng.random(n) < 0.2, rng.integers(0, 5000, n), 0).astype(np.uint64)
    ends = np.cumsum(lens.astype(np.uint64) + gaps)
    offs = (ends - lens.astype(np.uint64)).astype(np.uint64)
    total = int(ends[-1]) + int(rng.integers(0, 64))
    shift = int(rng.integers(0, 16))
    arena = torch.empty(total + shift + 64, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(arena, total + shift + 64)
    base = arena[shift:]
    mode = MODE_TCP if trial % 3 == 2 else 0
    src = d(rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32))
    dst = d(rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32))
    do, dl = d(offs), d(lens)
    kw = dict(src=src, dst=dst, mode=mode) if mode else {}
    ref = tulips_amd.batch_arena(base, do, dl, arena_bytes=total, **kw)
    torch.cuda.synchronize()
    ref = ref.cpu().numpy().view(np.uint16)
    for var in VARIANTS:
        out = torch.zeros(n, dtype=torch.int16, device=dev)
        # a contract-breaking batch first (every segment doubled over the
        # previous one), then the valid batch twice on the same words
        if n > 4:
            o2 = d(np.maximum(offs.astype(np.int64) - 7000, 0).astype(np.uint64))
            launch(var, base.data_ptr(), total, o2, dl, out, n, mode, src, dst)
        for _ in range(2):
            launch(var, base.data_ptr(), total, do, dl, out, n, mode, src, dst)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint16)
            cases += 1
            if not np.array_equal(got, ref):
                bad.append({"trial": trial, "var": var, "n": n, "kind": kind, "mode": mode,
                            "mismatch": int((got != ref).sum())})
print(json.dumps({"parity_cases": cases, "mismatches": bad[:20]}), flush=True)

# --- ZIPF digest and timing -------------------------------------------------
NSEG = 65536
lens = bench.zipf_lengths(NSEG)
offs = np.zeros(NSEG, dtype=np.uint64)
np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
zb = int(lens.astype(np.int64).sum())
nz = 8
az = torch.empty(nz * zb + 256, dtype=torch.uint8, device=dev)
csum.fill_splitmix(az, nz * zb)
doffs, dlens = d(offs), d(lens)
oz = torch.empty(nz * NSEG, dtype=torch.int16, device=dev)
gold = bench.golden_digests()["ZIPF"]["fnv1a64"]
res = {}
ROUNDS = int(os.environ.get("ROUNDS", "3"))
for rnd in range(ROUNDS):
    for var in VARIANTS:
        def fz(i, st, var=var):
            b = i % nz
            launch(var, az.data_ptr() + b * zb, zb, doffs, dlens, oz[b * NSEG:], NSEG, st=st)
        oz.zero_()
        for i in range(nz):
            fz(i, stream.cuda_stream)
        ts = timer(fz, 80)
        tp = timer(fz, 80, branches=4)
        ok = bench.fnv1a_u16(oz[:NSEG].cpu().numpy().view(np.uint16)) == gold
        res.setdefault(var, []).append((round(ts * 1e6, 3), round(tp * 1e6, 3), ok))
        print(f"round {rnd} variant {var}: serial {ts * 1e6:6.2f} us  4-branch {tp * 1e6:6.2f} us "
              f"digest {'ok' if ok else 'MISMATCH'}", flush=True)
summ = {}
for var, v in res.items():
    summ[var] = {"serial_median": float(np.median([x[0] for x in v])),
                 "serial_min": min(x[0] for x in v),
                 "branch4_median": float(np.median([x[1] for x in v])),
                 "digest": all(x[2] for x in v)}
    print(f"variant {var}: serial median {summ[var]['serial_median']:.2f} "
          f"(min {summ[var]['serial_min']:.2f})  4-branch median {summ[var]['branch4_median']:.2f}")
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "span_early.json"), "w") as f:
    json.dump({"parity_cases": cases, "mismatches": bad, "ab": res, "summary": summ}, f, indent=1)

# --- stamps: per-workgroup phase times (us from the launch's first wave) ---
if os.environ.get("STAMPS", "1") == "1":
    sl.span_early_stamped.restype = C.c_int
    sl.span_early_stamped.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                      C.c_void_p, C.c_void_p]
    ranges = zb // (4096 * 7) + 2
    NL = 16
    stamps = torch.zeros(NL, ranges * 4 * 8, dtype=torch.int64, device=dev)
    names = ["start", "issued", "window", "scanned", "stored", "end", "data_in"]
    st_out = {}
    for var in (0, 1):
        def fs(i, st, var=var):
            b = i % nz
            assert sl.span_early_stamped(az.data_ptr() + b * zb, zb, doffs.data_ptr(),
                                         dlens.data_ptr(), oz[b * NSEG:].data_ptr(), NSEG,
                                         slots.data_ptr(), NSLOTS, 0x5eed, var,
                                         stamps[i % NL].data_ptr(), st) == 0
        stamps.zero_()
        t_us = timer(fs, NL) * 1e6
        a = stamps.cpu().numpy().reshape(NL, ranges, 4, 8)
        per = []
        for li in range(nz, NL):
            s_ = a[li]
            s_ = s_[s_[:, 0, 0] != 0]
            t0 = s_[:, :, 0].min()
            rel = (s_[:, :, :7] - t0) * 0.01
            wg = {nm: (rel[:, :, j].min(1) if j == 0 else rel[:, :, j].max(1))
                  for j, nm in enumerate(names)}
            per.append({nm: [round(float(np.percentile(v, q)), 2) for q in (50, 90, 100)]
                        for nm, v in wg.items()})
        med = {nm: [float(np.median([p_[nm][j] for p_ in per])) for j in range(3)] for nm in names}
        st_out[var] = {"us_per_launch": round(t_us, 3), "p50_p90_max_us": med}
        print(f"stamps variant {var}: {t_us:.2f} us/launch", json.dumps(med), flush=True)
    with open(os.path.join(ROOT, "gpurun_out", "span_early_stamps.json"), "w") as f:
        json.dump(st_out, f, indent=1)
