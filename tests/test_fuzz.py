"""Seeded, time-budgeted fuzz of the batch entry points against the oracle.

Each case draws a batch shape at random - segment count (0 to 40,000,
log-uniform), a length mix (empty, tiny, Zipf-like, uniform to 65,535, one
fixed length), an arena with all-0x00 / all-0xFF stretches, a base alignment
and gaps between segments - and runs it through every entry that accepts it:
tulips_csum_batch (any layout: the offsets shuffled and overlapping),
tulips_csum_batch_arena (in order, with gaps), tulips_csum_verify_arena
(its count against the oracle's) and tulips_csum_batch_fixed (fixed stride),
in a random mode (RAW / INET / TCP, with or without seeds, complemented or
not). Expected values: oracle/csum_oracle.c (pinned to the reference by
tests/test_oracle.py). Bar: bit-exact.

TULIPS_FUZZ_SECONDS (default 8) bounds the run; TULIPS_FUZZ_SEED (default 1)
picks the sequence. A failure names its case seed; TULIPS_FUZZ_CASE=<case
seed> runs that case alone.
"""
import os
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import FLAG_COMPLEMENT, MODE_INET, MODE_RAW, MODE_TCP  # noqa: E402

from tulips_amd import csum  # noqa: E402

DEV = "cuda:0"
ARENA_MAX = 48 << 20   # bytes per case: the oracle finishes a case in well under a second


def _d(a):
    return torch.from_numpy(np.array(a, copy=True, order="C")).to(DEV)


def _u16(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint16)


def _lengths(rng, n):
    kind = rng.integers(0, 6)
    if kind == 0:      # Zipf-like, mostly short
        lens = np.minimum(np.minimum(rng.zipf(1.3, n), 1000) * 40, 9000)
    elif kind == 1:    # uniform to the maximum
        lens = rng.integers(0, 65536, n)
    elif kind == 2:    # tiny
        lens = rng.integers(0, 80, n)
    elif kind == 3:    # MTU-ish with jumbo outliers
        lens = rng.integers(1400, 1515, n)
        lens[rng.random(n) < 0.02] = 9000
    elif kind == 4:    # one fixed length
        lens = np.full(n, int(rng.choice([0, 1, 15, 16, 17, 1500, 1514, 9000, 65535])))
    else:              # mixed, with runs of empty segments
        lens = rng.integers(0, 3000, n)
        lens[rng.random(n) < 0.2] = 0
        if n > 64:
            s = int(rng.integers(0, n - 64))
            lens[s:s + 64] = 0
    lens = np.asarray(lens, dtype=np.int64)
    # keep the arena bounded
    total = int(lens.sum())
    if total > ARENA_MAX // 2:
        lens = (lens * (ARENA_MAX // 2) // max(total, 1)).astype(np.int64)
    return lens.astype(np.uint16)


def _arena(rng, nbytes):
    a = rng.integers(0, 256, nbytes, dtype=np.uint8)
    for _ in range(int(rng.integers(0, 4))):      # all-0x00 / all-0xFF stretches
        s = int(rng.integers(0, max(nbytes - 1, 1)))
        e = min(nbytes, s + int(rng.integers(1, 70000)))
        a[s:e] = 0xFF if rng.random() < 0.5 else 0
    return a


def _mode(rng):
    m = [MODE_RAW, MODE_INET, MODE_TCP][int(rng.integers(0, 3))]
    if rng.random() < 0.3:
        m |= FLAG_COMPLEMENT
    return m


def _case(oracle, seed):
    rng = np.random.default_rng(seed)
    n = int(np.exp(rng.uniform(0, np.log(40001)))) - 1
    lens = _lengths(rng, n)
    gaps = rng.integers(0, 40, n) * (rng.random(n) < 0.5)
    base = int(rng.integers(0, 16))
    offs = np.zeros(n, dtype=np.uint64)
    if n:
        offs[:] = base + np.concatenate(([0], np.cumsum(lens.astype(np.int64) + gaps)[:-1]))
    nbytes = int(offs[-1]) + int(lens[-1]) + 64 if n else 64
    arena = _arena(rng, nbytes)
    mode = _mode(rng)
    seeds = rng.integers(0, 65536, n, dtype=np.uint16) if rng.random() < 0.5 else None
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    if (mode & 0xff) == MODE_TCP:
        seeds = None
    exp = oracle.batch(arena, offs, lens, seeds=seeds, src=src, dst=dst, mode=mode, nthreads=8)
    da, dl = _d(arena), _d(lens.view(np.int16))
    ds = _d(seeds.view(np.int16)) if seeds is not None else None
    dsrc, ddst = _d(src.view(np.int32)), _d(dst.view(np.int32))
    what = f"case seed {seed}: n={n} mode={mode:#x} base={base}"
    # in order, with gaps
    do = _d(offs.view(np.int64))
    got = csum.batch_arena(da, do, dl, arena_bytes=nbytes, seeds=ds, src=dsrc, dst=ddst,
                           mode=mode)
    np.testing.assert_array_equal(_u16(got), exp, err_msg=f"batch_arena {what}")
    # any layout: shuffled, and some segments re-pointed to overlap others
    perm = rng.permutation(n)
    offs2, lens2 = offs[perm].copy(), lens[perm].copy()
    if n > 1:
        k = rng.integers(0, n, max(1, n // 20))
        src_k = rng.integers(0, n, len(k))
        offs2[k], lens2[k] = offs2[src_k], lens2[src_k]
    exp2 = oracle.batch(arena, offs2, lens2, seeds=None if seeds is None else seeds[perm],
                        src=src[perm], dst=dst[perm], mode=mode, nthreads=8)
    got2 = csum.batch(da, _d(offs2.view(np.int64)), _d(lens2.view(np.int16)),
                      seeds=None if seeds is None else _d(seeds[perm].view(np.int16)),
                      src=_d(src[perm].view(np.int32)), dst=_d(dst[perm].view(np.int32)),
                      mode=mode)
    np.testing.assert_array_equal(_u16(got2), exp2, err_msg=f"batch {what}")
    # verify counts (INET / TCP without the complement flag)
    vmode = mode & 0xff
    if vmode in (MODE_INET, MODE_TCP) and seeds is None:
        bad = csum.verify_arena(da, do, dl, arena_bytes=nbytes, src=dsrc, dst=ddst, mode=vmode)
        torch.cuda.synchronize()
        want = int(np.count_nonzero(oracle.batch(arena, offs, lens, src=src, dst=dst,
                                                 mode=vmode, nthreads=8) != 0xFFFF))
        assert int(bad.item()) == want, f"verify_arena {what}"
    # fixed stride over the same arena
    if n:
        L = int(lens[0])
        stride = L + int(rng.integers(0, 48))
        nf = max(0, min(n, (nbytes - base - L) // max(stride, 1) + 1)) if stride else 0
        if nf:
            offs3 = (base + np.arange(nf, dtype=np.uint64) * np.uint64(stride))
            lens3 = np.full(nf, L, dtype=np.uint16)
            exp3 = oracle.batch(arena, offs3, lens3, mode=mode, nthreads=8,
                                src=src[:nf], dst=dst[:nf])
            got3 = csum.batch_fixed(da, stride, L, nf, src=dsrc[:nf], dst=ddst[:nf],
                                    mode=mode, base_offset=base)
            np.testing.assert_array_equal(_u16(got3), exp3, err_msg=f"batch_fixed {what} "
                                                                    f"L={L} stride={stride}")


def test_fuzz_batch_entries_vs_oracle(oracle):
    if os.environ.get("TULIPS_FUZZ_CASE"):
        _case(oracle, int(os.environ["TULIPS_FUZZ_CASE"]))
        return
    budget = float(os.environ.get("TULIPS_FUZZ_SECONDS", "8"))
    seed0 = int(os.environ.get("TULIPS_FUZZ_SEED", "1"))
    t0 = time.monotonic()
    done = 0
    last = t0
    while done == 0 or time.monotonic() - t0 < budget:
        _case(oracle, seed0 * 1_000_003 + done)
        done += 1
        if time.monotonic() - last > 20:      # progress for long runs
            last = time.monotonic()
            print(f"fuzz: {done} cases, {last - t0:.0f} s", flush=True)
    print(f"fuzz: {done} cases in {time.monotonic() - t0:.1f} s", flush=True)
    assert done >= 1


# ------------------------------------------------ frames and segmentation ----
def _frame(oracle, rng, payload, doff):
    """Ethernet/IPv4/TCP frame, checksums generated by the oracle."""
    from test_segment import super_frame
    return super_frame(oracle, rng, payload, doff=doff)


def _frame_set(oracle, rng, n, max_payload):
    frames = []
    for _ in range(n):
        kind = rng.random()
        if kind < 0.6:                                   # well formed, any size
            pay = int(rng.integers(0, max_payload + 1)) if rng.random() < 0.8 else \
                int(rng.choice([0, 1, 1459, 1460, 1461, max_payload]))
            f = bytearray(_frame(oracle, rng, pay, int(rng.integers(5, 16))))
        elif kind < 0.8:                                 # corrupted header or payload bytes
            f = bytearray(_frame(oracle, rng, int(rng.integers(0, 3000)), 5))
            for _ in range(int(rng.integers(1, 4))):
                at = int(rng.integers(0, min(len(f), 64) if rng.random() < 0.7 else len(f)))
                f[at] ^= int(rng.integers(1, 256))
        elif kind < 0.9:                                 # truncated (declared > present)
            f = bytearray(_frame(oracle, rng, int(rng.integers(10, 3000)), 5))
            f = f[:int(rng.integers(14, len(f)))]
        else:                                            # runts and non-IPv4 frames
            f = bytearray(rng.integers(0, 256, int(rng.integers(0, 80)), dtype=np.uint8).tobytes())
        frames.append(bytes(f))
    from test_frames import pack
    return pack(frames, rng, gap=24, lead=int(rng.integers(0, 16)))


def _frames_case(oracle, seed):
    from test_frames import fields_of
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 1500))
    arena, offs, lens = _frame_set(oracle, rng, n, 9000 if rng.random() < 0.3 else 1460)
    what = f"frames case seed {seed}: n={n}"
    a, o, l = _d(arena), _d(offs.view(np.int64)), _d(lens.view(np.int16))
    # validation: flags and counters
    exp = oracle.validate_frames(arena, offs, lens)
    cnt = torch.zeros(4, dtype=torch.int32, device=DEV)
    fl = csum.validate_frames(a, o, l, counters=cnt)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(fl.cpu().numpy(), exp, err_msg=f"validate {what}")
    from test_frames import counters_of
    np.testing.assert_array_equal(cnt.cpu().numpy().astype(np.uint32), counters_of(exp),
                                  err_msg=f"counters {what}")
    # generation: compact fields, then in place
    exp_arena, exp_flags = oracle.generate_frames(arena, offs, lens)
    fields, ffl = csum.generate_fields(a, o, l)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ffl.cpu().numpy(), exp_flags, err_msg=f"fields flags {what}")
    np.testing.assert_array_equal(fields.cpu().numpy().view(np.uint32),
                                  fields_of(exp_arena, offs, lens, exp_flags),
                                  err_msg=f"fields {what}")
    gfl = csum.generate_frames(a, o, l)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(gfl.cpu().numpy(), exp_flags, err_msg=f"generate {what}")
    got = a.cpu().numpy()
    assert np.array_equal(got, exp_arena), (what, np.nonzero(got != exp_arena)[0][:8])


def _segment_case(oracle, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 200))
    arena, offs, lens = _frame_set(oracle, rng, n, int(rng.choice([1460, 9000, 30000])))
    mss = int(rng.choice([int(rng.integers(1, 65536)), int(rng.integers(16, 1461)), 536,
                          1460, 8960]))
    if mss < 16 and int(lens.astype(np.int64).sum()) > 200000:
        mss = 16                                       # keep the output bounded
    stride = 16 * ((94 + min(mss, 9000) + 15) // 16) + 16 * int(rng.integers(0, 3))
    what = f"segment case seed {seed}: n={n} mss={mss} stride={stride}"
    e_first, e_out, e_lens = oracle.segment_frames(arena, offs, lens, mss, stride)
    total = int(e_first[-1])
    a, o, l = _d(arena), _d(offs.view(np.int64)), _d(lens.view(np.int16))
    keep = np.arange(stride)[None, :] < e_lens.astype(np.int64)[:, None]
    want = e_out.reshape(total, stride)[keep]
    # the device-counted form
    out, ol, first = csum.segment_frames(a, o, l, mss, stride=stride)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(first.cpu().numpy().view(np.uint32), e_first,
                                  err_msg=f"first {what}")
    got_l = ol.cpu().numpy().view(np.uint16)[:total]
    np.testing.assert_array_equal(got_l, e_lens, err_msg=f"lengths {what}")
    got = out.cpu().numpy()[:total * stride].reshape(total, stride)[keep]
    assert np.array_equal(got, want), f"bytes {what}"
    # the planned form, plan from the host
    plan = csum.segment_plan(arena, offs, lens, mss)
    np.testing.assert_array_equal(plan, e_first, err_msg=f"plan {what}")
    out2, ol2 = csum.segment_frames_planned(a, o, l, mss, _d(plan.view(np.int32)), stride=stride)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ol2.cpu().numpy().view(np.uint16)[:total], e_lens,
                                  err_msg=f"planned lengths {what}")
    got2 = out2.cpu().numpy()[:total * stride].reshape(total, stride)[keep]
    assert np.array_equal(got2, want), f"planned bytes {what}"


def test_fuzz_frames_and_segmentation_vs_oracle(oracle):
    if os.environ.get("TULIPS_FUZZ_CASE"):
        s = int(os.environ["TULIPS_FUZZ_CASE"])
        _frames_case(oracle, s)
        _segment_case(oracle, s)
        return
    budget = float(os.environ.get("TULIPS_FUZZ_SECONDS", "8"))
    seed0 = int(os.environ.get("TULIPS_FUZZ_SEED", "1"))
    t0 = last = time.monotonic()
    done = 0
    while done == 0 or time.monotonic() - t0 < budget:
        s = seed0 * 1_000_033 + done
        _frames_case(oracle, s)
        _segment_case(oracle, s)
        done += 1
        if time.monotonic() - last > 20:
            last = time.monotonic()
            print(f"fuzz frames: {done} cases, {last - t0:.0f} s", flush=True)
    print(f"fuzz frames: {done} cases in {time.monotonic() - t0:.1f} s", flush=True)


# --------------------------------------------------------------- Toeplitz ----
def _rss_case(oracle, seed):
    rng = np.random.default_rng(seed)
    n = int(np.exp(rng.uniform(0, np.log(200001))))
    key = rng.integers(0, 256, int(rng.integers(4, 61)), dtype=np.uint8).tobytes()
    init = int(rng.integers(0, 2**32)) if rng.random() < 0.3 else 0
    sa = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    da = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    sp = rng.integers(0, 65536, n, dtype=np.uint32).astype(np.uint16)
    dp = rng.integers(0, 65536, n, dtype=np.uint32).astype(np.uint16)
    # arrays at a random element offset: the 4-tuples-per-thread path needs
    # 16-byte aligned addresses, the one-tuple path takes any
    sh = int(rng.integers(0, 4))

    def dev(x, dt):
        t = _d(np.concatenate([np.zeros(sh, x.dtype), x]).view(dt))
        return t[sh:]
    out = csum.rss_batch(dev(sa, np.int32), dev(da, np.int32), dev(sp, np.int16),
                         dev(dp, np.int16), key, init)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    for k in rng.integers(0, n, min(n, 64)):
        k = int(k)
        want = oracle.toeplitz(int(sa[k]), int(da[k]), int(sp[k]), int(dp[k]), key, init)
        assert int(got[k]) == want, f"rss case seed {seed}: n={n} tuple {k} key {len(key)} B"


def test_fuzz_toeplitz_vs_oracle(oracle):
    if os.environ.get("TULIPS_FUZZ_CASE"):
        _rss_case(oracle, int(os.environ["TULIPS_FUZZ_CASE"]))
        return
    budget = min(float(os.environ.get("TULIPS_FUZZ_SECONDS", "8")), 60.0) / 2
    seed0 = int(os.environ.get("TULIPS_FUZZ_SEED", "1"))
    t0 = time.monotonic()
    done = 0
    while done == 0 or time.monotonic() - t0 < budget:
        _rss_case(oracle, seed0 * 1_000_037 + done)
        done += 1
    print(f"fuzz toeplitz: {done} cases in {time.monotonic() - t0:.1f} s", flush=True)


# ---------------------------------------------------- host-memory context ----
def _host_case(oracle, ctxs, seed):
    """Host-resident batches through the staging pipeline (chunk sizes from
    the minimum up, so segments straddle chunk boundaries in every way):
    checksums, frame validation (staged and zero-copy) and in-place
    generation against the oracle."""
    rng = np.random.default_rng(seed)
    ctx = ctxs[int(rng.integers(0, len(ctxs)))]
    n = int(np.exp(rng.uniform(0, np.log(20001)))) - 1
    lens = _lengths(rng, n)
    if int(lens.astype(np.int64).sum()) > (8 << 20):
        lens = (lens.astype(np.int64) * (8 << 20) // int(lens.astype(np.int64).sum())
                ).astype(np.uint16)
    gaps = rng.integers(0, 40, n) * (rng.random(n) < 0.5)
    base = int(rng.integers(0, 16))
    offs = np.zeros(n, dtype=np.uint64)
    if n:
        offs[:] = base + np.concatenate(([0], np.cumsum(lens.astype(np.int64) + gaps)[:-1]))
    if n and rng.random() < 0.5:          # any order (the host path packs what it stages)
        perm = rng.permutation(n)
        offs, lens = offs[perm], lens[perm]
    nbytes = (int(offs.max()) + 65600) if n else 64
    arena = _arena(rng, nbytes)
    mode = _mode(rng)
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    exp = oracle.batch(arena, offs, lens, src=src, dst=dst, mode=mode, nthreads=8)
    got = ctx.batch(arena, offs, lens, src=src, dst=dst, mode=mode)
    np.testing.assert_array_equal(got, exp, err_msg=f"host batch case seed {seed}: n={n}")
    # frames
    nf = int(rng.integers(1, 600))
    farena, foffs, flens = _frame_set(oracle, rng, nf, 9000 if rng.random() < 0.3 else 1460)
    fexp = oracle.validate_frames(farena, foffs, flens)
    for low in (False, True):
        fl = ctx.validate_frames(farena, foffs, flens, low_latency=low)
        np.testing.assert_array_equal(fl, fexp, err_msg=f"host validate ({low}) case seed {seed}")
    g = np.array(farena, copy=True)
    e_arena, e_flags = oracle.generate_frames(farena, foffs, flens)
    gfl = ctx.generate_frames(g, foffs, flens)
    np.testing.assert_array_equal(gfl, e_flags, err_msg=f"host generate flags case seed {seed}")
    assert np.array_equal(g, e_arena), f"host generate bytes case seed {seed}"


def test_fuzz_host_context_vs_oracle(oracle):
    ctxs = [csum.HostContext(0, c) for c in (0, 65536 + 16, 1 << 20)]
    try:
        if os.environ.get("TULIPS_FUZZ_CASE"):
            _host_case(oracle, ctxs, int(os.environ["TULIPS_FUZZ_CASE"]))
            return
        budget = float(os.environ.get("TULIPS_FUZZ_SECONDS", "8"))
        seed0 = int(os.environ.get("TULIPS_FUZZ_SEED", "1"))
        t0 = last = time.monotonic()
        done = 0
        while done == 0 or time.monotonic() - t0 < budget:
            _host_case(oracle, ctxs, seed0 * 1_000_039 + done)
            done += 1
            if time.monotonic() - last > 20:
                last = time.monotonic()
                print(f"fuzz host: {done} cases, {last - t0:.0f} s", flush=True)
        print(f"fuzz host: {done} cases in {time.monotonic() - t0:.1f} s", flush=True)
    finally:
        for c in ctxs:
            c.close()


# ------------------------------------------------ multi-device context -------
def _mctx_case(oracle, mctxs, seed):
    """The multi-device context over 1..5 logical devices (all GPU 0 here,
    peer and staged modes): host batches, device-resident arena and
    fixed-stride batches spread over the devices, host and device-resident
    flow-affine validation, against the oracle (device_of against the
    reference-pinned host hash mod the table)."""
    rng = np.random.default_rng(seed)
    m = mctxs[int(rng.integers(0, len(mctxs)))]
    n = int(np.exp(rng.uniform(0, np.log(30001)))) - 1
    lens = _lengths(rng, n)
    gaps = rng.integers(0, 40, n) * (rng.random(n) < 0.5)
    base = int(rng.integers(0, 16))
    offs = np.zeros(n, dtype=np.uint64)
    if n:
        offs[:] = base + np.concatenate(([0], np.cumsum(lens.astype(np.int64) + gaps)[:-1]))
    nbytes = int(offs[-1]) + int(lens[-1]) + 64 if n else 64
    arena = _arena(rng, nbytes)
    mode = _mode(rng)
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    what = f"mctx case seed {seed}: ndev={m.ndev} n={n}"
    exp = oracle.batch(arena, offs, lens, src=src, dst=dst, mode=mode, nthreads=8)
    np.testing.assert_array_equal(m.batch(arena, offs, lens, src=src, dst=dst, mode=mode), exp,
                                  err_msg=f"host {what}")
    if n:
        da, do, dl = _d(arena), _d(offs.view(np.int64)), _d(lens.view(np.int16))
        dsrc, ddst = _d(src.view(np.int32)), _d(dst.view(np.int32))
        got = m.batch_arena_device(da, do, dl, arena_bytes=nbytes, src=dsrc, dst=ddst, mode=mode)
        np.testing.assert_array_equal(_u16(got), exp, err_msg=f"arena device {what}")
        L = int(lens[0])
        stride = max(L + int(rng.integers(0, 48)), 1)
        nf = max(0, min(n, (nbytes - base - L) // stride + 1))
        if nf:
            offs3 = base + np.arange(nf, dtype=np.uint64) * np.uint64(stride)
            exp3 = oracle.batch(arena, offs3, np.full(nf, L, np.uint16), src=src[:nf],
                                dst=dst[:nf], mode=mode, nthreads=8)
            got3 = m.batch_fixed_device(da, stride, L, nf, src=dsrc[:nf], dst=ddst[:nf],
                                        mode=mode, base_offset=base)
            np.testing.assert_array_equal(_u16(got3), exp3, err_msg=f"fixed device {what}")
    # flow-affine validation
    nf = int(rng.integers(1, 500))
    farena, foffs, flens = _frame_set(oracle, rng, nf, 1460)
    key = rng.integers(0, 256, 40, dtype=np.uint8).tobytes()
    table = rng.integers(0, m.ndev, int(rng.integers(1, 129)), dtype=np.uint16)
    fexp = oracle.validate_frames(farena, foffs, flens)
    fl, devof = m.validate_frames_rss(farena, foffs, flens, key, table)
    np.testing.assert_array_equal(fl, fexp, err_msg=f"rss host flags {what}")
    fa, fo, fln = _d(farena), _d(foffs.view(np.int64)), _d(flens.view(np.int16))
    dfl, ddev = m.validate_frames_rss_device(fa, fo, fln, key, table)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dfl.cpu().numpy(), fexp, err_msg=f"rss device flags {what}")
    np.testing.assert_array_equal(ddev.cpu().numpy().view(np.uint16), devof,
                                  err_msg=f"rss device_of {what}")


def test_fuzz_multi_device_context_vs_oracle(oracle):
    mctxs = []
    try:
        for nd in (1, 2, 3, 5):
            m = csum.MultiContext([0] * nd)
            if nd == 3:
                m.set_peer_mode(True)   # staged through page-locked host memory
            mctxs.append(m)
        if os.environ.get("TULIPS_FUZZ_CASE"):
            _mctx_case(oracle, mctxs, int(os.environ["TULIPS_FUZZ_CASE"]))
            return
        budget = float(os.environ.get("TULIPS_FUZZ_SECONDS", "8"))
        seed0 = int(os.environ.get("TULIPS_FUZZ_SEED", "1"))
        t0 = last = time.monotonic()
        done = 0
        while done == 0 or time.monotonic() - t0 < budget:
            _mctx_case(oracle, mctxs, seed0 * 1_000_081 + done)
            done += 1
            if time.monotonic() - last > 20:
                last = time.monotonic()
                print(f"fuzz mctx: {done} cases, {last - t0:.0f} s", flush=True)
        print(f"fuzz mctx: {done} cases in {time.monotonic() - t0:.1f} s", flush=True)
    finally:
        for m in mctxs:
            m.close()


# ------------------------------------------------------ captured graphs ------
_KEPT_GRAPHS = []


class _Job:
    """One library call with its inputs on the device, its expected result,
    and output buffers made per use (a graph keeps the ones it captured)."""

    def __init__(self, kind, make_outs, call, check):
        self.kind, self.make_outs, self.call, self.check = kind, make_outs, call, check


def _graph_jobs(oracle, rng):
    from test_frames import counters_of
    from test_segment import pack as seg_pack
    from test_segment import super_frame
    jobs = []
    # checksums: in-order arena (span kernel, per-stream split words), verify
    # counts (counter shards), any layout (packed kernel)
    n = 6000
    lens = _lengths(rng, n)
    offs = np.concatenate(([0], np.cumsum(lens.astype(np.int64) + 3)[:-1])).astype(np.uint64)
    nbytes = int(offs[-1]) + int(lens[-1]) + 64
    arena = _arena(rng, nbytes)
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    da, do, dl = _d(arena), _d(offs.view(np.int64)), _d(lens.view(np.int16))
    dsrc, ddst = _d(src.view(np.int32)), _d(dst.view(np.int32))
    e_raw = oracle.batch(arena, offs, lens, mode=MODE_RAW, nthreads=8)
    e_tcp = oracle.batch(arena, offs, lens, src=src, dst=dst, mode=MODE_TCP, nthreads=8)
    e_bad = int(np.count_nonzero(e_tcp != 0xFFFF))

    def u16_out():
        return {"out": torch.empty(n, dtype=torch.int16, device=DEV)}
    jobs.append(_Job("arena", u16_out,
                     lambda o, s: csum.batch_arena(da, do, dl, arena_bytes=nbytes, mode=MODE_RAW,
                                                   out=o["out"], stream=s),
                     lambda o: np.array_equal(_u16(o["out"]), e_raw)))
    jobs.append(_Job("verify", lambda: {"bad": torch.empty(1, dtype=torch.int32, device=DEV)},
                     lambda o, s: csum.verify_arena(da, do, dl, arena_bytes=nbytes, src=dsrc,
                                                    dst=ddst, mode=MODE_TCP, bad=o["bad"],
                                                    stream=s),
                     lambda o: int(o["bad"].item()) == e_bad))
    perm = rng.permutation(n)
    po, pl = _d(offs[perm].view(np.int64)), _d(lens[perm].view(np.int16))
    e_perm = e_raw[perm]
    jobs.append(_Job("any", u16_out,
                     lambda o, s: csum.batch(da, po, pl, mode=MODE_RAW, out=o["out"], stream=s),
                     lambda o: np.array_equal(_u16(o["out"]), e_perm)))
    # frames: validation with counters
    farena, foffs, flens = _frame_set(oracle, rng, 800, 1460)
    fexp = oracle.validate_frames(farena, foffs, flens)
    fcnt = counters_of(fexp)
    fa, fo, fl = _d(farena), _d(foffs.view(np.int64)), _d(flens.view(np.int16))
    jobs.append(_Job("validate",
                     lambda: {"flags": torch.empty(800, dtype=torch.uint8, device=DEV),
                              "cnt": torch.empty(4, dtype=torch.int32, device=DEV)},
                     lambda o, s: csum.validate_frames(fa, fo, fl, flags=o["flags"],
                                                       counters=o["cnt"], stream=s),
                     lambda o: np.array_equal(o["flags"].cpu().numpy(), fexp) and
                     np.array_equal(o["cnt"].cpu().numpy().astype(np.uint32), fcnt)))
    # segmentation, device-counted (per-stream or per-capture workspace) and planned
    frames = [super_frame(oracle, rng, int(p)) for p in rng.integers(0, 30000, 40)]
    sarena, soffs, slens = seg_pack(frames, rng)
    mss, stride = 1460, 1536
    e_first, e_out, e_lens = oracle.segment_frames(sarena, soffs, slens, mss, stride)
    total = int(e_first[-1])
    keep = np.arange(stride)[None, :] < e_lens.astype(np.int64)[:, None]
    want = e_out.reshape(total, stride)[keep]
    sa, so, sl = _d(sarena), _d(soffs.view(np.int64)), _d(slens.view(np.int16))
    plan = _d(e_first.view(np.int32))

    def seg_outs():
        return {"out": torch.empty(total * stride, dtype=torch.uint8, device=DEV),
                "ol": torch.empty(total, dtype=torch.int16, device=DEV),
                "first": torch.empty(41, dtype=torch.int32, device=DEV)}

    def seg_call(o, s):
        rc = csum.lib.tulips_csum_segment_frames(
            sa.data_ptr(), so.data_ptr(), sl.data_ptr(), 40, mss, o["out"].data_ptr(), stride,
            total, o["ol"].data_ptr(), o["first"].data_ptr(), s.cuda_stream)
        assert rc == 0, rc

    def seg_ok(o, with_first):
        ok = np.array_equal(o["ol"].cpu().numpy().view(np.uint16), e_lens) and \
            np.array_equal(o["out"].cpu().numpy().reshape(total, stride)[keep], want)
        if with_first:
            ok = ok and np.array_equal(o["first"].cpu().numpy().view(np.uint32), e_first)
        return ok
    jobs.append(_Job("segment", seg_outs, seg_call, lambda o: seg_ok(o, True)))
    jobs.append(_Job("planned", seg_outs,
                     lambda o, s: csum.segment_frames_planned(sa, so, sl, mss, plan,
                                                              stride=stride, out=o["out"],
                                                              out_lengths=o["ol"],
                                                              capacity=total, stream=s),
                     lambda o: seg_ok(o, False)))
    return jobs


def _poison_outs(outs):
    for t in outs.values():
        t.view(torch.uint8).fill_(0xA5)


def test_fuzz_captured_graphs(oracle):
    """Random sequences of captures (1-6 calls of every stateful kind on 1-4
    branch streams from torch's pool), replays on random streams with the
    outputs poisoned first, direct calls beside them and graph drops: every
    replay and call checked. The stream-state lifetimes of VERDICT r04 #1
    (split words, counter shards, segmentation workspaces) under churn."""
    # A dropped graph is kept alive, not destroyed: destroying a multi-branch
    # graph makes a later hipGraphLaunch of the HIP runtime torch bundles
    # crash, with torch kernels alone too (tools/probe_graph_churn.py;
    # DESIGN.md §8). TULIPS_FUZZ_GRAPH_DESTROY=1 destroys them (that crash).
    destroy = bool(os.environ.get("TULIPS_FUZZ_GRAPH_DESTROY"))
    kept = _KEPT_GRAPHS    # (alive to the end of the process: later tests launch graphs)
    budget = float(os.environ.get("TULIPS_FUZZ_SECONDS", "8"))
    seed = int(os.environ.get("TULIPS_FUZZ_CASE") or os.environ.get("TULIPS_FUZZ_SEED", "1"))
    rng = np.random.default_rng(seed * 1_000_099)
    jobs = _graph_jobs(oracle, rng)
    if os.environ.get("TULIPS_FUZZ_KINDS"):              # (bisection: some kinds only)
        jobs = [j for j in jobs if j.kind in os.environ["TULIPS_FUZZ_KINDS"].split(",")]
    torch.cuda.synchronize()
    import benchlib
    benchlib.crash_backtrace()                          # a native crash names its frames
    trace = os.environ.get("TULIPS_FUZZ_TRACE")
    graphs = []       # (graph, [(job, outs)])
    t0 = last = time.monotonic()
    steps = 0
    while steps == 0 or time.monotonic() - t0 < budget:
        op = rng.random()
        if trace:
            print(f"step {steps} op {op:.3f} graphs {len(graphs)}", flush=True)
        if op < 0.3 or not graphs:                       # capture
            calls = [(jobs[int(rng.integers(0, len(jobs)))], None)
                     for _ in range(int(rng.integers(1, 7)))]
            calls = [(j, j.make_outs()) for j, _ in calls]
            cap = torch.cuda.Stream()
            side = [torch.cuda.Stream() for _ in range(int(rng.integers(1, 5)))]
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cap):
                main = torch.cuda.current_stream()
                for sd in side:
                    sd.wait_stream(main)
                for i, (j, o) in enumerate(calls):
                    j.call(o, side[i % len(side)])
                for sd in side:
                    main.wait_stream(sd)
            graphs.append((g, calls))
            if trace:
                print("  captured " + " ".join(f"{j.kind}@{i % len(side)}"
                                               for i, (j, _) in enumerate(calls)), flush=True)
            if len(graphs) > 8:
                gone = graphs.pop(int(rng.integers(0, len(graphs))))
                if not destroy:
                    kept.append(gone[0])
        elif op < 0.75:                                  # replay and check
            gi = int(rng.integers(0, len(graphs)))
            g, calls = graphs[gi]
            if trace:
                print(f"  replay graph {gi}: " + " ".join(j.kind for j, _ in calls), flush=True)
            for _, o in calls:
                _poison_outs(o)
            torch.cuda.synchronize()
            with torch.cuda.stream(torch.cuda.Stream()):
                g.replay()
            torch.cuda.synchronize()
            for j, o in calls:
                assert j.check(o), f"replayed {j.kind} (seed {seed}, step {steps})"
        elif op < 0.95:                                  # direct call beside the graphs
            j = jobs[int(rng.integers(0, len(jobs)))]
            o = j.make_outs()
            _poison_outs(o)
            s = torch.cuda.Stream()
            torch.cuda.synchronize()
            j.call(o, s)
            torch.cuda.synchronize()
            assert j.check(o), f"direct {j.kind} (seed {seed}, step {steps})"
        else:                                            # drop a graph
            gone = graphs.pop(int(rng.integers(0, len(graphs))))
            if not destroy:
                kept.append(gone[0])
        steps += 1
        if time.monotonic() - last > 20:
            last = time.monotonic()
            print(f"fuzz graphs: {steps} steps, {last - t0:.0f} s", flush=True)
    torch.cuda.synchronize()
    if not destroy:
        kept.extend(g for g, _ in graphs)
    print(f"fuzz graphs: {steps} steps in {time.monotonic() - t0:.1f} s", flush=True)
