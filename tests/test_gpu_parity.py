"""GPU parity: the gfx950 kernels (through the C ABI) against the reference.

Expected values come from the committed fixtures (computed by the reference's
own compiled src/stack, tests/golden/make_golden.py) and, for fresh random
cases, from the CPU restatement oracle/csum_oracle.c (itself pinned to the
reference by tests/test_oracle.py). Bar: bit-exact.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import (MODE_INET, MODE_RAW, MODE_TCP, FLAG_COMPLEMENT,  # noqa: E402
                    fixed_offsets, ip4, packed_offsets)

import tulips_amd  # noqa: E402
from tulips_amd import csum  # noqa: E402
import benchlib  # noqa: E402

DEV = "cuda:0"

SUB, PCK = csum.KIND_SUBGROUP, csum.KIND_PACKED
# The shipped geometries (include/tulips_csum.h, explicit kernel geometry). The library's defaults
# pick SUBGROUP 16x4 / 32x4 / 64x8 / 64x12 by fixed length and PACKED 8x4
# (double-buffered) for variable lengths at any offsets.
# (kind, group, unroll, nontemporal bits, sps)
SUBGROUP = [(16, 2), (16, 4), (16, 8), (32, 2), (32, 3), (32, 4), (32, 8), (64, 4), (64, 8),
            (64, 9), (64, 10), (64, 12)]
GEOMETRIES = [(SUB, g, u, nt, 0) for (g, u) in SUBGROUP for nt in (0, 1, 3)]
# packed kernel: `group` segments per wave, `unroll` 64-chunk windows per batch
PACKED = [(8, 2), (8, 4), (16, 2), (16, 4)]
GEOMETRIES += [(PCK, s, u, nt, 2) for (s, u) in PACKED for nt in (0, 1)]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def d(a, dtype=None):
    t = torch.from_numpy(np.array(a, copy=True, order="C"))  # (writable: from_numpy warns on read-only arrays)
    if dtype is not None:
        t = t.view(dtype)
    return t.to(DEV)


def h(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def u16(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint16)


def fnv(oracle, t):
    torch.cuda.synchronize()
    return f"{oracle.fnv1a_u16(u16(t)):016x}"


# -- fixtures ---------------------------------------------------------------
def test_adversarial_all_modes_default_geometry(golden):
    adv = golden.adversarial()
    offs, lens = d(adv["offsets"]), d(adv["lengths"])
    seeds, src, dst = d(adv["seeds"]), d(adv["src"]), d(adv["dst"])
    for name, (kind, mode, use_seeds) in golden.ADV_CASES.items():
        arena = d(golden.adv_arena(adv, kind))
        out = tulips_amd.batch(arena, offs, lens, seeds=seeds if use_seeds else None,
                               src=src, dst=dst, mode=mode)
        np.testing.assert_array_equal(u16(out), adv["expect_" + name], err_msg=name)


@pytest.mark.parametrize("geom", GEOMETRIES)
def test_adversarial_every_geometry(golden, geom):
    kind, g, u, nt, sps = geom
    adv = golden.adversarial()
    arena = d(adv["arena"])
    offs, lens = d(adv["offsets"]), d(adv["lengths"])
    src, dst, seeds = d(adv["src"]), d(adv["dst"]), d(adv["seeds"])
    for max_blocks in (0, 7):
        t = csum.Tuning(kind=kind, group=g, unroll=u, nontemporal=nt, max_blocks=max_blocks,
                        sps=sps)
        out = tulips_amd.batch(arena, offs, lens, src=src, dst=dst, mode=MODE_TCP, tuning=t)
        np.testing.assert_array_equal(u16(out), adv["expect_tcp"])
        out = tulips_amd.batch(arena, offs, lens, seeds=seeds, mode=MODE_RAW, tuning=t)
        np.testing.assert_array_equal(u16(out), adv["expect_raw_seed"])


def test_kat_through_device_batch(golden, oracle):
    """Every single-call known answer, as one device batch per function."""
    cases = golden.kat()
    for fn, mode in (("checksum", MODE_RAW), ("ipv4", MODE_INET), ("icmpv4", MODE_INET),
                     ("tcp", MODE_TCP)):
        rows = [c for c in cases if c["fn"] == fn]
        datas = [golden.kat_data(c, oracle) for c in rows]
        if fn == "ipv4":
            datas = [x[:20] for x in datas]
        if fn == "icmpv4":
            datas = [x[:8] for x in datas]
        lens = np.array([len(x) for x in datas], dtype=np.uint16)
        offs = packed_offsets(lens) + np.uint64(1)   # odd base: flips every parity
        arena = np.frombuffer(b"\x5a" + b"".join(datas) + b"\x5a" * 16, dtype=np.uint8)
        seeds = np.array([c.get("seed", 0) for c in rows], dtype=np.uint16)
        src = np.array([c.get("src", 0) for c in rows], dtype=np.uint32)
        dst = np.array([c.get("dst", 0) for c in rows], dtype=np.uint32)
        out = tulips_amd.batch(d(arena), d(offs), d(lens), seeds=d(seeds), src=d(src),
                               dst=d(dst), mode=mode)
        np.testing.assert_array_equal(u16(out), np.array([c["expect"] for c in rows],
                                                         dtype=np.uint16), err_msg=fn)


# -- SURVEY.md §8c batches: digests at full size -------------------------------
def _fill(nbytes, byte_off=0):
    buf = torch.empty(nbytes + 64, dtype=torch.uint8, device=DEV)
    benchlib.fill_splitmix(buf, nbytes, byte_off=byte_off)
    return buf


def test_device_fill_matches_spec(oracle):
    buf = _fill(1 << 20)
    np.testing.assert_array_equal(h(buf)[: 1 << 20], oracle.splitmix_bytes(1 << 20))
    for off in (1, 3, 8, 12345):
        buf = torch.zeros(4096, dtype=torch.uint8, device=DEV)
        benchlib.fill_splitmix(buf[5:], 1000, byte_off=off)
        got = h(buf)
        np.testing.assert_array_equal(got[5:1005], oracle.splitmix_bytes(1000, byte_off=off))
        assert not got[:5].any() and not got[1005:].any()


@pytest.mark.parametrize("name", ["F1500", "F9000", "F1500s2048", "F9000s9216", "F64",
                                  "F1500-tcp", "F9000-tcp"])
def test_fixed_digest(golden, oracle, name):
    b = golden.digests()["batches"][name]
    n, L, stride = b["n"], b["length"], b["stride"]
    arena = _fill(n * stride)
    if b["mode"] == "tcp":
        src = d(np.full(n, ip4(10, 1, 0, 1), np.uint32))
        dst = d(np.full(n, ip4(10, 1, 0, 2), np.uint32))
        out = tulips_amd.batch_fixed(arena, stride, L, n, src=src, dst=dst, mode=MODE_TCP)
    else:
        out = tulips_amd.batch_fixed(arena, stride, L, n)
    assert fnv(oracle, out) == b["fnv1a64"]
    # the variable-length entry point on the same segments agrees
    offs = d(fixed_offsets(n, stride))
    lens = d(np.full(n, L, np.uint16))
    if b["mode"] != "tcp":
        out2 = tulips_amd.batch(arena, offs, lens)
        assert fnv(oracle, out2) == b["fnv1a64"]


@pytest.mark.parametrize("name", ["ZIPF", "ZIPF-tcp"])
def test_zipf_digest(golden, oracle, name):
    b = golden.digests()["batches"][name]
    n = b["n"]
    lens = oracle.zipf_lengths(n)
    offs = packed_offsets(lens)
    arena = _fill(int(lens.astype(np.int64).sum()))
    kw = {}
    if b["mode"] == "tcp":
        kw = dict(src=d(np.full(n, ip4(10, 1, 0, 1), np.uint32)),
                  dst=d(np.full(n, ip4(10, 1, 0, 2), np.uint32)), mode=MODE_TCP)
    geoms = [None] + [(SUB, g, 1) for g in (16, 32, 64)]
    geoms += [(PCK, s_, 2, u_) for (s_, u_) in PACKED]
    for geo in geoms:
        t = None if geo is None else csum.Tuning(kind=geo[0], group=geo[1],
                                                 unroll=geo[3] if len(geo) > 3 else 4,
                                                 sps=geo[2])
        out = tulips_amd.batch(arena, d(offs), d(lens), tuning=t, **kw)
        assert fnv(oracle, out) == b["fnv1a64"], geo


def test_m8_all_shards(golden, oracle):
    """M8x1500 (8,388,608 segments, 12.6 GB): every shard's digest, each shard
    materialised in HBM at its global byte offset, as one rank of the 8-GPU
    run would hold it."""
    b = golden.digests()["batches"]["M8x1500"]
    shard_n, L = b["n"] // 8, 1500
    arena = torch.empty(shard_n * L + 64, dtype=torch.uint8, device=DEV)
    outs = []
    for r in range(8):
        benchlib.fill_splitmix(arena, shard_n * L, byte_off=r * shard_n * L)
        out = tulips_amd.batch_fixed(arena, L, L, shard_n)
        assert fnv(oracle, out) == b["shards"][r]["fnv1a64"], r
        outs.append(u16(out))
    assert f"{oracle.fnv1a_u16(np.concatenate(outs)):016x}" == b["fnv1a64"]


# -- fresh random cases vs the restatement ----------------------------------
def test_random_vs_oracle_all_alignments(oracle):
    rng = np.random.default_rng(355)
    arena = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
    n = 30000
    lens = rng.integers(0, 12000, n).astype(np.uint16)
    lens[:500] = rng.integers(0, 64, 500)
    lens[500:600] = rng.integers(60000, 65536, 100)
    offs = np.array([rng.integers(0, len(arena) - int(L)) for L in lens], dtype=np.uint64)
    seeds = rng.integers(0, 65536, n, dtype=np.uint16)
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    da, do, dl = d(arena), d(offs), d(lens)
    ds_, dsrc, ddst = d(seeds), d(src), d(dst)
    for mode in (MODE_RAW, MODE_INET, MODE_TCP, MODE_RAW | FLAG_COMPLEMENT,
                 MODE_TCP | FLAG_COMPLEMENT):
        exp = oracle.batch(arena, offs, lens, seeds=seeds, src=src, dst=dst, mode=mode,
                           nthreads=8)
        got = tulips_amd.batch(da, do, dl, seeds=ds_, src=dsrc, dst=ddst, mode=mode)
        np.testing.assert_array_equal(u16(got), exp, err_msg=hex(mode))


@pytest.mark.parametrize("geo", PACKED)
def test_packed_random_vs_oracle(oracle, geo):
    """PACKED kernel: segments laid end to end in one chunk space per wave,
    double-buffered windows. Lengths mix empty, 1..63 B, Zipf-like and up to
    65,535 B; any alignment; runs of empty segments at wave starts/ends; n not
    a multiple of the wave's segment count; grid-stride (max_blocks) on and
    off, several groups per wave when capped."""
    s_, u_ = geo
    rng = np.random.default_rng(1000 + s_ * 10 + u_)
    arena = rng.integers(0, 256, 2 << 20, dtype=np.uint8)
    arena[:4096] = 0                       # all-zero segments (result 0 vs 0xffff)
    arena[4096:8192] = 0xFF
    n = 20000 + s_ - 3
    lens = rng.integers(0, 3000, n).astype(np.uint16)
    lens[rng.random(n) < 0.15] = 0
    lens[:3 * s_] = 0                      # whole waves of empty segments
    lens[rng.integers(0, n, 60)] = rng.integers(60000, 65536, 60)
    lens[rng.integers(0, n, 300)] = rng.integers(1, 64, 300)
    offs = np.array([rng.integers(0, len(arena) - int(L)) for L in lens], dtype=np.uint64)
    zero_idx = rng.integers(0, n, 200)
    lens[zero_idx] = np.minimum(lens[zero_idx], 2000)
    offs[zero_idx] = rng.integers(0, 4096 - 2000, 200)
    ff_idx = rng.integers(0, n, 200)
    lens[ff_idx] = np.minimum(lens[ff_idx], 2000)
    offs[ff_idx] = 4096 + rng.integers(0, 4096 - 2000, 200)
    seeds = rng.integers(0, 65536, n, dtype=np.uint16)
    seeds[zero_idx[:100]] = 0
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    da, do, dl = d(arena), d(offs), d(lens)
    ds_, dsrc, ddst = d(seeds), d(src), d(dst)
    for mode in (MODE_RAW, MODE_TCP | FLAG_COMPLEMENT):
        exp = oracle.batch(arena, offs, lens, seeds=seeds, src=src, dst=dst, mode=mode,
                           nthreads=8)
        for max_blocks, sps in ((0, 2), (5, 2), (37, 2)):
            t = csum.Tuning(kind=PCK, group=s_, unroll=u_, nontemporal=1,
                            max_blocks=max_blocks, sps=sps)
            got = tulips_amd.batch(da, do, dl, seeds=ds_, src=dsrc, dst=ddst, mode=mode,
                                   tuning=t)
            np.testing.assert_array_equal(u16(got), exp, err_msg=f"{hex(mode)} {max_blocks} {sps}")


@pytest.mark.parametrize("L", [0, 1, 2, 3, 15, 16, 17, 63, 64, 65, 1499, 1500, 1501, 8999,
                               9000, 9001, 65535])
@pytest.mark.parametrize("base_off", [0, 1, 2, 7, 15])
def test_fixed_lengths_and_base_alignment(oracle, L, base_off):
    n = 257
    stride = max(L, 1) + 3  # odd-ish stride: every segment a different alignment
    rng = np.random.default_rng(L * 31 + base_off)
    arena = rng.integers(0, 256, n * stride + 64, dtype=np.uint8)
    exp = oracle.batch(arena[base_off:], stride=stride, fixed_len=L, n=n, mode=MODE_RAW)
    da = d(arena)
    for g, u in ((16, 2), (16, 8), (32, 2), (32, 3), (32, 8), (64, 4), (64, 9), (64, 10), (64, 12)):
        t = csum.Tuning(group=g, unroll=u, nontemporal=0, max_blocks=0)
        got = tulips_amd.batch_fixed(da, stride, L, n, tuning=t, base_offset=base_off)
        np.testing.assert_array_equal(u16(got), exp, err_msg=f"g{g} u{u}")


# -- verify and generate (the stack's two call patterns) ------------------------
def test_generate_then_verify_roundtrip_and_corruption(oracle):
    """Generate side writes ~csum into the TCP header (Send.cpp:448-449);
    the receive side accepts iff the recomputed value is 0xffff
    (Processor.cpp:121-131). Corrupt some segments: exactly those fail."""
    rng = np.random.default_rng(99)
    n, L = 4096, 1480
    segs = rng.integers(0, 256, (n, L), dtype=np.uint8)
    segs[:, 16:18] = 0                                   # chksum field zeroed
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    arena = d(segs.reshape(-1))
    offs = d(fixed_offsets(n, L))
    lens = d(np.full(n, L, np.uint16))
    gen = tulips_amd.batch(arena, offs, lens, src=d(src), dst=d(dst),
                           mode=MODE_TCP | FLAG_COMPLEMENT)
    g = u16(gen)
    segs[:, 16] = (g & 0xFF).astype(np.uint8)            # stored as the u16 in memory
    segs[:, 17] = (g >> 8).astype(np.uint8)
    bad_idx = rng.choice(n, 37, replace=False)
    for i in bad_idx:
        segs[i, int(rng.integers(0, L))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    arena = d(segs.reshape(-1))
    out = torch.empty(n, dtype=torch.uint16, device=DEV)
    bad = tulips_amd.verify(arena, offs, lens, src=d(src), dst=d(dst), mode=MODE_TCP, out=out)
    o = u16(out)
    assert int(h(bad)[0]) == 37
    assert set(np.nonzero(o != 0xFFFF)[0]) == set(bad_idx)
    exp = oracle.batch(segs.reshape(-1), fixed_offsets(n, L), np.full(n, L, np.uint16),
                       src=src, dst=dst, mode=MODE_TCP)
    np.testing.assert_array_equal(o, exp)


def test_verify_all_bad_repeat_and_two_streams(oracle):
    """The bad count is added per block into per-stream counter shards and
    summed by a finalize launch: an all-bad burst (random bytes) counts every
    segment, back-to-back calls on one stream each see zeroed shards, calls
    on two streams keep separate shards, and n = 0 writes 0."""
    rng = np.random.default_rng(7)
    n, L = 65536, 1500
    arena = d(rng.integers(0, 256, n * L, dtype=np.uint8))
    offs = d(fixed_offsets(n, L))
    lens = d(np.full(n, L, np.uint16))
    exp = oracle.batch(h(arena), fixed_offsets(n, L), np.full(n, L, np.uint16),
                       mode=MODE_INET, nthreads=8)
    want = int(np.count_nonzero(exp != 0xFFFF))
    assert want > n - 10
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    cnts = [torch.full((1,), -1, dtype=torch.int32, device=DEV) for _ in range(6)]
    torch.cuda.synchronize()
    for k, c in enumerate(cnts):
        st = (s1 if k % 2 else s2).cuda_stream
        sub = n if k < 4 else 1000 * k
        assert csum.lib.tulips_csum_verify(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                           None, None, None, c.data_ptr(), sub,
                                           MODE_INET, st) == 0
    torch.cuda.synchronize()
    got = [int(h(c)[0]) for c in cnts]
    assert got[:4] == [want] * 4
    assert got[4] == int(np.count_nonzero(exp[:4000] != 0xFFFF))
    assert got[5] == int(np.count_nonzero(exp[:5000] != 0xFFFF))
    c = torch.full((1,), -1, dtype=torch.int32, device=DEV)
    assert csum.lib.tulips_csum_verify(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                       None, None, None, c.data_ptr(), 0, MODE_INET,
                                       torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert int(h(c)[0]) == 0


def test_ipv4_headers_batch(oracle):
    rng = np.random.default_rng(4)
    n = 10000
    hdrs = rng.integers(0, 256, (n, 20), dtype=np.uint8)
    exp = np.array([oracle.ipv4_checksum(hdrs[i].tobytes()) for i in range(n)], np.uint16)
    out = tulips_amd.batch_fixed(d(hdrs.reshape(-1)), 20, 20, n, mode=MODE_INET)
    np.testing.assert_array_equal(u16(out), exp)


# -- end-to-end host path ---------------------------------------------------
@pytest.mark.parametrize("pinned", [False, True])
def test_host_context_path(golden, oracle, pinned):
    b = golden.digests()["batches"]["ZIPF"]
    n = b["n"]
    lens = oracle.zipf_lengths(n)
    offs = packed_offsets(lens)
    arena_np = oracle.splitmix_bytes(int(lens.astype(np.int64).sum()))
    if pinned:
        pt = torch.from_numpy(arena_np).pin_memory()
        arena_arg = pt.data_ptr()
    else:
        arena_arg = arena_np
    with csum.HostContext(0, chunk_bytes=8 << 20) as ctx:   # many chunks
        out = ctx.batch(arena_arg, offs, lens)
    assert f"{oracle.fnv1a_u16(out):016x}" == b["fnv1a64"]
    src = np.full(n, ip4(10, 1, 0, 1), np.uint32)
    dst = np.full(n, ip4(10, 1, 0, 2), np.uint32)
    with csum.HostContext(0) as ctx:
        out = ctx.batch(arena_np, offs, lens, src=src, dst=dst, mode=MODE_TCP)
    assert f"{oracle.fnv1a_u16(out):016x}" == golden.digests()["batches"]["ZIPF-tcp"]["fnv1a64"]


def test_host_context_span_straddling_two_pinned_blocks(oracle):
    """a chunk's segments in two separate page-locked
    allocations (offsets relative to the first, reaching into the second).
    Their hull is not one allocation, so the context must pack them rather
    than DMA the hull (which would read memory between the blocks); results
    equal the oracle's either way. Also blocks allocated back to back, so the
    hull is small enough for the direct path."""
    import ctypes as C
    lib = csum.lib
    rng = np.random.default_rng(606)
    size = 1 << 20
    ptrs = []
    try:
        for _ in range(4):
            p = C.c_void_p()
            assert lib.tulips_csum_host_alloc(size, C.byref(p)) == 0
            ptrs.append(p.value)
        for a, b in ((ptrs[0], ptrs[1]), (ptrs[2], ptrs[3])):
            va = np.ctypeslib.as_array((C.c_uint8 * size).from_address(a))
            vb = np.ctypeslib.as_array((C.c_uint8 * size).from_address(b))
            va[:] = rng.integers(0, 256, size, dtype=np.uint8)
            vb[:] = rng.integers(0, 256, size, dtype=np.uint8)
            n = 400
            lens = rng.integers(1, 3000, n).astype(np.uint16)
            at = rng.integers(0, size - 3000, n).astype(np.uint64)
            in_b = np.arange(n) >= n // 2
            offs = np.array([(int(at[i]) + (b - a if in_b[i] else 0)) % 2**64
                             for i in range(n)], dtype=np.uint64)
            exp = np.array([oracle.checksum(0, (vb if in_b[i] else va)
                                            [int(at[i]):int(at[i]) + int(lens[i])].tobytes())
                            for i in range(n)], np.uint16)
            with csum.HostContext(0) as ctx:
                got = ctx.batch(a, offs, lens)
            np.testing.assert_array_equal(got, exp)
    finally:
        for p in ptrs:
            lib.tulips_csum_host_free(C.c_void_p(p))


def test_empty_batch_is_noop():
    arena = torch.zeros(16, dtype=torch.uint8, device=DEV)
    offs = torch.zeros(0, dtype=torch.int64, device=DEV)
    lens = torch.empty(0, dtype=torch.uint16, device=DEV)
    out = tulips_amd.batch(arena, offs, lens)
    assert out.numel() == 0


@pytest.mark.parametrize("length,group,unroll", [(1500, 32, 4), (9000, 64, 12), (64, 16, 2)])
def test_fixed_small_workgroups(length, group, unroll):
    """Fixed-length batches also take 64- and 128-thread workgroups (one
    subgroup per segment, nothing shared in the workgroup): results equal the
    default launch's, odd counts and a capped grid included."""
    n = 4099
    arena = torch.empty(n * length + 64, dtype=torch.uint8, device=DEV)
    benchlib.fill_splitmix(arena, n * length, seed=0x5EED + length)
    st = torch.cuda.current_stream().cuda_stream
    want = torch.empty(n, dtype=torch.int16, device=DEV)   # u16 results, viewed signed
    assert csum.lib.tulips_csum_batch_fixed(arena.data_ptr(), length, length, None, None, None,
                                            want.data_ptr(), n, 0, st) == 0
    for block, cap in ((64, 0), (128, 0), (64, 5), (128, 9)):
        got = torch.full((n,), 0xA5A5 - 0x10000, dtype=torch.int16, device=DEV)   # poison
        t = csum.Tuning(group=group, unroll=unroll, nontemporal=1, block=block, max_blocks=cap)
        assert csum.lib.tulips_csum_batch_fixed_tuned(arena.data_ptr(), length, length, None,
                                                      None, None, got.data_ptr(), n, 0, t,
                                                      st) == 0
        torch.cuda.synchronize()
        assert torch.equal(got, want), (block, cap)
    bad = csum.Tuning(group=group, unroll=unroll, block=96)
    assert csum.lib.tulips_csum_batch_fixed_tuned(arena.data_ptr(), length, length, None, None,
                                                  None, want.data_ptr(), n, 0, bad, st) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("group,unroll,stride,length", [(32, 3, 1500, 1500), (16, 6, 2048, 1514),
                                                        (32, 3, 1501, 37)])
def test_gpu_stream_read_slots_geom(group, unroll, stride, length):
    """The load-pattern ceilings bench.py quotes run on any slot alignment and
    read only inside the slots' 16-byte chunks (the buffer ends right after
    the last slot's last chunk)."""
    import torch
    from tulips_amd import csum
    n = 4097
    nbytes = ((n - 1) * stride + length + 15) // 16 * 16
    buf = torch.zeros(nbytes, dtype=torch.uint8, device="cuda:0")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda:0")
    assert benchlib.lib.tulips_csum_stream_read_slots_geom(buf.data_ptr(), stride, length, n,
                                                           group, unroll, sink.data_ptr(),
                                                           None) == 0
    torch.cuda.synchronize()
    assert int(sink.sum().item()) == 0
