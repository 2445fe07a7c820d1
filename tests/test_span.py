"""In-order arena batches (tulips_csum_batch_arena / tulips_csum_verify_arena,
KIND_SPAN in tulips_amd/csrc/csum_kernels.hip): the work is cut by arena
bytes, each segment finished by the workgroup its first byte falls in.

Checked against the reference's ZIPF / ZIPF-tcp digests (tests/golden) and the
CPU restatement (oracle/csum_oracle.c, pinned by tests/test_oracle.py) on
layouts that reach every branch of the kernel: empty, tiny (< 16 B, many per
chunk) and maximal (65,535 B, crossing several ranges) segments, gaps, an
unaligned arena base, empty segments at the arena end, more than 320 / 512
segments starting in one range, batches past 65,536 segments (more search
rounds), n = 1. Bar: bit-exact.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import (FLAG_COMPLEMENT, MODE_INET, MODE_RAW, MODE_TCP,  # noqa: E402
                    ip4, packed_offsets)

import tulips_amd  # noqa: E402
from tulips_amd import csum  # noqa: E402

DEV = "cuda:0"
# (chunks per lane, form): the split form, 0 = default (= 7). The library
# default is 7 chunks per lane (28 KiB ranges).
GEOMS = ((4, 0), (5, 0), (6, 0), (7, 7), (7, 0), (8, 0),
         # the tail-shaped cut (group 9; third entry: tail percent, 0 = 12)
         (7, 9), (8, 9, 50), (6, 9, 3),
         # ranges prioritised by quarter (group 10, the r05 ZIPF experiment)
         (7, 10), (6, 10))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def d(a):
    return torch.from_numpy(np.array(a, copy=True, order="C")).to(DEV)


def u16(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint16)


def tuning(geo, nt=1):
    u, halo = geo[:2]
    return csum.Tuning(kind=csum.KIND_SPAN, unroll=u, group=halo, nontemporal=nt,
                       sps=geo[2] if len(geo) > 2 else 0)


def in_order(rng, lens, max_gap=0, gap_p=0.0):
    """Offsets laying `lens` out in order with random gaps; returns
    (offsets, end of the last segment)."""
    gaps = np.where(rng.random(len(lens)) < gap_p,
                    rng.integers(0, max_gap + 1, len(lens)), 0).astype(np.uint64)
    ends = np.cumsum(lens.astype(np.uint64) + gaps)
    offs = ends - lens.astype(np.uint64)
    return offs.astype(np.uint64), int(ends[-1]) if len(ends) else 0


@pytest.mark.parametrize("name", ["ZIPF", "ZIPF-tcp"])
def test_zipf_digest(golden, oracle, name):
    import benchlib
    b = golden.digests()["batches"][name]
    n = b["n"]
    lens = oracle.zipf_lengths(n)
    offs = packed_offsets(lens)
    total = int(lens.astype(np.int64).sum())
    arena = torch.empty(total + 64, dtype=torch.uint8, device=DEV)
    benchlib.fill_splitmix(arena, total)
    kw = {}
    if b["mode"] == "tcp":
        kw = dict(src=d(np.full(n, ip4(10, 1, 0, 1), np.uint32)),
                  dst=d(np.full(n, ip4(10, 1, 0, 2), np.uint32)), mode=MODE_TCP)
    do, dl = d(offs), d(lens)
    for t in [None] + [tuning(g) for g in GEOMS]:
        out = tulips_amd.batch_arena(arena, do, dl, arena_bytes=total, tuning=t, **kw)
        assert f"{oracle.fnv1a_u16(u16(out)):016x}" == b["fnv1a64"], t


def _mixed(rng, n):
    lens = rng.integers(0, 3000, n).astype(np.uint16)
    lens[rng.random(n) < 0.1] = 0
    tiny = rng.random(n) < 0.1
    lens[tiny] = rng.integers(1, 16, int(tiny.sum()))
    k = rng.integers(0, n, 40)
    lens[k] = rng.integers(60000, 65536, 40)          # cross several ranges
    lens[n // 2:n // 2 + 3] = 65535
    t0 = n // 3
    lens[t0:t0 + 1500] = rng.integers(0, 6, 1500)     # > 512 starts in one range
    return lens


@pytest.mark.parametrize("u", GEOMS)
@pytest.mark.parametrize("base_off", [0, 1, 6, 15])
def test_random_layouts_vs_oracle(oracle, u, base_off):
    rng = np.random.default_rng(9100 + 16 * u[0] + 4 * u[1] + base_off)
    n = 12000 + base_off
    lens = _mixed(rng, n)
    lens[-3:] = 0                 # empty segments at the very end of the arena
    offs, arena_bytes = in_order(rng, lens, max_gap=200, gap_p=0.3)
    buf = rng.integers(0, 256, base_off + arena_bytes + 32, dtype=np.uint8)
    buf[base_off:base_off + 5000] = 0
    buf[base_off + 5000:base_off + 9000] = 0xFF
    arena = buf[base_off:base_off + arena_bytes]
    seeds = rng.integers(0, 65536, n, dtype=np.uint16)
    seeds[:50] = 0
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dbuf = d(buf)
    da = dbuf[base_off:]
    do, dl, ds_, dsrc, ddst = d(offs), d(lens), d(seeds), d(src), d(dst)
    for mode in (MODE_RAW, MODE_INET, MODE_TCP | FLAG_COMPLEMENT):
        exp = oracle.batch(np.ascontiguousarray(arena), offs, lens, seeds=seeds, src=src,
                           dst=dst, mode=mode, nthreads=8)
        for nt in (0, 1, 3):
            got = tulips_amd.batch_arena(da, do, dl, arena_bytes=arena_bytes, seeds=ds_,
                                         src=dsrc, dst=ddst, mode=mode, tuning=tuning(u, nt))
            np.testing.assert_array_equal(u16(got), exp, err_msg=f"{hex(mode)} nt={nt}")


@pytest.mark.parametrize("u", GEOMS)
def test_many_segments_more_search_rounds(oracle, u):
    """300,000 segments (two 256-ary rounds before the windows), short and
    tiny lengths, a few long ones."""
    rng = np.random.default_rng(77 + 4 * u[0] + u[1])
    n = 300000
    lens = rng.integers(0, 80, n).astype(np.uint16)
    lens[rng.integers(0, n, 30)] = 65535
    offs, end = in_order(rng, lens, max_gap=40, gap_p=0.2)
    arena = rng.integers(0, 256, end + 16, dtype=np.uint8)
    exp = oracle.batch(arena, offs, lens, mode=MODE_INET, nthreads=8)
    got = tulips_amd.batch_arena(d(arena), d(offs), d(lens), arena_bytes=end, mode=MODE_INET,
                                 tuning=tuning(u))
    np.testing.assert_array_equal(u16(got), exp)


@pytest.mark.parametrize("u", GEOMS)
def test_skewed_arena_falls_back_to_search(oracle, u):
    """Segment density far from even (the first tenth of the arena holds 95 %
    of the segments): the speculative offset window misses for most ranges
    and the workgroup's search takes over."""
    rng = np.random.default_rng(31 + 4 * u[0] + u[1])
    n = 40000
    lens = np.concatenate([rng.integers(0, 40, 38000), rng.integers(30000, 65536, 2000)])
    lens = lens.astype(np.uint16)
    offs, end = in_order(rng, lens, max_gap=3, gap_p=0.1)
    arena = rng.integers(0, 256, end + 16, dtype=np.uint8)
    exp = oracle.batch(arena, offs, lens, mode=MODE_INET, nthreads=8)
    got = tulips_amd.batch_arena(d(arena), d(offs), d(lens), arena_bytes=end, mode=MODE_INET,
                                 tuning=tuning(u))
    np.testing.assert_array_equal(u16(got), exp)
    # an arena much larger than the segments' span (trailing free space)
    got = tulips_amd.batch_arena(d(np.concatenate([arena, np.zeros(end, np.uint8)])), d(offs),
                                 d(lens), arena_bytes=2 * end, mode=MODE_INET,
                                 tuning=tuning(u))
    np.testing.assert_array_equal(u16(got), exp)


@pytest.mark.parametrize("lens", [[0], [1], [17], [65535], [0, 0, 0], [3, 0, 65535, 0, 9]])
def test_small_batches(oracle, lens):
    rng = np.random.default_rng(len(lens))
    lens = np.array(lens, np.uint16)
    offs, end = in_order(rng, lens, max_gap=7, gap_p=0.5)
    arena = rng.integers(0, 256, max(end, 1) + 16, dtype=np.uint8)
    exp = oracle.batch(arena, offs, lens, mode=MODE_RAW)
    for u in GEOMS:
        got = tulips_amd.batch_arena(d(arena), d(offs), d(lens), arena_bytes=end,
                                     tuning=tuning(u))
        np.testing.assert_array_equal(u16(got), exp, err_msg=str(u))


def test_verify_arena_counts(oracle):
    rng = np.random.default_rng(5)
    n = 40000
    lens = rng.integers(20, 1600, n).astype(np.uint16)
    offs, end = in_order(rng, lens)
    arena = rng.integers(0, 256, end + 16, dtype=np.uint8)
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    exp = oracle.batch(arena, offs, lens, src=src, dst=dst, mode=MODE_TCP, nthreads=8)
    want_bad = int(np.count_nonzero(exp != 0xFFFF))
    out = torch.empty(n, dtype=torch.int16, device=DEV)
    bad = tulips_amd.verify_arena(d(arena), d(offs), d(lens), arena_bytes=end, src=d(src),
                                  dst=d(dst), mode=MODE_TCP, out=out)
    torch.cuda.synchronize()
    assert int(bad.item()) == want_bad
    np.testing.assert_array_equal(u16(out), exp)
    bad = tulips_amd.verify_arena(d(arena), d(offs), d(lens), arena_bytes=end, src=d(src),
                                  dst=d(dst), mode=MODE_TCP)
    torch.cuda.synchronize()
    assert int(bad.item()) == want_bad


def test_generated_frames_verify_clean(oracle):
    """INET verification of in-order segments whose checksums were made to
    verify (seeded with the complement of their own sum): count 0."""
    rng = np.random.default_rng(8)
    n = 5000
    lens = rng.integers(40, 3000, n).astype(np.uint16) & ~np.uint16(1)
    offs, end = in_order(rng, lens, max_gap=64, gap_p=0.5)
    arena = rng.integers(0, 256, end + 16, dtype=np.uint8)
    raw = oracle.batch(arena, offs, lens, mode=MODE_RAW | FLAG_COMPLEMENT, nthreads=8)
    # store the complement as the last two bytes' big-endian word after zeroing them
    for i in range(n):
        o, L = int(offs[i]), int(lens[i])
        arena[o + L - 2:o + L] = 0
    raw = oracle.batch(arena, offs, lens, mode=MODE_RAW | FLAG_COMPLEMENT, nthreads=8)
    for i in range(n):
        o, L = int(offs[i]), int(lens[i])
        arena[o + L - 2] = raw[i] >> 8
        arena[o + L - 1] = raw[i] & 0xFF
    exp = oracle.batch(arena, offs, lens, mode=MODE_INET, nthreads=8)
    assert np.all(exp == 0xFFFF)
    bad = tulips_amd.verify_arena(d(arena), d(offs), d(lens), arena_bytes=end,
                                  mode=MODE_INET)
    torch.cuda.synchronize()
    assert int(bad.item()) == 0


def test_rejects_bad_arguments():
    t = csum.Tuning(kind=csum.KIND_PACKED, group=8, unroll=4)
    rc = csum.lib.tulips_csum_batch_arena_tuned(1, 16, 1, 1, None, None, None, 1, 4, 0, t,
                                                None)
    assert rc == 1
    t = tuning((13, 0))
    rc = csum.lib.tulips_csum_batch_arena_tuned(1, 16, 1, 1, None, None, None, 1, 4, 0, t,
                                                None)
    assert rc == 1
    # n == 0 is a no-op
    assert csum.lib.tulips_csum_batch_arena(None, 0, None, None, None, None, None, None,
                                            0, 0, None) == 0


@pytest.mark.parametrize("u", GEOMS)
def test_split_words_survive_contract_breaking_batch(oracle, u):
    """The split form's per-range words are left non-zero only by a batch that
    breaks the arena contract (overlapping segments); such residue carries an
    older epoch and must not leak into the next, valid, batch on the stream."""
    rng = np.random.default_rng(404 + u[0])
    n = 20000
    lens = rng.integers(1000, 9000, n).astype(np.uint16)
    offs, end = in_order(rng, lens)
    arena = rng.integers(0, 256, end + 16, dtype=np.uint8)
    da, dl = d(arena), d(lens)
    bad = offs.copy()
    bad[1::3] -= np.minimum(bad[1::3], np.uint64(6000))   # overlaps its predecessors
    bad = np.maximum.accumulate(bad)                      # sorted, still overlapping
    tulips_amd.batch_arena(da, d(bad), dl, arena_bytes=end, tuning=tuning(u))
    exp = oracle.batch(arena, offs, lens, mode=MODE_RAW, nthreads=8)
    for _ in range(3):
        got = tulips_amd.batch_arena(da, d(offs), dl, arena_bytes=end, tuning=tuning(u))
        np.testing.assert_array_equal(u16(got), exp)


@pytest.mark.parametrize("u", GEOMS)
def test_unsorted_and_out_of_arena_offsets_stay_inside(oracle, u):
    """offsets that break the arena contract — shuffled,
    past arena_bytes, near 2^64 — give undefined results but must not send a
    split part to a word outside the stream's array (or fault); the next valid
    batch on the stream is exact."""
    rng = np.random.default_rng(505 + u[0])
    n = 20000
    lens = rng.integers(100, 9000, n).astype(np.uint16)
    offs, end = in_order(rng, lens)
    arena = rng.integers(0, 256, end + 16, dtype=np.uint8)
    da, dl = d(arena), d(lens)
    exp = oracle.batch(arena, offs, lens, mode=MODE_RAW, nthreads=8)
    shuffled = rng.permutation(offs)
    far = offs.copy()
    far[::7] += np.uint64(end) * np.uint64(3)               # past the arena
    far[5::11] = np.uint64(2**64 - 4096) + far[5::11] % np.uint64(4000)  # wraps below base
    for bad in (shuffled, far, np.sort(far)):
        tulips_amd.batch_arena(da, d(bad.view(np.int64)), dl, arena_bytes=end, tuning=tuning(u))
        torch.cuda.synchronize()
        got = tulips_amd.batch_arena(da, d(offs), dl, arena_bytes=end, tuning=tuning(u))
        np.testing.assert_array_equal(u16(got), exp)
