"""Batched receive-side frame validation.

Pins: tests/golden/frames.npz — 3000 Ethernet frames (well-formed, with IP /
TCP bit flips, IP options, fragments, UDP, ARP, truncations, runts, bogus
total lengths) whose expected TULIPS_FRAME_* flags were computed with the
REFERENCE's own ipv4::checksum and tcpv4::Processor::checksum
(tests/golden/make_golden.py::frames). Larger cases (mutations, jumbo
frames, every base alignment) are checked against the oracle's
orc_validate_frames, itself pinned to the fixture here.
"""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "frames.npz")

IPV4, IP_OK, TCP, L4_OK, TRUNC = 0x01, 0x02, 0x04, 0x08, 0x10


def frames_fixture():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def counters_of(flags):
    f = np.asarray(flags)
    ipv4 = (f & IPV4) != 0
    tcp = (f & TCP) != 0
    return np.array([ipv4.sum(), (ipv4 & ((f & IP_OK) == 0)).sum(), tcp.sum(),
                     (tcp & ((f & L4_OK) == 0)).sum()], dtype=np.uint32)


def make_frame(oracle, rng, payload):
    """Well-formed Ethernet/IPv4/TCP frame, checksums from the oracle."""
    src = int(rng.integers(0, 2**32))
    dst = int(rng.integers(0, 2**32))
    tcp = bytearray(rng.integers(0, 256, 20, dtype=np.uint8).tobytes())
    tcp[12] = 0x50
    tcp[16:18] = b"\0\0"
    seg = bytes(tcp) + rng.integers(0, 256, payload, dtype=np.uint8).tobytes()
    c = (~oracle.tcp_checksum(src, dst, seg)) & 0xFFFF
    seg = seg[:16] + c.to_bytes(2, "little") + seg[18:]
    ip = bytearray(b"\x45\x00" + (20 + len(seg)).to_bytes(2, "big") + b"\x12\x34\x40\x00\x40\x06"
                   + b"\0\0" + src.to_bytes(4, "little") + dst.to_bytes(4, "little"))
    c = (~oracle.ipv4_checksum(bytes(ip))) & 0xFFFF
    ip[10:12] = c.to_bytes(2, "little")
    return bytes(rng.integers(0, 256, 12, dtype=np.uint8).tobytes() + b"\x08\x00" + ip + seg)


def pack(frames, rng, gap=16, lead=0):
    offs, pos, parts = [], lead, [bytes(lead)]
    for f in frames:
        offs.append(pos)
        g = int(rng.integers(0, gap)) if gap else 0
        parts.append(f + bytes(g))
        pos += len(f) + g
    arena = np.frombuffer(b"".join(parts) + bytes(64), dtype=np.uint8)
    return arena, np.array(offs, dtype=np.uint64), np.array([len(f) for f in frames],
                                                             dtype=np.uint16)


def mutate(fx, rng, nflips):
    """The fixture arena with random byte flips (header-heavy)."""
    arena = fx["arena"].copy()
    offs, lens = fx["offsets"], fx["lengths"]
    pick = rng.integers(0, len(offs), nflips)
    where = np.minimum(rng.integers(0, 64, nflips), np.maximum(lens[pick].astype(np.int64) - 1, 0))
    arena[offs[pick].astype(np.int64) + where] ^= rng.integers(1, 256, nflips, dtype=np.uint8)
    return arena


# ---------------------------------------------------------------- CPU -----
def test_oracle_matches_fixture(oracle):
    fx = frames_fixture()
    got = oracle.validate_frames(fx["arena"], fx["offsets"], fx["lengths"])
    np.testing.assert_array_equal(got, fx["expect"])


def test_fixture_covers_every_outcome():
    fx = frames_fixture()
    seen = set(int(x) for x in np.unique(fx["expect"]))
    # not IPv4, runt, IPv4 only (bad/good csum), TCP good/bad, truncated
    for want in (0, TRUNC, IPV4, IPV4 | IP_OK, IPV4 | IP_OK | TCP | L4_OK,
                 IPV4 | IP_OK | TCP, IPV4 | TCP | L4_OK, IPV4 | IP_OK | TCP | TRUNC):
        assert want in seen, hex(want)
    assert int(fx["lengths"].min()) == 0 and int(fx["lengths"].max()) >= 1514


def test_oracle_jumbo_frames(oracle):
    rng = np.random.default_rng(5)
    fr = [make_frame(oracle, rng, p) for p in (8946, 9000 - 54, 65535 - 54)]
    arena, offs, lens = pack(fr, rng)
    assert list(oracle.validate_frames(arena, offs, lens)) == [0x0F] * 3


def test_capi_arguments_without_gpu():
    from tulips_amd import csum
    L = csum.lib
    assert L.tulips_csum_validate_frames(None, None, None, 0, None, None, None) == 0
    # neither flags nor counters
    assert L.tulips_csum_validate_frames(0x1000, 0x1000, 0x1000, 4, None, None, None) == 1
    assert L.tulips_csum_validate_frames(None, 0x1000, 0x1000, 4, 0x1000, None, None) == 1
    assert L.tulips_csum_validate_frames_host(None, None, None, None, 0, None, None) == 1
    for name in ("FRAME_IPV4", "FRAME_IP_CSUM_OK", "FRAME_TCP", "FRAME_L4_CSUM_OK",
                 "FRAME_TRUNCATED"):
        assert hasattr(csum, name)
    assert (csum.FRAME_IPV4, csum.FRAME_IP_CSUM_OK, csum.FRAME_TCP, csum.FRAME_L4_CSUM_OK,
            csum.FRAME_TRUNCATED) == (IPV4, IP_OK, TCP, L4_OK, TRUNC)


def test_cpu_validation_matches_fixture():
    """tulips_csum_validate_frames_cpu (the library's host code, used by the
    gpucsum decorator below its crossover) against the reference-computed
    flags, and its counters."""
    from tulips_amd import csum
    fx = frames_fixture()
    got, cnt = csum.validate_frames_cpu(fx["arena"], fx["offsets"], fx["lengths"],
                                        with_counters=True)
    np.testing.assert_array_equal(got, fx["expect"])
    np.testing.assert_array_equal(cnt, counters_of(fx["expect"]))


def test_cpu_validation_mutations_and_jumbo(oracle):
    from tulips_amd import csum
    fx = frames_fixture()
    rng = np.random.default_rng(404)
    for _ in range(4):
        arena = mutate(fx, rng, 2500)
        exp = oracle.validate_frames(arena, fx["offsets"], fx["lengths"])
        np.testing.assert_array_equal(
            csum.validate_frames_cpu(arena, fx["offsets"], fx["lengths"]), exp)
    fr = [make_frame(oracle, rng, p) for p in (0, 1, 8946, 65535 - 54)]
    for lead in (0, 1, 3):
        arena, offs, lens = pack(fr, rng, lead=lead)
        assert list(csum.validate_frames_cpu(arena, offs, lens)) == [0x0F] * 4
    # arguments: n == 0 is a no-op; neither flags nor counters
    L = csum.lib
    assert L.tulips_csum_validate_frames_cpu(None, None, None, 0, None, None) == 0
    assert L.tulips_csum_validate_frames_cpu(0x1000, 0x1000, 0x1000, 3, None, None) == 1


# ---------------------------------------------------------------- GPU -----
def _dev(*arrs):
    import torch
    return [torch.from_numpy(np.array(a, copy=True)).to("cuda:0") for a in arrs]


def _run(arena, offs, lens, counters=True):
    import torch
    from tulips_amd import csum
    a, o, l = _dev(arena, offs.astype(np.int64), lens.view(np.int16))
    cnt = torch.full((4,), -1, dtype=torch.int32, device="cuda:0") if counters else None
    fl = csum.validate_frames(a, o, l, counters=cnt)
    torch.cuda.synchronize()
    c = cnt.cpu().numpy().view(np.uint32) if counters else None
    return fl.cpu().numpy(), c


@pytest.mark.gpu
def test_gpu_fixture():
    fx = frames_fixture()
    got, cnt = _run(fx["arena"], fx["offsets"], fx["lengths"])
    np.testing.assert_array_equal(got, fx["expect"])
    np.testing.assert_array_equal(cnt, counters_of(fx["expect"]))


@pytest.mark.gpu
def test_gpu_counters_repeat_streams_and_grid_caps():
    """Counters are summed per block into per-stream shards and finalised
    after the launch: back-to-back calls on one stream (the shards must come
    back zeroed), two streams at once, and capped grids (many frames per
    block) all give the oracle's totals."""
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    exp = counters_of(fx["expect"])
    a, o, l = _dev(fx["arena"], fx["offsets"].astype(np.int64), fx["lengths"].view(np.int16))
    n = len(fx["offsets"])
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    cnts = [torch.full((4,), -1, dtype=torch.int32, device="cuda:0") for _ in range(6)]
    torch.cuda.synchronize()
    for k, c in enumerate(cnts):
        st = (s1 if k % 2 else s2).cuda_stream
        assert csum.lib.tulips_csum_validate_frames(a.data_ptr(), o.data_ptr(), l.data_ptr(),
                                                    n, None, c.data_ptr(), st) == 0
    torch.cuda.synchronize()
    for c in cnts:
        np.testing.assert_array_equal(c.cpu().numpy().view(np.uint32), exp)
    st = torch.cuda.current_stream().cuda_stream
    for cap, blk in ((1, 256), (3, 1024), (40, 256), (0, 512), (0, 64), (5, 128)):
        t = csum.Tuning(group=16, unroll=6, nontemporal=1, max_blocks=cap, block=blk)
        c = torch.full((4,), -1, dtype=torch.int32, device="cuda:0")
        assert csum.lib.tulips_csum_frames_tuned(0, a.data_ptr(), o.data_ptr(), l.data_ptr(),
                                                 n, None, c.data_ptr(), t, st) == 0
        torch.cuda.synchronize()
        np.testing.assert_array_equal(c.cpu().numpy().view(np.uint32), exp, err_msg=f"{cap} {blk}")


@pytest.mark.gpu
def test_gpu_counters_only():
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    a, o, l = _dev(fx["arena"], fx["offsets"].astype(np.int64), fx["lengths"].view(np.int16))
    cnt = torch.zeros(4, dtype=torch.int32, device="cuda:0")
    assert csum.validate_frames(a, o, l, counters=cnt, want_flags=False) is None
    torch.cuda.synchronize()
    np.testing.assert_array_equal(cnt.cpu().numpy().view(np.uint32),
                                  counters_of(fx["expect"]))


@pytest.mark.gpu
@pytest.mark.parametrize("shift", range(16))
def test_gpu_every_base_alignment(shift):
    fx = frames_fixture()
    arena = np.concatenate([np.zeros(shift, np.uint8), fx["arena"]])
    got, _ = _run(arena, fx["offsets"] + np.uint64(shift), fx["lengths"], counters=False)
    np.testing.assert_array_equal(got, fx["expect"])


@pytest.mark.gpu
def test_gpu_mutations_vs_oracle(oracle):
    fx = frames_fixture()
    rng = np.random.default_rng(11)
    for rnd in range(4):
        arena = mutate(fx, rng, 2000)
        exp = oracle.validate_frames(arena, fx["offsets"], fx["lengths"])
        got, cnt = _run(arena, fx["offsets"], fx["lengths"])
        np.testing.assert_array_equal(got, exp, err_msg=f"round {rnd}")
        np.testing.assert_array_equal(cnt, counters_of(exp))


@pytest.mark.gpu
def test_gpu_jumbo_and_max_frames(oracle):
    rng = np.random.default_rng(6)
    pays = [8946, 9000 - 54, 16000, 32768, 65535 - 54, 0, 1, 1460]
    fr = [make_frame(oracle, rng, p) for p in pays]
    bad = bytearray(fr[4])
    bad[-1] ^= 0x40                     # last byte of a 65535-byte frame
    fr.append(bytes(bad))
    arena, offs, lens = pack(fr, rng)
    exp = oracle.validate_frames(arena, offs, lens)
    assert list(exp[:-1]) == [0x0F] * len(pays) and exp[-1] == 0x07
    got, _ = _run(arena, offs, lens)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.gpu
def test_gpu_large_batch_tiled():
    """The fixture tiled 256x (768k frames, ~312 MB) — many grid-stride rounds."""
    fx = frames_fixture()
    reps = 256
    span = np.uint64(len(fx["arena"]))
    arena = np.tile(fx["arena"], reps)
    offs = (fx["offsets"][None, :] + span * np.arange(reps, dtype=np.uint64)[:, None]).ravel()
    lens = np.tile(fx["lengths"], reps)
    got, cnt = _run(arena, offs, lens)
    exp = np.tile(fx["expect"], reps)
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(cnt, counters_of(exp))


@pytest.mark.gpu
@pytest.mark.parametrize("pinned", [False, True])
def test_gpu_host_context(oracle, pinned):
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    rng = np.random.default_rng(12)
    arena = mutate(fx, rng, 1500)
    exp = oracle.validate_frames(arena, fx["offsets"], fx["lengths"])
    if pinned:
        t = torch.from_numpy(arena).pin_memory()
        src = t.numpy()
    else:
        src = arena
    # a small chunk so the 1.2 MB batch crosses many pipeline stages
    with csum.HostContext(0, chunk_bytes=1 << 17) as ctx:
        got, cnt = ctx.validate_frames(src, fx["offsets"], fx["lengths"], with_counters=True)
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(cnt, counters_of(exp))


@pytest.mark.gpu
@pytest.mark.parametrize("resident", [False, True])
@pytest.mark.parametrize("pinned", [True, False])
def test_gpu_zero_copy_bursts(oracle, pinned, resident):
    """tulips_csum_validate_frames_zc (the resident server, zc_mailbox.h):
    bursts of 1..1024 fixture frames (mutated) read in place from one
    page-locked arena, or packed from pageable memory, against the oracle;
    the arena rewritten between rounds (no stale bytes may survive in GPU
    caches); a burst past TULIPS_CSUM_ZC_MAX_FRAMES takes the staged path;
    counters; an idle gap longer than the server's 100 ms timeout (it exits
    and is restarted)."""
    import time
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    rng = np.random.default_rng(77 if pinned else 78)
    buf = torch.empty(len(fx["arena"]), dtype=torch.uint8)
    if pinned:
        buf = buf.pin_memory()
    arena = buf.numpy()
    n = len(fx["offsets"])
    with csum.HostContext(0, chunk_bytes=1 << 17) as ctx:
        ctx.set_lowlat(resident)
        for rnd in range(3):
            arena[:] = mutate(fx, rng, 1500)
            exp = oracle.validate_frames(arena, fx["offsets"], fx["lengths"])
            i = 0
            for b in (1, 1, 7, 61, 62, 63, 64, 65, 200, 1024, 1, 1025, 3):
                if i + b > n:
                    i = 0
                o, ln = fx["offsets"][i:i + b], fx["lengths"][i:i + b]
                got, cnt = ctx.validate_frames(arena, o, ln, with_counters=True,
                                               low_latency=True)
                np.testing.assert_array_equal(got, exp[i:i + b], err_msg=f"{rnd} {b}")
                np.testing.assert_array_equal(cnt, counters_of(exp[i:i + b]))
                i += b
            if rnd == 1:
                time.sleep(0.25)               # past the server's idle timeout
        # every frame of the fixture, one burst each
        for k in range(0, n, 97):
            got = ctx.validate_frames(arena, fx["offsets"][k:k + 1], fx["lengths"][k:k + 1],
                                      low_latency=True)
            assert got[0] == exp[k], k


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_gpu_zero_copy_tag_wraparound(oracle):
    """One launch per burst publishes a 16-bit tag per answering workgroup
    (tags cycle through 1..65535). A 1,024-frame burst (16 workgroups) under
    tag T, then 65,534 one-frame bursts (one workgroup each), then a
    1,024-frame burst of different bytes, tagged T again: its flags must be
    its own (the words of the earlier T are cleared before each launch), not
    the earlier burst's (csum_host.hip). Three wraps, the first
    starting at tag 65,530 (real requests: no test hook moves the sequence)."""
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    buf = torch.empty(len(fx["arena"]), dtype=torch.uint8).pin_memory()
    arena = buf.numpy()
    o = np.ascontiguousarray(fx["offsets"][:1024], dtype=np.uint64)
    ln = np.ascontiguousarray(fx["lengths"][:1024], dtype=np.uint16)
    one = np.empty(1, dtype=np.uint8)
    zc = csum.lib.tulips_csum_validate_frames_zc

    def fillers(k, ctx):
        for _ in range(k):
            assert zc(ctx._h, arena.ctypes.data, o.ctypes.data, ln.ctypes.data, 1,
                      one.ctypes.data, None) == 0

    with csum.HostContext(0) as ctx:
        arena[:] = fx["arena"]
        fillers(65529, ctx)                              # the next request is tagged 65,530
        for wrap in range(3):
            arena[:] = fx["arena"]
            got = ctx.validate_frames(arena, o, ln, low_latency=True)       # tag T
            np.testing.assert_array_equal(got, fx["expect"][:1024])
            fillers(65534, ctx)                          # every other tag once
            # the same tag again, different bytes (every frame's IP header hit)
            arena[o.astype(np.int64) + 15] ^= 0xFF
            exp = oracle.validate_frames(arena, o, ln)
            assert not np.array_equal(exp, fx["expect"][:1024])
            got = ctx.validate_frames(arena, o, ln, low_latency=True)       # tag T
            np.testing.assert_array_equal(got, exp)
            fillers(977, ctx)                            # the next wrap starts elsewhere


@pytest.mark.gpu
def test_gpu_zero_copy_pinned_range_reused(oracle):
    """The zero-copy path looks the page-locked allocation up on every call:
    an arena freed and replaced by another allocation (page-locked or
    pageable) at the same or another address is read from where it is now
    (csum_host.hip zc_validate)."""
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    rng = np.random.default_rng(12)
    o, ln = fx["offsets"][:200], fx["lengths"][:200]
    with csum.HostContext(0) as ctx:
        for rnd in range(6):
            data = mutate(fx, rng, 400)
            exp = oracle.validate_frames(data, o, ln)
            buf = torch.from_numpy(data.copy())
            if rnd % 2 == 0:
                buf = buf.pin_memory()
            got = ctx.validate_frames(buf.numpy(), o, ln, low_latency=True)
            np.testing.assert_array_equal(got, exp, err_msg=str(rnd))
            del buf


@pytest.mark.gpu
def test_gpu_zero_copy_two_contexts_and_destroy_while_serving(oracle):
    """Two contexts with live servers on one GPU, calls interleaved, a staged
    (non-zc) batch on one of them in between; destroying a context stops its
    server (the call returns, the other keeps serving)."""
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    arena = torch.from_numpy(mutate(fx, np.random.default_rng(5), 900)).pin_memory().numpy()
    exp = oracle.validate_frames(arena, fx["offsets"], fx["lengths"])
    a = csum.HostContext(0)
    a.set_lowlat(True)                          # one resident, one launch per burst
    with csum.HostContext(0) as b:
        for k in range(0, 2000, 50):
            sl = slice(k, k + 50)
            for ctx in (a, b):
                got = ctx.validate_frames(arena, fx["offsets"][sl], fx["lengths"][sl],
                                          low_latency=True)
                np.testing.assert_array_equal(got, exp[sl])
            if k == 500:
                got = a.validate_frames(arena, fx["offsets"], fx["lengths"])
                np.testing.assert_array_equal(got, exp)
        a.close()
        got = b.validate_frames(arena, fx["offsets"][:64], fx["lengths"][:64], low_latency=True)
        np.testing.assert_array_equal(got, exp[:64])


def test_zero_copy_arguments_without_gpu():
    from tulips_amd import csum
    f = csum.lib.tulips_csum_validate_frames_zc
    assert f(None, 1, 1, 1, 4, 1, None) == 1                 # no context
    assert f(None, None, None, None, 0, None, None) == 1
    assert csum.lib.tulips_csum_ctx_set_lowlat(None, 1) == 1


# ------------------------------------------------- send-side generation -----
def scramble_fields(fx, rng):
    """The fixture arena with both checksum fields of every frame overwritten
    by random bytes (generation must not depend on what they held)."""
    arena = fx["arena"].copy()
    for o, ln in zip(fx["offsets"].astype(np.int64), fx["lengths"].astype(np.int64)):
        for fld in (24, 50):
            if ln >= fld + 2:
                arena[o + fld:o + fld + 2] = rng.integers(0, 256, 2, dtype=np.uint8)
    return arena


def test_oracle_generate_reproduces_reference_bytes(oracle):
    """Frames the fixture built with the reference's own ipv4::checksum and
    tcpv4 checksum (make_golden.py::_make_frame) are reproduced bit-exactly."""
    fx = frames_fixture()
    rng = np.random.default_rng(21)
    gen, flags = oracle.generate_frames(scramble_fields(fx, rng), fx["offsets"], fx["lengths"])
    good = np.nonzero(fx["expect"] == (IPV4 | IP_OK | TCP | L4_OK))[0]
    assert len(good) > 500
    for i in good:
        o, ln = int(fx["offsets"][i]), int(fx["lengths"][i])
        assert bytes(gen[o:o + ln]) == bytes(fx["arena"][o:o + ln]), i
        assert flags[i] == (IPV4 | IP_OK | TCP | L4_OK)
    # after generation every complete frame verifies
    v = oracle.validate_frames(gen, fx["offsets"], fx["lengths"])
    wrote_l4 = (flags & L4_OK) != 0
    assert np.all((v[(flags & IPV4) != 0] & IP_OK) != 0)
    assert np.all((v[wrote_l4] & L4_OK) != 0)


@pytest.mark.gpu
@pytest.mark.parametrize("shift", [0, 1, 2, 3, 5, 8, 13, 15])
def test_gpu_generate_matches_oracle(oracle, shift):
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    rng = np.random.default_rng(100 + shift)
    src = np.concatenate([np.zeros(shift, np.uint8), scramble_fields(fx, rng)])
    offs = fx["offsets"] + np.uint64(shift)
    exp_arena, exp_flags = oracle.generate_frames(src, offs, fx["lengths"])
    a, o, l = _dev(src, offs.astype(np.int64), fx["lengths"].view(np.int16))
    fl = csum.generate_frames(a, o, l)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(fl.cpu().numpy(), exp_flags)
    got = a.cpu().numpy()
    assert np.array_equal(got, exp_arena), np.nonzero(got != exp_arena)[0][:10]


@pytest.mark.gpu
@pytest.mark.parametrize("slot,shift", [(2048, 0), (64, 0), (2048, 64), (2048, 32), (128, 0)])
def test_gpu_generate_in_slots_writes_whole_lines(oracle, slot, shift):
    """In-place generation on frames in slots (the receive/transmit ring
    layout, 64-byte aligned or not): every byte of the arena equals the
    oracle's (fields generated, nothing else changed, bytes between the
    frames untouched), the fixture's short frames and runts included."""
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    rng = np.random.default_rng(slot + shift)
    src = scramble_fields(fx, rng)
    lens = fx["lengths"].copy()
    keep = lens <= slot
    offs_fx, lens = fx["offsets"][keep], lens[keep]
    n = len(lens)
    arena = rng.integers(0, 256, shift + n * slot + 64, dtype=np.uint8)
    offs = (np.arange(n, dtype=np.uint64) * np.uint64(slot) + np.uint64(shift))
    for i in range(n):
        o, ln = int(offs_fx[i]), int(lens[i])
        arena[int(offs[i]):int(offs[i]) + ln] = src[o:o + ln]
    exp_arena, exp_flags = oracle.generate_frames(arena, offs, lens)
    a, o, l = _dev(arena, offs.astype(np.int64), lens.view(np.int16))
    fl = csum.generate_frames(a, o, l)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(fl.cpu().numpy(), exp_flags)
    got = a.cpu().numpy()
    assert np.array_equal(got, exp_arena), np.nonzero(got != exp_arena)[0][:10]


@pytest.mark.gpu
def test_gpu_generate_mutated_and_jumbo(oracle):
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    rng = np.random.default_rng(31)
    arena = mutate(fx, rng, 3000)
    exp_arena, exp_flags = oracle.generate_frames(arena, fx["offsets"], fx["lengths"])
    a, o, l = _dev(arena, fx["offsets"].astype(np.int64), fx["lengths"].view(np.int16))
    fl = csum.generate_frames(a, o, l)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(fl.cpu().numpy(), exp_flags)
    assert np.array_equal(a.cpu().numpy(), exp_arena)
    # jumbo / maximum frames, fields zeroed
    fr = [bytearray(make_frame(oracle, rng, p)) for p in (8946, 32768, 65535 - 54, 0)]
    want = [bytes(f) for f in fr]
    for f in fr:
        f[24:26] = b"\0\0"
        f[50:52] = b"\0\0"
    arena, offs, lens = pack([bytes(f) for f in fr], rng)
    a, o, l = _dev(arena, offs.astype(np.int64), lens.view(np.int16))
    csum.generate_frames(a, o, l, want_flags=False)
    torch.cuda.synchronize()
    got = a.cpu().numpy()
    for i, w in enumerate(want):
        assert bytes(got[int(offs[i]):int(offs[i]) + len(w)]) == w, i


def fields_of(arena, offs, lens, flags):
    """The compact fields a generated arena carries: IPv4 field (frame bytes
    24-25 as a little-endian u16) low, TCP field (50-51) high, 0 where the
    flags say nothing was written."""
    out = np.zeros(len(offs), np.uint32)
    for i, (o, ln) in enumerate(zip(offs.astype(np.int64), lens.astype(np.int64))):
        v = 0
        if flags[i] & IP_OK:
            v |= int(arena[o + 24]) | int(arena[o + 25]) << 8
        if flags[i] & L4_OK:
            v |= (int(arena[o + 50]) | int(arena[o + 51]) << 8) << 16
        out[i] = v
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("shift", [0, 1, 6, 15])
def test_gpu_generate_fields_matches_oracle(oracle, shift):
    """tulips_csum_generate_fields: the values orc_generate_frames writes
    (pinned to the reference-generated frames above), the frames untouched;
    fixture frames plus mutations, at several base alignments."""
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    rng = np.random.default_rng(700 + shift)
    for arena0 in (scramble_fields(fx, rng), mutate(fx, rng, 3000)):
        src = np.concatenate([np.zeros(shift, np.uint8), arena0])
        offs = fx["offsets"] + np.uint64(shift)
        exp_arena, exp_flags = oracle.generate_frames(src, offs, fx["lengths"])
        a, o, l = _dev(src, offs.astype(np.int64), fx["lengths"].view(np.int16))
        fields, fl = csum.generate_fields(a, o, l)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(fl.cpu().numpy(), exp_flags)
        np.testing.assert_array_equal(fields.cpu().numpy().view(np.uint32),
                                      fields_of(exp_arena, offs, fx["lengths"], exp_flags))
        assert np.array_equal(a.cpu().numpy(), src)          # read only
    good = np.nonzero(fx["expect"] == (IPV4 | IP_OK | TCP | L4_OK))[0]
    # on the reference-built frames the fields are the reference's own bytes
    a, o, l = _dev(fx["arena"], fx["offsets"].astype(np.int64), fx["lengths"].view(np.int16))
    fields, fl = csum.generate_fields(a, o, l, want_flags=False)
    torch.cuda.synchronize()
    got = fields.cpu().numpy().view(np.uint32)
    ref = fields_of(fx["arena"], fx["offsets"], fx["lengths"],
                    np.full(len(fx["offsets"]), IP_OK | L4_OK, np.uint8))
    np.testing.assert_array_equal(got[good], ref[good])


def test_generate_fields_arguments_without_gpu():
    from tulips_amd import csum
    f = csum.lib.tulips_csum_generate_fields
    assert f(None, None, None, 0, None, None, None) == 0       # n == 0: no-op
    assert f(None, 1, 1, 4, 1, None, None) == 1
    assert f(1, 1, 1, 4, None, None, None) == 1               # fields required


FRAME_GEOMETRIES = [(16, 4), (16, 6), (16, 8), (8, 8), (8, 16), (32, 3), (32, 4), (64, 2)]


@pytest.mark.gpu
@pytest.mark.parametrize("geo", FRAME_GEOMETRIES)
@pytest.mark.parametrize("nt,shift", [(1, 5), (0, 5), (1, 14)])
def test_gpu_every_frame_geometry(oracle, geo, nt, shift):
    """Validation and generation through tulips_csum_frames_tuned at every
    geometry, on mutated fixture frames shifted to an odd base (5: header
    words one dword and one byte into the chunk; 14: three dwords and two
    bytes, the other select bit of the per-lane funnel shift)."""
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    rng = np.random.default_rng(geo[0] * 100 + geo[1] + nt + shift)
    arena = np.concatenate([np.zeros(shift, np.uint8), mutate(fx, rng, 1500)])
    offs = fx["offsets"] + np.uint64(shift)
    t = csum.Tuning(group=geo[0], unroll=geo[1], nontemporal=nt, block=256 if nt else 512)
    a, o, l = _dev(arena, offs.astype(np.int64), fx["lengths"].view(np.int16))
    fl = torch.empty(len(offs), dtype=torch.uint8, device="cuda:0")
    cnt = torch.zeros(4, dtype=torch.int32, device="cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    ft = csum.lib.tulips_csum_frames_tuned
    assert ft(0, a.data_ptr(), o.data_ptr(), l.data_ptr(), len(offs), fl.data_ptr(),
              cnt.data_ptr(), t, st) == 0
    torch.cuda.synchronize()
    exp = oracle.validate_frames(arena, offs, fx["lengths"])
    np.testing.assert_array_equal(fl.cpu().numpy(), exp)
    np.testing.assert_array_equal(cnt.cpu().numpy().view(np.uint32), counters_of(exp))
    assert ft(1, a.data_ptr(), o.data_ptr(), l.data_ptr(), len(offs), fl.data_ptr(), None,
              t, st) == 0
    torch.cuda.synchronize()
    exp_arena, exp_flags = oracle.generate_frames(arena, offs, fx["lengths"])
    np.testing.assert_array_equal(fl.cpu().numpy(), exp_flags)
    assert np.array_equal(a.cpu().numpy(), exp_arena)


@pytest.mark.gpu
@pytest.mark.parametrize("sps", [2, 3])
@pytest.mark.parametrize("max_blocks", [0, 7, 300])
def test_gpu_validation_two_frames_per_subgroup(oracle, max_blocks, sps):
    """Validation at 16 x 6 with two frames per subgroup in flight
    (tuning.sps = 2) and as a software pipeline (sps = 3): mutated fixture
    frames at an odd base, odd frame counts (the second frame of the last
    subgroup absent), grid caps that make subgroups loop; flags and counters
    vs the oracle."""
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    rng = np.random.default_rng(2 + max_blocks)
    arena = np.concatenate([np.zeros(3, np.uint8), mutate(fx, rng, 2000)])
    for n in (len(fx["offsets"]), 2999, 17, 1):
        offs = fx["offsets"][:n] + np.uint64(3)
        lens = fx["lengths"][:n]
        t = csum.Tuning(group=16, unroll=6, nontemporal=1, max_blocks=max_blocks, sps=sps)
        a, o, l = _dev(arena, offs.astype(np.int64), lens.view(np.int16))
        fl = torch.full((n,), 0xA5, dtype=torch.uint8, device="cuda:0")
        cnt = torch.zeros(4, dtype=torch.int32, device="cuda:0")
        assert csum.lib.tulips_csum_frames_tuned(0, a.data_ptr(), o.data_ptr(), l.data_ptr(), n,
                                                 fl.data_ptr(), cnt.data_ptr(), t,
                                                 torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        exp = oracle.validate_frames(arena, offs, lens)
        np.testing.assert_array_equal(fl.cpu().numpy(), exp, err_msg=str(n))
        np.testing.assert_array_equal(cnt.cpu().numpy().view(np.uint32), counters_of(exp))


def test_frames_tuned_rejects_bad_geometry():
    from tulips_amd import csum
    f = csum.lib.tulips_csum_frames_tuned
    A = 0x1000
    assert f(0, A, A, A, 4, A, None, csum.Tuning(group=24, unroll=4), None) == 1
    assert f(2, A, A, A, 4, A, None, csum.Tuning(group=16, unroll=4), None) == 1
    assert f(0, A, A, A, 4, A, None, csum.Tuning(group=16, unroll=4, block=384), None) == 1
    assert f(0, A, A, A, 0, None, None, csum.Tuning(group=16, unroll=6), None) == 0
    # the pipelined form (sps 3) is built for at most 256 threads per block
    for blk in (512, 1024):
        assert f(0, A, A, A, 4, A, None,
                 csum.Tuning(group=16, unroll=6, sps=3, block=blk), None) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("pinned", [False, True])
def test_gpu_generate_host_context(oracle, pinned):
    """tulips_csum_generate_frames_host: host frames through the pinned
    pipeline, only the 4 field bytes per frame written back — byte-exact with
    the oracle (itself pinned to reference-generated frames above), across
    many pipeline stages (small chunk)."""
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    rng = np.random.default_rng(77)
    src = scramble_fields(fx, rng)
    exp_arena, exp_flags = oracle.generate_frames(src, fx["offsets"], fx["lengths"])
    arena = torch.from_numpy(src.copy()).pin_memory().numpy() if pinned else src.copy()
    with csum.HostContext(0, chunk_bytes=1 << 17) as ctx:
        fl = ctx.generate_frames(arena, fx["offsets"], fx["lengths"])
    np.testing.assert_array_equal(fl, exp_flags)
    assert np.array_equal(arena, exp_arena), np.nonzero(arena != exp_arena)[0][:10]
