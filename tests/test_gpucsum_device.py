"""transport::gpucsum::Device — the batched receive-validation decorator
(integration/include/tulips/transport/gpucsum/Device.h).

integration/_build/libgpucsum_test.so (integration/Makefile) is the decorator
compiled against the reference's headers, wrapping the reference's own
list::Device (src/transport/list/Device.cpp). The frames of
tests/golden/frames.npz are committed on a peer list device, polled through
the decorator, and the frames reaching the stack's Processor must be exactly
those whose reference-derived flags pass the VALIDATE_IP_CSUM /
VALIDATE_L4_CSUM hints, in arrival order (the drop rules of
src/transport/ofed/Device.cpp:528-545 and src/transport/ena/Device.cpp:316-340).
"""
import ctypes as C
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "integration", "_build", "libgpucsum_test.so")
GOLDEN = os.path.join(ROOT, "tests", "golden", "frames.npz")

VALIDATE_IP_CSUM, VALIDATE_L4_CSUM = 0x1, 0x2   # include/tulips/transport/Device.h:29-30

needs_harness = pytest.mark.skipif(not os.path.exists(HARNESS),
                                   reason="integration/_build not built (no reference tree)")


def harness():
    from tulips_amd import csum  # noqa: F401  (torch's HIP runtime first, then ours)
    lib = C.CDLL(HARNESS)
    f = lib.gpucsum_run
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint16,
                  C.c_int, C.c_void_p, C.c_void_p]
    return f


def fixture():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def expected_forwarded(flags, hints):
    f = flags.astype(np.int64)
    bad_ip = ((hints & VALIDATE_IP_CSUM) != 0) & ((f & 0x01) != 0) & ((f & 0x02) == 0)
    bad_l4 = ((hints & VALIDATE_L4_CSUM) != 0) & ((f & 0x04) != 0) & ((f & 0x08) == 0)
    bad_l4 &= ~bad_ip
    return (~(bad_ip | bad_l4)).astype(np.uint8), int(bad_ip.sum()), int(bad_l4.sum())


def run(fx, burst, hints, use_wait, n=None):
    f = harness()
    n = len(fx["offsets"]) if n is None else n
    arena = np.ascontiguousarray(fx["arena"])
    offs = np.ascontiguousarray(fx["offsets"][:n])
    lens = np.ascontiguousarray(fx["lengths"][:n])
    fwd = np.zeros(n, dtype=np.uint8)
    stats = np.zeros(5, dtype=np.uint64)
    rc = f(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, n, burst, hints,
           int(use_wait), fwd.ctypes.data, stats.ctypes.data)
    assert rc == 0, f"gpucsum_run rc={rc}"
    return fwd, stats


@needs_harness
def test_harness_exports():
    from tulips_amd import csum  # noqa: F401  (loading needs torch's runtime first)
    lib = C.CDLL(HARNESS)
    assert hasattr(lib, "gpucsum_run")
    # the decorator's vtable is in the library (C++ symbol of its poll override)
    assert hasattr(lib, "_ZN6tulips9transport7gpucsum6Device4pollERNS0_9ProcessorE")


@needs_harness
@pytest.mark.gpu
@pytest.mark.parametrize("hints", [3, 1, 2, 0])
@pytest.mark.parametrize("use_wait", [False, True])
def test_forwarded_frames_follow_hints(hints, use_wait):
    fx = fixture()
    fwd, st = run(fx, 256, hints, use_wait)
    exp, bad_ip, bad_l4 = expected_forwarded(fx["expect"], hints)
    np.testing.assert_array_equal(fwd, exp)
    n = len(exp)
    assert int(st[0]) == n and int(st[1]) == int(exp.sum())
    assert (int(st[2]), int(st[3])) == (bad_ip, bad_l4)
    assert int(st[4]) >= (n + 255) // 256


@needs_harness
@pytest.mark.gpu
@pytest.mark.parametrize("burst", [1, 7, 4096])
def test_burst_sizes(burst):
    fx = fixture()
    n = 600 if burst == 1 else None
    fwd, st = run(fx, burst, 3, False, n=n)
    exp, _, _ = expected_forwarded(fx["expect"][:len(fwd)], 3)
    np.testing.assert_array_equal(fwd, exp)
    if burst == 4096:
        assert int(st[4]) == 1          # the whole poll burst in one launch


def run_cpu_below(fx, burst, cpu_below, n=None):
    from tulips_amd import csum  # noqa: F401
    lib = C.CDLL(HARNESS)
    f = lib.gpucsum_run_cpu_below
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint16,
                  C.c_int64, C.c_void_p, C.c_void_p]   # int64_t cpu_below (gpucsum_harness.cpp)
    n = len(fx["offsets"]) if n is None else n
    arena = np.ascontiguousarray(fx["arena"])
    offs = np.ascontiguousarray(fx["offsets"][:n])
    lens = np.ascontiguousarray(fx["lengths"][:n])
    fwd = np.zeros(n, dtype=np.uint8)
    stats = np.zeros(6, dtype=np.uint64)
    rc = f(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, n, burst, 3, cpu_below,
           fwd.ctypes.data, stats.ctypes.data)
    assert rc == 0, f"gpucsum_run_cpu_below rc={rc}"
    return fwd, stats


@needs_harness
@pytest.mark.gpu
@pytest.mark.parametrize("burst", [1, 2, 8, 31, 32, 64, 256, 1024, 4096])
def test_cpu_crossover_by_burst(burst):
    """Config::cpu_below (default 32): bursts below it are validated on the
    polling thread by tulips_csum_validate_frames_cpu, the rest on the GPU;
    either way the frames forwarded are exactly those the reference-derived
    flags pass, in arrival order."""
    fx = fixture()
    n = min(len(fx["offsets"]), max(64 * burst, 600) if burst < 32 else len(fx["offsets"]))
    fwd, st = run_cpu_below(fx, burst, 32, n=n)
    exp, bad_ip, bad_l4 = expected_forwarded(fx["expect"][:n], 3)
    np.testing.assert_array_equal(fwd, exp)
    assert (int(st[2]), int(st[3])) == (bad_ip, bad_l4)
    full, rest = divmod(n, burst)         # one poll burst per `burst` frames
    gpu = (full if burst >= 32 else 0) + (1 if rest >= 32 else 0)
    cpu = (full if burst < 32 else 0) + (1 if 0 < rest < 32 else 0)
    assert (int(st[4]), int(st[5])) == (gpu, cpu)


def run_default_crossover(arena, offs, lens, burst):
    from tulips_amd import csum  # noqa: F401
    lib = C.CDLL(HARNESS)
    f = lib.gpucsum_run_cpu_below
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint16,
                  C.c_int64, C.c_void_p, C.c_void_p]
    n = len(offs)
    fwd = np.zeros(n, dtype=np.uint8)
    stats = np.zeros(6, dtype=np.uint64)
    rc = f(np.ascontiguousarray(arena).ctypes.data, np.ascontiguousarray(offs).ctypes.data,
           np.ascontiguousarray(lens).ctypes.data, n, burst, 3, -1, fwd.ctypes.data,
           stats.ctypes.data)
    assert rc == 0, f"gpucsum_run_cpu_below rc={rc}"
    return fwd, stats


@needs_harness
@pytest.mark.gpu
@pytest.mark.parametrize("burst", [1, 8, 64, 95, 96, 128, 256])
def test_default_crossover_frames_side(burst):
    """The decorator's default crossover (tulips_csum_burst_prefers_cpu: fewer
    than 96 frames and 96 x 1514 bytes, from the cold-frame measurement):
    fixture bursts (<= 1514 B frames) below 96 frames stay on the CPU, the
    others go to the GPU; the forwarded frames are exactly those the
    reference-derived flags pass."""
    from tulips_amd import csum
    fx = fixture()
    n = min(len(fx["offsets"]), 40 * burst) // burst * burst    # whole bursts only
    offs, lens = fx["offsets"][:n], fx["lengths"][:n]
    fwd, st = run_default_crossover(fx["arena"], offs, lens, burst)
    exp, bad_ip, bad_l4 = expected_forwarded(fx["expect"][:n], 3)
    np.testing.assert_array_equal(fwd, exp)
    cpu = gpu = 0
    for b0 in range(0, n, burst):
        ln = lens[b0:b0 + burst]
        if csum.lib.tulips_csum_burst_prefers_cpu(len(ln), int(ln.astype(np.int64).sum())):
            cpu += 1
        else:
            gpu += 1
    assert (int(st[4]), int(st[5])) == (gpu, cpu)
    assert (cpu > 0) == (burst < 96) and (gpu > 0) == (burst >= 96)


@needs_harness
@pytest.mark.gpu
def test_default_crossover_bytes_side(oracle):
    """Jumbo frames (9,014 B): fewer than 96 frames but past the bytes limit
    (145 KB) goes to the GPU, 12 of them (108 KB) stay on the CPU; corrupted
    frames are dropped either way."""
    from test_frames import make_frame
    rng = np.random.default_rng(96)
    frames = [bytearray(make_frame(oracle, rng, 8960)) for _ in range(120)]
    for k in range(0, 120, 7):
        frames[k][200] ^= 0x10          # bad TCP checksum
    offs = np.arange(120, dtype=np.uint64) * np.uint64(9216)
    arena = np.zeros(120 * 9216, dtype=np.uint8)
    for k, f in enumerate(frames):
        arena[k * 9216:k * 9216 + len(f)] = np.frombuffer(bytes(f), dtype=np.uint8)
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    assert lens[0] > 9000
    exp, _, bad_l4 = expected_forwarded(oracle.validate_frames(arena, offs, lens), 3)
    assert bad_l4 == len(range(0, 120, 7))
    from tulips_amd import csum
    for burst in (12, 128):
        fwd, st = run_default_crossover(arena, offs, lens, burst)
        np.testing.assert_array_equal(fwd, exp)
        # the decorator's flushes: `burst` frames or a full staging arena
        # (max(burst x 2 KiB, 128 KiB), frames 16 B-aligned), each sent to
        # the CPU or the GPU by the crossover
        cap, used, cur, cpu, gpu = max(burst * 2048, 1 << 17), 0, [], 0, 0
        for ln in list(lens) + [None]:
            if ln is None or len(cur) == burst or used + int(ln) > cap:
                if cur:
                    if csum.lib.tulips_csum_burst_prefers_cpu(len(cur), sum(cur)):
                        cpu += 1
                    else:
                        gpu += 1
                used, cur = 0, []
            if ln is not None:
                cur.append(int(ln))
                used = (used + int(ln) + 15) // 16 * 16
        assert (int(st[4]), int(st[5])) == (gpu, cpu)
        # 12 jumbo frames (108 KB) stay on the CPU; 128-frame bursts flush
        # at 29 frames (261 KB, past the bytes limit) and go to the GPU
        assert (cpu, gpu) == ((10, 0) if burst == 12 else (1, 4))


@needs_harness
@pytest.mark.gpu
def test_cpu_crossover_off_keeps_every_burst_on_the_gpu():
    fx = fixture()
    fwd, st = run_cpu_below(fx, 1, 0, n=300)
    exp, _, _ = expected_forwarded(fx["expect"][:300], 3)
    np.testing.assert_array_equal(fwd, exp)
    assert int(st[4]) == 300 and int(st[5]) == 0


# ------------------------------------------------------------ transmit -----
def tx_run(arena, offs, lens, mss, tx_burst, tso, wire_mtu=1514):
    from tulips_amd import csum  # noqa: F401
    lib = C.CDLL(HARNESS)
    f = lib.gpucsum_tx_run
    f.restype = C.c_int64
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint16, C.c_uint32,
                  C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32,
                  C.c_void_p]
    n = len(offs)
    cap_n = int(sum(int(x) // max(mss, 1) + 2 for x in lens)) + 16
    out = np.zeros(cap_n * wire_mtu, dtype=np.uint8)
    olen = np.zeros(cap_n, dtype=np.uint16)
    st = np.zeros(5, dtype=np.uint64)
    arena = np.ascontiguousarray(arena)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    k = f(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, n, mss, tx_burst, tso,
          wire_mtu, out.ctypes.data, out.nbytes, olen.ctypes.data, cap_n, st.ctypes.data)
    assert k >= 0, f"gpucsum_tx_run rc={k}"
    olen = olen[:k]
    pos = np.concatenate([[0], np.cumsum(olen.astype(np.int64))])
    frames = [bytes(out[pos[i]:pos[i + 1]]) for i in range(k)]
    return frames, st


@needs_harness
@pytest.mark.gpu
@pytest.mark.parametrize("tx_burst", [1, 5, 64])
def test_tx_generates_checksums_before_the_wire(oracle, tx_burst):
    """Config::tx: the fixture's frames (checksum fields scrambled) committed
    through the decorator reach the wire exactly as the oracle's generation
    writes them (pinned to reference-generated bytes in test_frames.py), in
    commit order; the stack's buffers are reported sent and released."""
    from test_frames import scramble_fields
    fx = fixture()
    rng = np.random.default_rng(tx_burst)
    src = scramble_fields(fx, rng)
    n = 700
    offs, lens = fx["offsets"][:n], fx["lengths"][:n]
    keep = lens <= 1514                       # what fits the list device's buffers
    offs, lens = offs[keep], lens[keep]
    exp_arena, exp_flags = oracle.generate_frames(src, offs, lens)
    frames, st = tx_run(src, offs, lens, 0, tx_burst, 0)
    assert len(frames) == len(offs)
    for i, f in enumerate(frames):
        o, ln = int(offs[i]), int(lens[i])
        assert f == bytes(exp_arena[o:o + ln]), i
    assert int(st[0]) == len(offs) and int(st[1]) == len(offs)
    assert int(st[2]) == (len(offs) + tx_burst - 1) // tx_burst
    assert int(st[3]) == len(offs) and int(st[4]) == len(offs)


@needs_harness
@pytest.mark.gpu
@pytest.mark.parametrize("mss", [0, 536, 1460])
def test_tx_tso_segments_super_frames(oracle, mss):
    """Config::tso: super-frames up to 64 KB committed with the stack's MSS
    are cut on the GPU into wire frames that (1) equal the oracle's
    segmentation, (2) verify with the REFERENCE's own ipv4::checksum and
    tcpv4::Processor::checksum (oracle/_ref), and (3) reassemble to the
    super-frame's payload; one sent() per super-frame reaches the stack.
    mss 0 = the largest that fits the inner buffer, as the OFED device
    adjusts it (src/transport/ofed/Device.cpp:711-714)."""
    from oracle import Reference
    from test_segment import check_properties, pack, super_frame
    ref = Reference()
    rng = np.random.default_rng(mss + 1)
    pays = [0, 40, 1460, 1461, 3000, 9000, 20000, 65535 - 54 - 40]
    frames_in = [super_frame(oracle, rng, p, doff=[5, 8][i % 2]) for i, p in enumerate(pays)]
    arena, offs, lens = pack(frames_in, rng)
    wire, st = tx_run(arena, offs, lens, mss, 4, 65535)
    eff = []
    for f in frames_in:
        hl = 34 + 4 * (f[46] >> 4)
        lm = mss if mss and mss <= 1514 - hl else 1514 - hl
        eff.append(lm)
    # group the wire frames back per super-frame and check each
    at = 0
    for f, lm in zip(frames_in, eff):
        hl = 34 + 4 * (f[46] >> 4)
        total = f[16] << 8 | f[17]
        npay = total - 20 - (hl - 34)
        cnt = 1 if len(f) <= 1514 else max(1, -(-npay // lm))
        segs = wire[at:at + cnt]
        at += cnt
        if len(f) <= 1514:
            exp_arena, _ = oracle.generate_frames(np.frombuffer(f, np.uint8).copy(),
                                                  np.zeros(1, np.uint64),
                                                  np.array([len(f)], np.uint16))
            assert segs[0] == bytes(exp_arena)
        else:
            check_properties(oracle, f, segs, lm)
        for s in segs:
            ip = s[14:34]
            assert ref.ipv4_checksum(ip) == 0xFFFF
            src = int.from_bytes(s[26:30], "little")
            dst = int.from_bytes(s[30:34], "little")
            tl = (s[16] << 8 | s[17]) - 20
            assert ref.tcp_checksum(src, dst, s[34:34 + tl]) == 0xFFFF
    assert at == len(wire)
    assert int(st[0]) == len(frames_in) and int(st[1]) == len(wire)
    assert int(st[3]) == len(frames_in) and int(st[4]) == len(frames_in)
