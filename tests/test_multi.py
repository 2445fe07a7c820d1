"""Several GPUs in one process: tulips_csum_shard_plan and
the multi-device host context tulips_csum_mctx_* (tulips_amd/csrc/
csum_multi.hip). On the one-GPU test box every shard maps to device 0 —
independent contexts and pipelines on one card — which exercises the split,
the per-device workers and the in-order result assembly; the digests are the
reference's (tests/golden/digests.json: ZIPF, the M8x1500 shards)."""
import ctypes as C
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def golden():
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        return json.load(f)["batches"]


def check_plan(lens, k, b):
    n = len(lens)
    assert b[0] == 0 and b[-1] == n and len(b) == k + 1
    assert np.all(np.diff(b.astype(np.int64)) >= 0)
    pre = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    total = int(pre[-1])
    for j in range(1, k):
        # shard j starts at the first segment whose prefix reaches j/k of the bytes
        t = -(-total * j // k)
        i = int(b[j])
        assert pre[i] >= t or i == n
        assert i == 0 or pre[i - 1] < t


@pytest.mark.parametrize("k", [1, 2, 3, 8, 64])
def test_shard_plan_is_byte_balanced(oracle, k):
    from tulips_amd import csum
    lens = oracle.zipf_lengths(65536)
    b = csum.shard_plan(lens, k)
    check_plan(lens, k, b)
    bytes_ = np.add.reduceat(lens.astype(np.int64), b[:-1].astype(np.int64)) \
        if k > 1 else np.array([lens.astype(np.int64).sum()])
    # every shard within one maximal segment of the mean
    assert np.all(np.abs(bytes_ - lens.astype(np.int64).sum() / k) <= int(lens.max()))
    # a count split would be far off on Zipf lengths (the point of the plan)
    if k == 8:
        cnt = np.add.reduceat(lens.astype(np.int64), np.arange(0, 65536, 8192))
        assert cnt.max() - cnt.min() > 10 * (bytes_.max() - bytes_.min())


def test_shard_plan_edges():
    from tulips_amd import csum
    check_plan(np.zeros(0, np.uint16), 3, csum.shard_plan(np.zeros(0, np.uint16), 3))
    z = np.zeros(10, np.uint16)                     # all-empty segments
    check_plan(z, 4, csum.shard_plan(z, 4))
    one = np.array([65535], np.uint16)
    b = csum.shard_plan(one, 4)
    check_plan(one, 4, b)
    assert csum.lib.tulips_csum_shard_plan(None, 0, 0, None) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("ndev", [1, 4])
def test_mctx_zipf_digest(oracle, ndev):
    from tulips_amd import csum
    g = golden()["ZIPF"]
    lens = oracle.zipf_lengths(65536)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.astype(np.int64).sum())
    arena = oracle.splitmix_bytes(total + 64)
    with csum.MultiContext([0] * ndev, chunk_bytes=1 << 22) as m:
        out = m.batch(arena, offs, lens)
        b = m.bounds()
    check_plan(lens, ndev, b)
    assert f"{oracle.fnv1a_u16(out):016x}" == g["fnv1a64"]


@pytest.mark.gpu
def test_mctx_m8_two_shards_match_reference_digests():
    """M8x1500 shards 0 and 1 (2 x 1,048,576 x 1500 B = 3.1 GB of host
    memory) through a two-device context: the byte-balanced split of equal
    segments is the shard boundary itself, and each half's digest is the
    reference's shard digest."""
    import torch
    from tulips_amd import csum
    import benchlib
    gold = golden()["M8x1500"]["shards"]
    nseg, seg = 1 << 20, 1500
    host = np.empty(2 * nseg * seg + 64, dtype=np.uint8)
    dev = torch.empty(nseg * seg + 64, dtype=torch.uint8, device="cuda:0")
    for s in range(2):
        benchlib.fill_splitmix(dev, nseg * seg, byte_off=s * nseg * seg)
        host[s * nseg * seg:(s + 1) * nseg * seg] = dev[:nseg * seg].cpu().numpy()
    del dev
    offs = np.arange(2 * nseg, dtype=np.uint64) * np.uint64(seg)
    lens = np.full(2 * nseg, seg, np.uint16)
    with csum.MultiContext([0, 0]) as m:
        out = m.batch(host, offs, lens)
        b = m.bounds()
    assert list(b) == [0, nseg, 2 * nseg]
    from oracle import Oracle
    o = Oracle()
    for s in range(2):
        assert f"{o.fnv1a_u16(out[s * nseg:(s + 1) * nseg]):016x}" == gold[s]["fnv1a64"]


@pytest.mark.gpu
def test_mctx_validate_frames_and_counters(oracle):
    from tulips_amd import csum
    from test_frames import counters_of, frames_fixture, mutate
    fx = frames_fixture()
    arena = mutate(fx, np.random.default_rng(3), 900)
    exp = oracle.validate_frames(arena, fx["offsets"], fx["lengths"])
    with csum.MultiContext([0, 0, 0], chunk_bytes=1 << 17) as m:
        fl, cnt = m.validate_frames(arena, fx["offsets"], fx["lengths"], with_counters=True)
    np.testing.assert_array_equal(fl, exp)
    np.testing.assert_array_equal(cnt, counters_of(exp))


# -- device-resident batches over several devices (tulips_csum_mctx_batch_*_device)
def test_mctx_device_arguments_without_gpu():
    from tulips_amd import csum
    lib = csum.lib
    F = 16
    assert lib.tulips_csum_mctx_batch_fixed_device(None, F, 1500, 1500, None, None, None, F,
                                                   4, 0, None) == 1
    assert lib.tulips_csum_mctx_batch_arena_device(None, F, 16, F, F, None, None, None, F,
                                                   4, 0, None) == 1
    # n == 0 with a context is a no-op; without one it is an argument error
    assert lib.tulips_csum_mctx_batch_fixed_device(None, None, 0, 0, None, None, None, None,
                                                   0, 0, None) == 1


def _dev(a):
    import torch
    return torch.from_numpy(np.array(a, copy=True, order="C")).to("cuda:0")


@pytest.mark.gpu
@pytest.mark.parametrize("ndev", [1, 2, 4])
def test_mctx_device_arena_zipf_digests(oracle, ndev):
    """The golden ZIPF arena resident on GPU 0, spread over `ndev` logical
    devices (all GPU 0 on the test box: entry 0 works in place, the others
    pull their pieces with peer copies into their own buffers and send the
    results home): ZIPF and ZIPF-tcp digests, byte-balanced bounds."""
    import torch
    from tulips_amd import csum
    import benchlib
    from oracle import ip4
    g = golden()
    lens = oracle.zipf_lengths(65536)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.astype(np.int64).sum())
    arena = torch.empty(total + 64, dtype=torch.uint8, device="cuda:0")
    benchlib.fill_splitmix(arena, total)
    do, dl = _dev(offs.view(np.int64)), _dev(lens)
    src = _dev(np.full(65536, ip4(10, 1, 0, 1), np.uint32))
    dst = _dev(np.full(65536, ip4(10, 1, 0, 2), np.uint32))
    with csum.MultiContext([0] * ndev) as m:
        for rep in range(2):                       # buffers reused by a second call
            out = m.batch_arena_device(arena, do, dl, arena_bytes=total)
            torch.cuda.synchronize()
            assert f"{oracle.fnv1a_u16(out.cpu().numpy().view(np.uint16)):016x}" == \
                g["ZIPF"]["fnv1a64"], rep
        b = m.bounds()
        out = m.batch_arena_device(arena, do, dl, arena_bytes=total, src=src, dst=dst,
                                   mode=2)
        torch.cuda.synchronize()
        assert f"{oracle.fnv1a_u16(out.cpu().numpy().view(np.uint16)):016x}" == \
            g["ZIPF-tcp"]["fnv1a64"]
    assert b[0] == 0 and b[-1] == 65536 and np.all(np.diff(b.astype(np.int64)) >= 0)
    share = np.add.reduceat(lens.astype(np.int64), b[:-1].astype(np.int64)) if ndev > 1 else \
        np.array([total])
    assert np.all(np.abs(share - total / ndev) <= 2 * int(lens.max())), share


@pytest.mark.gpu
@pytest.mark.parametrize("ndev", [3, 5])
def test_mctx_device_arena_random_layouts(oracle, ndev):
    """In-order arena with gaps, empty / tiny / 65,535-byte segments, an odd
    base, seeds; and a later call on the same context with a smaller batch
    (stale buffers must not leak)."""
    import torch
    from tulips_amd import csum
    rng = np.random.default_rng(8800 + ndev)
    for n in (150000, 9000):
        lens = rng.integers(0, 3000, n).astype(np.uint16)
        lens[rng.random(n) < 0.1] = 0
        lens[rng.integers(0, n, 30)] = 65535
        gaps = np.where(rng.random(n) < 0.3, rng.integers(0, 300, n), 0).astype(np.uint64)
        ends = np.cumsum(lens.astype(np.uint64) + gaps)
        offs = (ends - lens.astype(np.uint64)).astype(np.uint64)
        total = int(ends[-1])
        buf = rng.integers(0, 256, total + 67, dtype=np.uint8)
        seeds = rng.integers(0, 65536, n, dtype=np.uint16)
        exp = oracle.batch(buf[3:3 + total], offs, lens, seeds=seeds, mode=1, nthreads=8)
        dbuf = _dev(buf)
        with csum.MultiContext([0] * ndev) as m:
            out = m.batch_arena_device(dbuf[3:], _dev(offs.view(np.int64)), _dev(lens),
                                       arena_bytes=total, seeds=_dev(seeds), mode=1)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), exp)


@pytest.mark.gpu
def test_mctx_device_fixed_m8_from_gpu0(oracle):
    """configs[4]: the whole M8x1500 batch (8,388,608 x 1500 B = 12.6 GB)
    resident on GPU 0, spread over 8 logical devices: every shard digest and
    the full-batch digest equal the reference's, the bounds are the shard
    boundaries. Then F1500-tcp through 3 logical devices."""
    import torch
    from tulips_amd import csum
    import benchlib
    from oracle import ip4
    g = golden()
    gold = g["M8x1500"]
    n, seg = 8 << 20, 1500
    arena = torch.empty(n * seg + 64, dtype=torch.uint8, device="cuda:0")
    benchlib.fill_splitmix(arena, n * seg)
    with csum.MultiContext([0] * 8) as m:
        out = m.batch_fixed_device(arena, seg, seg, n)
        torch.cuda.synchronize()
        b = m.bounds()
    o = out.cpu().numpy().view(np.uint16)
    assert list(b) == [k * (n // 8) for k in range(9)]
    for k in range(8):
        assert f"{oracle.fnv1a_u16(o[k * (n // 8):(k + 1) * (n // 8)]):016x}" == \
            gold["shards"][k]["fnv1a64"], k
    assert f"{oracle.fnv1a_u16(o):016x}" == gold["fnv1a64"]
    del arena, out
    bt = g["F1500-tcp"]
    nt = bt["n"]
    arena = torch.empty(nt * 1500 + 64, dtype=torch.uint8, device="cuda:0")
    benchlib.fill_splitmix(arena, nt * 1500)
    src = _dev(np.full(nt, ip4(10, 1, 0, 1), np.uint32))
    dst = _dev(np.full(nt, ip4(10, 1, 0, 2), np.uint32))
    with csum.MultiContext([0] * 3) as m:
        out = m.batch_fixed_device(arena, 1500, 1500, nt, src=src, dst=dst, mode=2)
        torch.cuda.synchronize()
    assert f"{oracle.fnv1a_u16(out.cpu().numpy().view(np.uint16)):016x}" == bt["fnv1a64"]


@pytest.mark.gpu
def test_mctx_device_staged_copies(oracle):
    """The staged form (no peer access between two devices, here forced with
    tulips_csum_mctx_set_peer_mode): pieces go source HBM -> page-locked
    bounce -> the device's HBM and results back the same way. F1500, F1500-tcp
    and ZIPF digests over 3 logical devices; then the same context switched
    back to peer copies (slots reused both ways)."""
    import torch
    from tulips_amd import csum
    import benchlib
    from oracle import ip4
    g = golden()
    n = 65536
    arena = torch.empty(n * 1500 + 64, dtype=torch.uint8, device="cuda:0")
    benchlib.fill_splitmix(arena, n * 1500)
    src = _dev(np.full(n, ip4(10, 1, 0, 1), np.uint32))
    dst = _dev(np.full(n, ip4(10, 1, 0, 2), np.uint32))
    lens = oracle.zipf_lengths(n)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    ztot = int(lens.astype(np.int64).sum())
    za = torch.empty(ztot + 64, dtype=torch.uint8, device="cuda:0")
    benchlib.fill_splitmix(za, ztot)
    do, dl = _dev(offs.view(np.int64)), _dev(lens)

    def dig(t):
        return f"{oracle.fnv1a_u16(t.cpu().numpy().view(np.uint16)):016x}"
    with csum.MultiContext([0, 0, 0], chunk_bytes=1 << 20) as m:
        for staged in (True, False, True):
            m.set_peer_mode(staged)
            out = m.batch_fixed_device(arena, 1500, 1500, n)
            torch.cuda.synchronize()
            assert dig(out) == g["F1500"]["fnv1a64"], staged
            out = m.batch_fixed_device(arena, 1500, 1500, n, src=src, dst=dst, mode=2)
            torch.cuda.synchronize()
            assert dig(out) == g["F1500-tcp"]["fnv1a64"], staged
            out = m.batch_arena_device(za, do, dl, arena_bytes=ztot)
            torch.cuda.synchronize()
            assert dig(out) == g["ZIPF"]["fnv1a64"], staged
        assert list(m.bounds()) != [0, 0, 0, 0]


@pytest.mark.gpu
def test_mctx_device_every_visible_gpu(oracle):
    """With more than one GPU visible, the device-resident path over real
    peers (xGMI peer DMA where hipDeviceCanAccessPeer allows it, staged
    otherwise): F1500 digest from GPU 0 over every device, both forms."""
    import torch
    from tulips_amd import csum
    import benchlib
    nd = torch.cuda.device_count()
    if nd < 2:
        pytest.skip("one GPU visible")
    g = golden()
    n = 65536
    arena = torch.empty(n * 1500 + 64, dtype=torch.uint8, device="cuda:0")
    benchlib.fill_splitmix(arena, n * 1500)
    with csum.MultiContext(list(range(nd))) as m:
        for staged in (False, True):
            m.set_peer_mode(staged)
            out = m.batch_fixed_device(arena, 1500, 1500, n)
            torch.cuda.synchronize()
            assert f"{oracle.fnv1a_u16(out.cpu().numpy().view(np.uint16)):016x}" == \
                g["F1500"]["fnv1a64"], staged


def test_mctx_peer_mode_arguments_without_gpu():
    from tulips_amd import csum
    f = csum.lib.tulips_csum_mctx_set_peer_mode
    assert f(None, 0) == 1


# -- flow-affine validation (tulips_csum_mctx_validate_frames_rss_host) -------
def _rss_frames(oracle, rng, fx_rss, reps=2):
    """One well-formed TCP frame per rss.npz tuple (addresses and ports set
    to the fixture's, checksums generated by the oracle), `reps` frames per
    flow interleaved with each other, plus non-TCP frames."""
    from test_frames import make_frame
    frames, flow = [], []
    ntup = len(fx_rss["saddr"])
    order = np.concatenate([rng.permutation(ntup) for _ in range(reps)])
    for j in order:
        f = bytearray(make_frame(oracle, rng, int(rng.integers(0, 600))))
        f[26:30] = int(fx_rss["saddr"][j]).to_bytes(4, "little")
        f[30:34] = int(fx_rss["daddr"][j]).to_bytes(4, "little")
        f[34:36] = int(fx_rss["sport"][j]).to_bytes(2, "big")
        f[36:38] = int(fx_rss["dport"][j]).to_bytes(2, "big")
        frames.append(bytes(f))
        flow.append(int(j))
    for _ in range(50):                                    # ARP-like, not IPv4
        frames.append(b"\xff" * 12 + b"\x08\x06" + bytes(46))
        flow.append(-1)
    from test_frames import pack
    arena, offs, lens = pack(frames, rng)
    arena = arena.copy()
    gen, _ = oracle.generate_frames(arena, offs, lens)     # fresh checksums
    return gen, offs, lens, np.array(flow)


@pytest.mark.gpu
@pytest.mark.parametrize("key_i,init,ndev", [(0, 0, 4), (9, 0xFFFFFFFF, 3), (7, 0, 2)])
def test_mctx_rss_flow_affine_matches_reference_hashes(oracle, key_i, init, ndev):
    """Each frame lands on table[reference hash % len] (the reference's own
    toeplitz over the same tuples, tests/golden/rss.npz), every frame of a
    flow on the same device, flags identical to one device's, counters
    summed; non-TCP frames go to table[0]."""
    from test_rss import rss_fixture
    from tulips_amd import csum
    fx = rss_fixture()
    key = fx[f"key_{key_i}"].tobytes()
    exp_hash = fx[f"expect_{key_i}_{'init0' if init == 0 else 'initff'}"]
    rng = np.random.default_rng(key_i * 7 + ndev)
    arena, offs, lens, flow = _rss_frames(oracle, rng, fx)
    table = (np.arange(128) * 7 % ndev).astype(np.uint16)
    table[0] = ndev - 1
    exp_flags = oracle.validate_frames(arena, offs, lens)
    with csum.MultiContext([0] * ndev, chunk_bytes=1 << 20) as m:
        flags, dev, cnt = m.validate_frames_rss(arena, offs, lens, key, table, init=init,
                                                with_counters=True)
        b = m.bounds()
    np.testing.assert_array_equal(flags, exp_flags)
    from test_frames import counters_of
    np.testing.assert_array_equal(cnt, counters_of(exp_flags))
    tcp = flow >= 0
    want = table[exp_hash[flow[tcp]].astype(np.int64) % len(table)]
    np.testing.assert_array_equal(dev[tcp], want)
    assert np.all(dev[~tcp] == table[0])
    for j in np.unique(flow[tcp])[:200]:
        assert len(set(dev[flow == j].tolist())) == 1
    assert list(np.diff(b)) == [int((dev == k).sum()) for k in range(ndev)]


def test_mctx_rss_arguments_without_gpu():
    from tulips_amd import csum
    f = csum.lib.tulips_csum_mctx_validate_frames_rss_host
    key = (C.c_uint8 * 40)()
    assert f(None, 1, 1, 1, 1, key, 40, 0, 1, 1, 1, None, None) == 1


@pytest.mark.gpu
def test_mctx_rss_fragments_go_to_slot0(oracle):
    """IPv4 fragments of a TCP flow (MF set, or a fragment offset) carry no
    ports a NIC would hash: they go to table[0] like other frames without a
    4-tuple, never to a device picked by payload bytes; the
    flow's unfragmented frames stay on one device."""
    from test_frames import make_frame, pack
    from tulips_amd import csum
    rng = np.random.default_rng(31)
    key = bytes(range(7, 47))
    frames, kind = [], []
    for k in range(400):
        f = bytearray(make_frame(oracle, rng, int(rng.integers(20, 900))))
        f[26:38] = bytes([10, 0, 0, 1, 10, 0, 0, 2, 0x1f, 0x90, 0x22, 0xb8])
        r = k % 4
        if r == 1:
            f[20] = (f[20] & 0xC0) | 0x20                 # MF: first fragment
        elif r == 2:
            f[20], f[21] = 0x00, 0xb9                     # non-first fragment
            f[34:38] = rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
        frames.append(bytes(f))
        kind.append(r)
    arena, offs, lens = pack(frames, rng)
    arena, _ = oracle.generate_frames(arena.copy(), offs, lens)
    kind = np.array(kind)
    table = np.array([3, 0, 1, 2] * 32, dtype=np.uint16)
    with csum.MultiContext([0] * 4, chunk_bytes=1 << 20) as m:
        flags, dev = m.validate_frames_rss(arena, offs, lens, key, table)
    np.testing.assert_array_equal(flags, oracle.validate_frames(arena, offs, lens))
    frag = (kind == 1) | (kind == 2)
    assert np.all(dev[frag] == table[0])
    whole = dev[~frag]
    assert len(set(whole.tolist())) == 1
    h = csum.toeplitz(int.from_bytes(bytes([10, 0, 0, 1]), "little"),
                      int.from_bytes(bytes([10, 0, 0, 2]), "little"), 0x1f90, 0x22b8, key)
    assert whole[0] == table[h % len(table)]


@pytest.mark.gpu
@pytest.mark.parametrize("key_i,init,ndev,lead", [(0, 0, 4, 0), (9, 0xFFFFFFFF, 3, 5),
                                                  (7, 0, 2, 3), (3, 7, 5, 1)])
def test_mctx_rss_device_matches_host_and_reference(oracle, key_i, init, ndev, lead):
    """tulips_csum_mctx_validate_frames_rss_device: frames resident on GPU 0
    (odd arena bases), hashed and ordered on the device, each device's run
    pulled and validated there: device_of equals table[reference hash %
    len] (tests/golden/rss.npz), equals the host form's, flags equal one
    device's, counters equal the flags', bounds count frames per device."""
    import torch
    from test_frames import counters_of
    from test_rss import rss_fixture
    from tulips_amd import csum
    fx = rss_fixture()
    key = fx[f"key_{key_i}"].tobytes()
    exp_hash = fx[f"expect_{key_i}_{'init0' if init == 0 else 'initff'}"] if init in (
        0, 0xFFFFFFFF) else None
    rng = np.random.default_rng(key_i * 11 + ndev)
    arena, offs, lens, flow = _rss_frames(oracle, rng, fx)
    table = (np.arange(128) * 5 % ndev).astype(np.uint16)
    table[0] = ndev - 1
    exp_flags = oracle.validate_frames(arena, offs, lens)
    buf = torch.zeros(len(arena) + lead, dtype=torch.uint8, device="cuda:0")
    buf[lead:] = torch.from_numpy(arena).to("cuda:0")
    cnt = torch.full((4,), -1, dtype=torch.int32, device="cuda:0")
    with csum.MultiContext([0] * ndev, chunk_bytes=1 << 20) as m:
        hflags, hdev = m.validate_frames_rss(arena, offs, lens, key, table, init=init)
        for rep in range(2):
            fl, dv = m.validate_frames_rss_device(
                buf[lead:], _dev(offs.view(np.int64)), _dev(lens.view(np.int16)), key, table,
                init=init, counters=cnt)
            torch.cuda.synchronize()
            dv = dv.cpu().numpy().view(np.uint16)
            np.testing.assert_array_equal(fl.cpu().numpy(), exp_flags)
            np.testing.assert_array_equal(dv, hdev)
            np.testing.assert_array_equal(cnt.cpu().numpy().view(np.uint32),
                                          counters_of(exp_flags))
            b = m.bounds()
            assert list(np.diff(b.astype(np.int64))) == [int((dv == k).sum())
                                                         for k in range(ndev)]
    np.testing.assert_array_equal(hflags, exp_flags)
    if exp_hash is not None:
        tcp = flow >= 0
        np.testing.assert_array_equal(dv[tcp],
                                      table[exp_hash[flow[tcp]].astype(np.int64) % len(table)])


@pytest.mark.gpu
@pytest.mark.parametrize("ndev", [2, 5])
def test_mctx_rss_device_staged_matches_peer(oracle, ndev):
    """with staging forced (tulips_csum_mctx_set_peer_mode),
    each device's packed run, offsets and lengths travel through the
    page-locked bounce and its flags come home the same way: flags, device_of
    and counters equal the peer-DMA form's and the oracle's."""
    import torch
    from test_frames import counters_of
    from test_rss import rss_fixture
    from tulips_amd import csum
    fx = rss_fixture()
    key = fx["key_3"].tobytes()
    rng = np.random.default_rng(300 + ndev)
    arena, offs, lens, _ = _rss_frames(oracle, rng, fx)
    table = (np.arange(128) * 7 % ndev).astype(np.uint16)
    exp = oracle.validate_frames(arena, offs, lens)
    a, o, ln = _dev(arena), _dev(offs.view(np.int64)), _dev(lens.view(np.int16))
    got = {}
    for staged in (False, True):
        with csum.MultiContext([0] * ndev, chunk_bytes=1 << 20) as m:
            m.set_peer_mode(staged)
            for rep in range(2):
                cnt = torch.full((4,), -1, dtype=torch.int32, device="cuda:0")
                fl, dv = m.validate_frames_rss_device(a, o, ln, key, table, counters=cnt)
                torch.cuda.synchronize()
                np.testing.assert_array_equal(fl.cpu().numpy(), exp)
                np.testing.assert_array_equal(cnt.cpu().numpy().view(np.uint32),
                                              counters_of(exp))
            got[staged] = (dv.cpu().numpy(), m.bounds())
    np.testing.assert_array_equal(got[True][0], got[False][0])
    np.testing.assert_array_equal(got[True][1], got[False][1])


@pytest.mark.gpu
def test_mctx_rss_device_alternating_streams(oracle):
    """Calls of one context alternated between two streams with no host
    synchronisation in between: each call overwrites the
    router's workspace (perm, rflags) that the previous call's last kernel,
    on the other stream, may still be reading; the context orders them
    (RouteWs::done), so every call's flags and counters equal the oracle's."""
    import torch
    from test_frames import counters_of
    from test_rss import rss_fixture
    from tulips_amd import csum
    fx = rss_fixture()
    key = fx["key_0"].tobytes()
    batches = []
    for seed, nf in ((71, None), (72, None)):
        rng = np.random.default_rng(seed)
        arena, offs, lens, _ = _rss_frames(oracle, rng, fx)
        if seed == 72:     # a different batch: fewer frames, different routing
            keep = len(offs) // 3
            offs, lens = offs[:keep], lens[:keep]
        batches.append((_dev(arena), _dev(offs.view(np.int64)), _dev(lens.view(np.int16)),
                        oracle.validate_frames(arena, offs, lens)))
    table = (np.arange(128) * 3 % 4).astype(np.uint16)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    with csum.MultiContext([0] * 4, chunk_bytes=1 << 20) as m:
        out = []
        for rep in range(6):
            a, o, ln, exp = batches[rep % 2]
            cnt = torch.full((4,), -1, dtype=torch.int32, device="cuda:0")
            fl, _ = m.validate_frames_rss_device(a, o, ln, key, table, counters=cnt,
                                                 stream=streams[rep % 2])
            out.append((fl, cnt, exp))
        torch.cuda.synchronize()
    for fl, cnt, exp in out:
        np.testing.assert_array_equal(fl.cpu().numpy(), exp)
        np.testing.assert_array_equal(cnt.cpu().numpy().view(np.uint32), counters_of(exp))


@pytest.mark.gpu
def test_mctx_rss_device_fixture_mutations_and_scale(oracle):
    """The reference-flagged frames.npz (mutated: bad checksums, fragments,
    runts, truncation, zero-length frames) routed over 3 devices, and a
    200,000-frame batch (several scan chunks of block histograms, frames up
    to 9 KB) over 8: flags equal the oracle's in arrival order."""
    import torch
    from test_frames import frames_fixture, make_frame, mutate, pack
    from tulips_amd import csum
    fx = frames_fixture()
    rng = np.random.default_rng(606)
    arena = mutate(fx, rng, 1500)
    exp = oracle.validate_frames(arena, fx["offsets"], fx["lengths"])
    key = bytes(range(40))
    with csum.MultiContext([0, 0, 0]) as m:
        fl, _ = m.validate_frames_rss_device(_dev(arena), _dev(fx["offsets"].view(np.int64)),
                                             _dev(fx["lengths"].view(np.int16)), key,
                                             [0, 1, 2, 2, 1])
        torch.cuda.synchronize()
        np.testing.assert_array_equal(fl.cpu().numpy(), exp)
    base = [make_frame(oracle, rng, int(p)) for p in rng.integers(0, 9000, 64)]
    idx = rng.integers(0, 64, 200000)
    frames = [base[i] for i in idx]
    arena, offs, lens = pack(frames, rng, gap=4)
    exp = oracle.validate_frames(arena, offs, lens)
    with csum.MultiContext(list(range(8)) if torch.cuda.device_count() >= 8 else [0] * 8) as m:
        fl, dv = m.validate_frames_rss_device(_dev(arena), _dev(offs.view(np.int64)),
                                              _dev(lens.view(np.int16)), key,
                                              np.arange(8, dtype=np.uint16))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(fl.cpu().numpy(), exp)
        assert len(np.unique(dv.cpu().numpy())) > 1


def test_mctx_rss_device_arguments_without_gpu():
    from tulips_amd import csum
    f = csum.lib.tulips_csum_mctx_validate_frames_rss_device
    key = (C.c_uint8 * 40)()
    tab = (C.c_uint16 * 4)()
    assert f(None, 1, 1, 1, 1, key, 40, 0, tab, 4, 1, None, None, None) == 1


# -- real peers: every cross-device entry across distinct GPUs -----------------
#  The tests above run the peer paths on logical device
# lists of GPU 0. These run them across every visible GPU, xGMI peer DMA where
# hipDeviceCanAccessPeer allows it and page-locked staging when forced, with
# the source on the first and on the last device; they skip on a one-GPU box.
# Reference analogue: NIC multi-queue spreading,
# /root/reference/src/transport/ena/RedirectionTable.cpp:74-98.
def _real_devices():
    import torch
    nd = torch.cuda.device_count()
    if nd < 2:
        pytest.skip("needs two or more GPUs (real peers)")
    return list(range(nd))


def _digest(oracle, t):
    import torch
    torch.cuda.synchronize()
    return f"{oracle.fnv1a_u16(t.cpu().numpy().view(np.uint16)):016x}"


@pytest.mark.gpu
@pytest.mark.parametrize("source", ["first", "last"])
def test_real_peers_arena_device_zipf(oracle, source):
    """tulips_csum_mctx_batch_arena_device across distinct GPUs: the device-side
    cut plan, each peer's pieces pulled with offs_bias, results sent home:
    ZIPF and ZIPF-tcp digests in peer and staged mode."""
    import torch
    from tulips_amd import csum
    import benchlib
    from oracle import ip4
    devs = _real_devices()
    src_dev = devs[0] if source == "first" else devs[-1]
    g = golden()
    lens = oracle.zipf_lengths(65536)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.astype(np.int64).sum())
    with torch.cuda.device(src_dev):
        dev = f"cuda:{src_dev}"
        arena = torch.empty(total + 64, dtype=torch.uint8, device=dev)
        benchlib.fill_splitmix(arena, total)
        do = torch.from_numpy(offs.view(np.int64).copy()).to(dev)
        dl = torch.from_numpy(lens.copy()).to(dev)
        src = torch.from_numpy(np.full(65536, ip4(10, 1, 0, 1), np.uint32)).to(dev)
        dst = torch.from_numpy(np.full(65536, ip4(10, 1, 0, 2), np.uint32)).to(dev)
        st = torch.cuda.current_stream(src_dev)
        with csum.MultiContext(devs) as m:
            for staged in (False, True):
                m.set_peer_mode(staged)
                out = m.batch_arena_device(arena, do, dl, arena_bytes=total, stream=st)
                assert _digest(oracle, out) == g["ZIPF"]["fnv1a64"], staged
                b = m.bounds()
                assert b[0] == 0 and b[-1] == 65536 and len(b) == len(devs) + 1
                out = m.batch_arena_device(arena, do, dl, arena_bytes=total, src=src, dst=dst,
                                           mode=2, stream=st)
                assert _digest(oracle, out) == g["ZIPF-tcp"]["fnv1a64"], staged


@pytest.mark.gpu
@pytest.mark.parametrize("source", ["first", "last"])
def test_real_peers_fixed_device(oracle, source):
    """tulips_csum_mctx_batch_fixed_device across distinct GPUs with the
    source on the first or the last device: F1500 and F1500-tcp digests in
    peer and staged mode."""
    import torch
    from tulips_amd import csum
    import benchlib
    from oracle import ip4
    devs = _real_devices()
    src_dev = devs[0] if source == "first" else devs[-1]
    g = golden()
    n = 65536
    with torch.cuda.device(src_dev):
        dev = f"cuda:{src_dev}"
        arena = torch.empty(n * 1500 + 64, dtype=torch.uint8, device=dev)
        benchlib.fill_splitmix(arena, n * 1500)
        src = torch.from_numpy(np.full(n, ip4(10, 1, 0, 1), np.uint32)).to(dev)
        dst = torch.from_numpy(np.full(n, ip4(10, 1, 0, 2), np.uint32)).to(dev)
        st = torch.cuda.current_stream(src_dev)
        with csum.MultiContext(devs) as m:
            for staged in (False, True):
                m.set_peer_mode(staged)
                out = m.batch_fixed_device(arena, 1500, 1500, n, stream=st)
                assert _digest(oracle, out) == g["F1500"]["fnv1a64"], staged
                out = m.batch_fixed_device(arena, 1500, 1500, n, src=src, dst=dst, mode=2,
                                           stream=st)
                assert _digest(oracle, out) == g["F1500-tcp"]["fnv1a64"], staged


@pytest.mark.gpu
@pytest.mark.parametrize("key_i,init", [(0, 0), (9, 0xFFFFFFFF)])
def test_real_peers_rss_device(oracle, key_i, init):
    """tulips_csum_mctx_validate_frames_rss_device across distinct GPUs: the
    source's hash and stable scatter, packed runs pulled by real peers, flags
    scattered home. device_of equals table[reference hash % len]
    (tests/golden/rss.npz) and the host form's; flags and counters equal the
    oracle's; the reference-flagged frames.npz (mutated) validates exactly;
    peer and staged mode agree."""
    import torch
    from test_frames import counters_of, frames_fixture, mutate
    from test_rss import rss_fixture
    from tulips_amd import csum
    devs = _real_devices()
    nd = len(devs)
    fx = rss_fixture()
    key = fx[f"key_{key_i}"].tobytes()
    exp_hash = fx[f"expect_{key_i}_{'init0' if init == 0 else 'initff'}"]
    rng = np.random.default_rng(4000 + key_i)
    arena, offs, lens, flow = _rss_frames(oracle, rng, fx)
    table = (np.arange(128) * 5 % nd).astype(np.uint16)
    table[0] = nd - 1
    exp_flags = oracle.validate_frames(arena, offs, lens)
    tcp = flow >= 0
    want_dev = table[exp_hash[flow[tcp]].astype(np.int64) % len(table)]
    a, o, ln = _dev(arena), _dev(offs.view(np.int64)), _dev(lens.view(np.int16))
    ffx = frames_fixture()
    fa = mutate(ffx, np.random.default_rng(77), 1200)
    fexp = oracle.validate_frames(fa, ffx["offsets"], ffx["lengths"])
    with csum.MultiContext(devs, chunk_bytes=1 << 20) as m:
        hflags, hdev = m.validate_frames_rss(arena, offs, lens, key, table, init=init)
        np.testing.assert_array_equal(hflags, exp_flags)
        np.testing.assert_array_equal(hdev[tcp], want_dev)
        got = {}
        for staged in (False, True):
            m.set_peer_mode(staged)
            cnt = torch.full((4,), -1, dtype=torch.int32, device="cuda:0")
            fl, dv = m.validate_frames_rss_device(a, o, ln, key, table, init=init, counters=cnt)
            torch.cuda.synchronize()
            dv = dv.cpu().numpy().view(np.uint16)
            np.testing.assert_array_equal(fl.cpu().numpy(), exp_flags, err_msg=str(staged))
            np.testing.assert_array_equal(dv, hdev)
            np.testing.assert_array_equal(dv[tcp], want_dev)
            np.testing.assert_array_equal(cnt.cpu().numpy().view(np.uint32),
                                          counters_of(exp_flags))
            b = m.bounds()
            assert list(np.diff(b.astype(np.int64))) == [int((dv == k).sum()) for k in range(nd)]
            got[staged] = dv
            fl, _ = m.validate_frames_rss_device(_dev(fa), _dev(ffx["offsets"].view(np.int64)),
                                                 _dev(ffx["lengths"].view(np.int16)), key, table,
                                                 init=init)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(fl.cpu().numpy(), fexp, err_msg=str(staged))
        np.testing.assert_array_equal(got[False], got[True])


@pytest.mark.gpu
def test_real_peers_host_entries(oracle):
    """tulips_csum_mctx_batch_host and tulips_csum_mctx_validate_frames_host
    over every visible GPU (each device its own pinned pipeline): ZIPF digest,
    byte-balanced bounds, frames.npz flags and counters; with the context in
    peer and in staged mode (the host entries must not depend on it)."""
    from test_frames import counters_of, frames_fixture, mutate
    from tulips_amd import csum
    devs = _real_devices()
    g = golden()["ZIPF"]
    lens = oracle.zipf_lengths(65536)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.astype(np.int64).sum())
    arena = oracle.splitmix_bytes(total + 64)
    fx = frames_fixture()
    fa = mutate(fx, np.random.default_rng(5), 900)
    fexp = oracle.validate_frames(fa, fx["offsets"], fx["lengths"])
    with csum.MultiContext(devs, chunk_bytes=1 << 22) as m:
        for staged in (False, True):
            m.set_peer_mode(staged)
            out = m.batch(arena, offs, lens)
            assert f"{oracle.fnv1a_u16(out):016x}" == g["fnv1a64"], staged
            check_plan(lens, len(devs), m.bounds())
            fl, cnt = m.validate_frames(fa, fx["offsets"], fx["lengths"], with_counters=True)
            np.testing.assert_array_equal(fl, fexp)
            np.testing.assert_array_equal(cnt, counters_of(fexp))
