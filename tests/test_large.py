"""Arenas past 4 GiB: every offset-taking entry point with its segments,
frames and super-frames placed beyond 2^32 bytes of one 4.5 GiB device
allocation (an MI355X holds 288 GB; a receive ring mirrored in HBM can be
that large). Offsets are 64-bit throughout the C ABI (include/tulips_csum.h);
these tests pin it: fixed-stride, in-order arena, any-layout and counting
batches compared with the oracle on the segments at the start, across the
4 GiB line and at the end; frame validation (tests/golden/frames.npz flags,
computed by the reference's own checksums) and segmentation (vs the oracle)
on inputs that start past 4 GiB. Semantics: /root/reference/src/stack/
Utils.cpp:14-42, src/stack/tcpv4/Processor.cpp:337-357."""
import numpy as np
import pytest

from test_frames import frames_fixture
from test_segment import pack as seg_pack, super_frame

GIB = 1 << 30
SIZE = 4 * GIB + GIB // 2
LINE = 1 << 32
MODE_RAW, MODE_INET, MODE_TCP = 0, 1, 2


@pytest.fixture(scope="module")
def big():
    import torch
    import benchlib
    a = torch.empty(SIZE + 64, dtype=torch.uint8, device="cuda:0")
    benchlib.fill_splitmix(a, SIZE, seed=0x4C41524745)
    torch.cuda.synchronize()
    yield a
    del a
    torch.cuda.empty_cache()


def _samples(starts, lens, k=48):
    """Indices of the first k, the k around the 4 GiB line and the last k."""
    n = len(starts)
    ends = starts + lens
    mid = int(np.searchsorted(ends, LINE))
    idx = set(range(min(k, n))) | set(range(max(0, n - k), n))
    idx |= set(range(max(0, mid - k // 2), min(n, mid + k // 2)))
    return np.array(sorted(idx), dtype=np.int64), mid


def _oracle_of(oracle, a, starts, lens, idx, mode=MODE_RAW, src=None, dst=None):
    """The oracle's results for segments idx, their bytes copied to the host."""
    parts, offs, pos = [], [], 0
    for i in idx:
        s, ln = int(starts[i]), int(lens[i])
        parts.append(a[s:s + ln].cpu().numpy())
        offs.append(pos)
        pos += ln
    buf = np.concatenate(parts + [np.zeros(64, np.uint8)])
    kw = {}
    if mode == MODE_TCP:
        kw = dict(src=src[idx], dst=dst[idx])
    return oracle.batch(buf, np.array(offs, np.uint64), lens[idx].astype(np.uint16),
                        mode=mode, nthreads=8, **kw)


@pytest.mark.gpu
def test_fixed_stride_past_4gib(big, oracle):
    import tulips_amd
    stride = length = 9000
    n = SIZE // stride
    assert (n - 1) * stride > LINE
    out = tulips_amd.batch_fixed(big, stride, length, n)
    starts = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    lens = np.full(n, length, np.uint16)
    idx, mid = _samples(starts, lens)
    assert int(starts[mid]) < LINE < int(starts[mid]) + length       # one straddles the line
    got = out.cpu().numpy().view(np.uint16)[idx]
    np.testing.assert_array_equal(got, _oracle_of(oracle, big, starts, lens, idx))


@pytest.mark.gpu
def test_arena_any_layout_and_verify_past_4gib(big, oracle):
    import torch
    import tulips_amd
    rng = np.random.default_rng(4242)
    n = 142_000
    lens = rng.integers(1, 65536, n).astype(np.uint16)
    lens[rng.integers(0, n, 2000)] = 0                               # empty segments too
    gaps = rng.integers(0, 16, n).astype(np.uint64)
    starts = np.zeros(n, np.uint64)
    np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1], out=starts[1:])
    starts += np.uint64(5)                                           # odd base alignment
    arena_bytes = int(starts[-1]) + int(lens[-1])
    assert LINE < arena_bytes <= SIZE
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    d_offs = torch.from_numpy(starts.view(np.int64)).to("cuda:0")
    d_lens = torch.from_numpy(lens.view(np.int16)).to("cuda:0")
    d_src = torch.from_numpy(src.view(np.int32)).to("cuda:0")
    d_dst = torch.from_numpy(dst.view(np.int32)).to("cuda:0")
    idx, mid = _samples(starts, lens)
    # in-order arena (span kernel), RAW and TCP
    raw = tulips_amd.batch_arena(big, d_offs, d_lens, arena_bytes=arena_bytes)
    tcp = tulips_amd.batch_arena(big, d_offs, d_lens, arena_bytes=arena_bytes, src=d_src,
                                 dst=d_dst, mode=MODE_TCP)
    raw_h = raw.cpu().numpy().view(np.uint16)
    tcp_h = tcp.cpu().numpy().view(np.uint16)
    np.testing.assert_array_equal(raw_h[idx], _oracle_of(oracle, big, starts, lens, idx))
    np.testing.assert_array_equal(
        tcp_h[idx], _oracle_of(oracle, big, starts, lens, idx, MODE_TCP, src, dst))
    # any layout (offsets only, packed kernel): the same results everywhere
    anyl = tulips_amd.batch(big, d_offs, d_lens)
    np.testing.assert_array_equal(anyl.cpu().numpy().view(np.uint16), raw_h)
    # counting over the whole arena: the results that are not 0xffff
    bad = tulips_amd.verify_arena(big, d_offs, d_lens, arena_bytes=arena_bytes, src=d_src,
                                  dst=d_dst, mode=MODE_TCP)
    torch.cuda.synchronize()
    assert int(bad.cpu().numpy().view(np.uint32)[0]) == int(np.count_nonzero(tcp_h != 0xFFFF))


@pytest.mark.gpu
def test_frames_and_segmentation_past_4gib(big, oracle):
    import torch
    from tulips_amd import csum
    # the golden frames, copied in past the 4 GiB line
    fx = frames_fixture()
    at = LINE + 4099
    fa = fx["arena"]
    big[at:at + len(fa)].copy_(torch.from_numpy(fa))
    offs = torch.from_numpy((fx["offsets"] + np.uint64(at)).view(np.int64)).to("cuda:0")
    lens = torch.from_numpy(fx["lengths"].view(np.int16)).to("cuda:0")
    flags = csum.validate_frames(big, offs, lens)
    np.testing.assert_array_equal(flags.cpu().numpy(), fx["expect"])
    # super-frames past the line, segmented against the oracle
    rng = np.random.default_rng(11)
    frames = [super_frame(oracle, rng, int(p)) for p in rng.integers(1, 60000, 24)]
    sa, so, sl = seg_pack(frames, rng)
    at2 = LINE + GIB // 4 + 3
    big[at2:at2 + len(sa)].copy_(torch.from_numpy(sa.copy()))   # (a writable copy)
    mss, stride = 1460, 2048
    efirst, eout, elens = oracle.segment_frames(sa, so, sl, mss, stride)
    d_so = torch.from_numpy((so + np.uint64(at2)).view(np.int64)).to("cuda:0")
    d_sl = torch.from_numpy(sl.view(np.int16)).to("cuda:0")
    out, olens, first = csum.segment_frames(big, d_so, d_sl, mss, stride=stride)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(first.cpu().numpy().view(np.uint32), efirst)
    got_l = olens.cpu().numpy().view(np.uint16)[:len(elens)]
    np.testing.assert_array_equal(got_l, elens)
    got = out.cpu().numpy()[:len(eout)].reshape(-1, stride)
    want = eout.reshape(-1, stride)
    for j in range(len(elens)):
        assert np.array_equal(got[j, :elens[j]], want[j, :elens[j]]), j


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_segmentation_at_max_frames(oracle):
    """tulips_csum_segment_frames at its limit, n = 2^24 frames
    (include/tulips_csum.h): small TCP frames of 0-10 payload bytes in 64 B
    slots, MSS 4, so frames become 1-3 segments and the count scan runs over
    all 65,536 of its blocks; first[], every segment length and every segment
    byte against the oracle (orc_segment_frames)."""
    import torch
    from tulips_amd import csum
    n = 1 << 24
    slot, mss = 64, 4
    rng = np.random.default_rng(24)
    pay = rng.integers(0, 11, n).astype(np.uint16)
    f = rng.integers(0, 256, (n, slot), dtype=np.uint8)
    f[:, 12], f[:, 13], f[:, 14], f[:, 15] = 0x08, 0x00, 0x45, 0x00
    tot = 40 + pay
    f[:, 16], f[:, 17] = (tot >> 8).astype(np.uint8), (tot & 0xFF).astype(np.uint8)
    f[:, 20], f[:, 21], f[:, 22], f[:, 23] = 0x40, 0x00, 64, 6
    f[:, 46] = 0x50
    arena = f.reshape(-1)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(slot)
    lens = (54 + pay).astype(np.uint16)
    efirst, eout, elens = oracle.segment_frames(arena, offs, lens, mss, slot)
    total = int(efirst[-1])
    assert total > n
    d_ar = torch.from_numpy(arena).to("cuda:0")
    d_offs = torch.from_numpy(offs.view(np.int64)).to("cuda:0")
    d_lens = torch.from_numpy(lens.view(np.int16)).to("cuda:0")
    out, olens, first = csum.segment_frames(d_ar, d_offs, d_lens, mss, stride=slot)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(first.cpu().numpy().view(np.uint32), efirst)
    np.testing.assert_array_equal(olens.cpu().numpy().view(np.uint16)[:total], elens)
    got = out.cpu().numpy()[:total * slot].reshape(total, slot)
    want = eout.reshape(total, slot)
    keep = np.arange(slot)[None, :] < elens.astype(np.int64)[:, None]
    assert np.array_equal(got[keep], want[keep])
