"""Several GPUs in one process: tulips_csum_shard_plan and
the multi-device host context tulips_csum_mctx_* (tulips_amd/csrc/
csum_multi.hip). On the one-GPU test box every shard maps to device 0 —
independent contexts and pipelines on one card — which exercises the split,
the per-device workers and the in-order result assembly; the digests are the
reference's (tests/golden/digests.json: ZIPF, the M8x1500 shards)."""
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
    gold = golden()["M8x1500"]["shards"]
    nseg, seg = 1 << 20, 1500
    host = np.empty(2 * nseg * seg + 64, dtype=np.uint8)
    dev = torch.empty(nseg * seg + 64, dtype=torch.uint8, device="cuda:0")
    for s in range(2):
        csum.fill_splitmix(dev, nseg * seg, byte_off=s * nseg * seg)
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
