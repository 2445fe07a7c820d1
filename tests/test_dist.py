"""N>1 path on CPU: two gloo ranks run the bench's shard harness
(tulips_amd/shard.py) with the oracle standing in for the GPU kernel.

Checks that rank r materialises exactly M8x1500 shard r (its digest equals
the reference's per-shard digest), and the control-plane reductions the
bench uses (max-over-ranks time, parity vote, digest gather).
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from tulips_amd.shard import (NBATCH, NSEG, SEG, SHARD_SEGMENTS, all_ranks_ok,
                              gather_results, gather_strings, max_over_ranks, shard_for)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    sys.path.insert(0, os.path.join(root, "tests"))
    from oracle import Oracle
    import golden_util

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}",
                            rank=rank, world_size=world)
    try:
        orc = Oracle()
        sh = shard_for(rank, world)
        arena = orc.splitmix_bytes(sh.nbytes, byte_off=sh.byte_offset)
        out = orc.batch(arena, stride=SEG, fixed_len=SEG, n=sh.seg_count, nthreads=4)
        digest = f"{orc.fnv1a_u16(out):016x}"
        gold = golden_util.digests()["batches"]["M8x1500"]["shards"][rank]["fnv1a64"]
        t = max_over_ranks(float(rank + 1) * 0.5, dist)
        ok_all = all_ranks_ok(digest == gold, dist)
        veto = all_ranks_ok(rank == 0, dist)   # rank 1 votes no
        digests = gather_strings(digest, dist)
        import torch
        words = torch.from_numpy(out.view(np.int16).copy()).view(torch.uint16)
        allw = gather_results(words, dist, torch.device("cpu")).view(torch.int16).numpy()
        gathered = [f"{orc.fnv1a_u16(allw[r * len(out):(r + 1) * len(out)].view(np.uint16)):016x}"
                    for r in range(world)]
        q.put((rank, digest == gold, t, ok_all, veto, digests, sh.byte_offset,
               sh.batch_offset(3), gathered))
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
def test_two_rank_shards_match_reference_digests():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, t, ok_all, veto, digests, boff, b3, gathered in res:
        assert gathered == digests            # results all-gather, rank order
        assert ok, f"rank {rank} shard digest != reference M8 shard {rank}"
        assert t == 1.0                       # max over ranks of 0.5, 1.0
        assert ok_all and not veto
        assert digests == [res[0][5][0], res[1][5][1]]
        assert boff == rank * SHARD_SEGMENTS * SEG
        assert b3 == 3 * NSEG * SEG


def test_shard_layout():
    s = shard_for(3, 8)
    assert s.seg_begin == 3 * NBATCH * NSEG and s.seg_count == NBATCH * NSEG
    assert s.nbytes == NBATCH * NSEG * SEG
    assert s.batch_offset(NBATCH + 1) == NSEG * SEG
    with pytest.raises(ValueError):
        shard_for(2, 2)
    # single-process fallbacks
    assert max_over_ranks(2.5) == 2.5 and all_ranks_ok(True) and gather_strings("x") == ["x"]
    assert np.uint64(s.byte_offset) == np.uint64(3 * 2**20 * 1500)


def _zipf_worker(rank, world, port, q):
    """World 4 / 8: the golden ZIPF batch cut by byte_shard_for (the plan the
    bench's zipf leg uses), each rank checksumming its contiguous shard of the
    packed arena (oracle standing in for the kernel), results padded to the
    longest shard and all-gathered (gather_results): reassembled in rank order
    they must give the reference's ZIPF digest. Also the M8 shard layout at
    this world size and the control-plane reductions."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    sys.path.insert(0, os.path.join(root, "tests"))
    import torch
    from oracle import Oracle
    import golden_util
    from tulips_amd.shard import byte_shard_for

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}",
                            rank=rank, world_size=world)
    try:
        orc = Oracle()
        lens = orc.zipf_lengths(NSEG)
        bs = byte_shard_for(rank, world, lens)
        ll = lens[bs.seg_begin:bs.seg_begin + bs.seg_count]
        offs = np.zeros(len(ll), np.uint64)
        if len(ll) > 1:
            np.cumsum(ll[:-1], dtype=np.uint64, out=offs[1:])
        arena = orc.splitmix_bytes(bs.nbytes + 16, byte_off=bs.byte_offset)
        out = orc.batch(arena, offs, ll, nthreads=2) if len(ll) else np.zeros(0, np.uint16)
        cmax = int(max_over_ranks(float(len(ll)), dist))
        pad = torch.zeros(cmax, dtype=torch.int16)
        pad[:len(ll)] = torch.from_numpy(out.view(np.int16).copy())
        allw = gather_results(pad.view(torch.uint16), dist, torch.device("cpu"))
        allw = allw.view(torch.int16).numpy().view(np.uint16)
        counts = [int(c) for c in gather_strings(str(len(ll)), dist)]
        glob = np.concatenate([allw[r * cmax:r * cmax + counts[r]] for r in range(world)])
        gold = golden_util.digests()["batches"]["ZIPF"]["fnv1a64"]
        sh = shard_for(rank, world)
        q.put((rank, f"{orc.fnv1a_u16(glob):016x}" == gold, counts, bs.seg_begin,
               bs.byte_offset, sh.byte_offset, max_over_ranks(float(rank), dist),
               all_ranks_ok(rank != world - 1, dist)))
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("world", [4, 8])
def test_world_4_and_8_byte_shards_gather_in_rank_order(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_zipf_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    counts = res[0][2]
    assert sum(counts) == NSEG and all(r[2] == counts for r in res)
    begins = np.concatenate([[0], np.cumsum(counts)[:-1]])
    for rank, ok, _, seg_begin, boff, m8off, tmax, veto in res:
        assert ok, f"rank {rank}: reassembled ZIPF results != reference digest"
        assert seg_begin == begins[rank]
        assert m8off == rank * SHARD_SEGMENTS * SEG
        assert tmax == world - 1 and not veto
    # byte offsets are the prefix sums of the shards' lengths
    assert res[0][4] == 0 and all(res[r][4] < res[r + 1][4] for r in range(world - 1))
