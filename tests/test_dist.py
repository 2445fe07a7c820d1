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
