"""N>1 path with the real HIP kernels: four ranks (processes) on the one GPU
of the box, joined by gloo, each running the bench's shard harness through
the product library (tulips_amd/libtulips_csum.so), not the oracle.

Rank r fills M8x1500 shard r on the device (tulips_csum_fill_splitmix, the
§8c stream at the shard's byte offset) and checksums its 16 batches with
tulips_csum_batch_fixed; the shard digest must equal the reference's. The
results are all-gathered in rank order (tulips_amd.shard.gather_results, the
exchange §8e names) and every rank checks every other rank's shard in the
gathered words. Then the golden ZIPF batch is cut by bytes
(byte_shard_for -> tulips_csum_shard_plan), each rank checksums its shard of
the packed arena with tulips_csum_batch_arena, and the gathered results
reassembled in rank order must give the reference's ZIPF digest.

The 8-GPU RCCL run is the driver's; this covers the rank-count-dependent
code with the GPU kernels in the loop (four processes on one card stay well
inside the box's limit of 16)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tulips_amd.shard import NBATCH, NSEG, SEG, SHARD_SEGMENTS

pytestmark = pytest.mark.gpu

WORLD = 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist
    import bench
    from tulips_amd import csum
    import benchlib
    from tulips_amd.shard import (all_ranks_ok, byte_shard_for, gather_results,
                                  gather_strings, shard_for)

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}",
                            rank=rank, world_size=world)
    try:
        gold = bench.golden_digests()
        lib = csum.lib
        st = torch.cuda.current_stream().cuda_stream
        # M8x1500 shard <rank>, as bench.py lays it out
        sh = shard_for(rank, world)
        arena = torch.empty(sh.nbytes + 256, dtype=torch.uint8, device=dev)
        benchlib.fill_splitmix(arena, sh.nbytes, seed=bench.DATA_SEED, byte_off=sh.byte_offset)
        outs = torch.empty(NBATCH * NSEG, dtype=torch.uint16, device=dev)
        for b in range(NBATCH):
            rc = lib.tulips_csum_batch_fixed(arena.data_ptr() + sh.batch_offset(b), SEG, SEG,
                                             None, None, None, outs.data_ptr() + b * NSEG * 2,
                                             NSEG, 0, st)
            assert rc == 0, rc
        torch.cuda.synchronize()
        del arena
        host = outs.cpu()
        mine = bench.fnv1a_u16(host.view(torch.int16).numpy().view(np.uint16))
        allw = gather_results(host, dist, torch.device("cpu"))
        allw = allw.view(torch.int16).numpy().view(np.uint16)
        m8 = [s["fnv1a64"] for s in gold["M8x1500"]["shards"]]
        # (rank 0 digests every rank's part of the gathered words)
        gathered = m8[:world] if rank else [
            bench.fnv1a_u16(allw[r * SHARD_SEGMENTS:(r + 1) * SHARD_SEGMENTS])
            for r in range(world)]
        digests = gather_strings(mine, dist)

        # ZIPF cut by bytes, each shard through the arena entry point
        lens = bench.zipf_lengths(NSEG)
        bs = byte_shard_for(rank, world, lens)
        ll = lens[bs.seg_begin:bs.seg_begin + bs.seg_count]
        offs = np.zeros(len(ll), dtype=np.uint64)
        if len(ll) > 1:
            np.cumsum(ll[:-1], dtype=np.uint64, out=offs[1:])
        az = torch.empty(bs.nbytes + 256, dtype=torch.uint8, device=dev)
        benchlib.fill_splitmix(az, bs.nbytes, byte_off=bs.byte_offset)
        doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
        dlens = torch.from_numpy(ll.view(np.int16).copy()).to(dev)
        zo = torch.empty(max(1, len(ll)), dtype=torch.uint16, device=dev)
        rc = lib.tulips_csum_batch_arena(az.data_ptr(), bs.nbytes, doffs.data_ptr(),
                                         dlens.data_ptr(), None, None, None, zo.data_ptr(),
                                         len(ll), 0, st)
        assert rc == 0, rc
        torch.cuda.synchronize()
        counts = [int(c) for c in gather_strings(str(len(ll)), dist)]
        cmax = max(counts)
        pad = torch.zeros(cmax, dtype=torch.uint16)
        pad[:len(ll)] = zo[:len(ll)].cpu()
        zall = gather_results(pad, dist, torch.device("cpu"))
        zall = zall.view(torch.int16).numpy().view(np.uint16)
        glob = np.concatenate([zall[r * cmax:r * cmax + counts[r]] for r in range(world)])
        zipf_ok = bench.fnv1a_u16(glob) == gold["ZIPF"]["fnv1a64"]
        q.put((rank, mine == m8[rank], gathered == m8[:world], digests == m8[:world],
               zipf_ok, counts, all_ranks_ok(mine == m8[rank] and zipf_ok, dist)))
    finally:
        dist.destroy_process_group()


def test_four_ranks_on_gpu_shards_and_gather_match_reference_digests():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=150) for _ in range(WORLD))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    counts = res[0][5]
    assert sum(counts) == NSEG and all(r[5] == counts for r in res)
    for rank, own, gathered, digests, zipf_ok, _, all_ok in res:
        assert own, f"rank {rank}: M8 shard {rank} digest != reference"
        assert gathered, f"rank {rank}: all-gathered shard results out of rank order"
        assert digests
        assert zipf_ok, f"rank {rank}: byte-sharded ZIPF results != reference digest"
        assert all_ok
