"""Sharding of the checksum workload across ranks (one process per GPU).

Segments are independent: rank r owns a contiguous shard of
the batch stream and computes it with no data-path collective. The only
cross-rank traffic is control: the timing barrier, the max-over-ranks time,
the parity vote and (outside any timed region) the per-shard digests.

Layout (M8x1500, BASELINE configs[4]): 8,388,608 segments of 1500 B; shard r
is segments [r * 2^20, (r+1) * 2^20), i.e. SplitMix64 stream bytes
[r * 2^20 * 1500, (r+1) * 2^20 * 1500). A shard is 16 batches of 65,536
segments (one batch = one bench step).
"""
from __future__ import annotations

from dataclasses import dataclass

SEG = 1500
NSEG = 65536           # segments per batch (one step)
NBATCH = 16            # batches per shard
SHARD_SEGMENTS = NSEG * NBATCH


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    seg_begin: int      # global index of the shard's first segment
    seg_count: int
    byte_offset: int    # offset of the shard in the global SplitMix64 stream
    nbytes: int

    def batch_offset(self, b: int) -> int:
        """Byte offset of batch b inside the shard's arena."""
        return (b % NBATCH) * NSEG * SEG


def shard_for(rank: int, world: int) -> Shard:
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    begin = rank * SHARD_SEGMENTS
    return Shard(rank, world, begin, SHARD_SEGMENTS, begin * SEG, SHARD_SEGMENTS * SEG)


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """Slowest rank's time (the contract's max-over-ranks)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_ranks_ok(ok: bool, dist=None, device=None) -> bool:
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return ok
    import torch
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item()) == 1


def gather_strings(s: str, dist=None) -> list:
    """Per-rank strings (e.g. shard digests) at every rank."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [s]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, s)
    return out


def gather_results(out, dist=None, device=None):
    """All ranks' result words (uint16, same count per rank) at every rank, in
    rank order: the one data-path exchange the sharded path could have
    (an all-gather of the uint16 outputs, 2 MiB per GPU for
    M8x1500). Under RCCL the bytes move GPU to GPU over xGMI; under gloo
    (CPU rehearsal) through host memory. Returns a tensor on out.device."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return out.clone()
    world = dist.get_world_size()
    flat = out.contiguous().view(torch.uint8)      # RCCL has no 16-bit integer type
    if device is not None and device.type == "cpu":
        src = flat.cpu()
        dst = torch.empty(world * src.numel(), dtype=torch.uint8)
        dist.all_gather_into_tensor(dst, src)
        return dst.to(out.device).view(out.dtype)
    dst = torch.empty(world * flat.numel(), dtype=torch.uint8, device=flat.device)
    dist.all_gather_into_tensor(dst, flat)
    return dst.view(out.dtype)


@dataclass(frozen=True)
class ByteShard:
    """A rank's part of a variable-length batch, cut by the library's
    byte-balanced plan (tulips_csum_shard_plan)."""
    rank: int
    world: int
    seg_begin: int
    seg_count: int
    byte_offset: int    # offset of the shard's first segment in the packed arena
    nbytes: int


def byte_shard_for(rank: int, world: int, lengths) -> ByteShard:
    """Contiguous shard `rank` of a packed batch with these lengths, balanced
    by bytes ("balance by bytes for Zipf (prefix sum of
    lengths)"); every rank computes the same plan locally, no exchange."""
    import numpy as np
    from tulips_amd import csum
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    lens = np.ascontiguousarray(lengths, dtype=np.uint16)
    b = csum.shard_plan(lens, world)
    i0, i1 = int(b[rank]), int(b[rank + 1])
    pre = int(lens[:i0].astype(np.int64).sum())
    nb = int(lens[i0:i1].astype(np.int64).sum())
    return ByteShard(rank, world, i0, i1 - i0, pre, nb)
