#!/usr/bin/env python3
"""Generate the committed golden fixtures from the REFERENCE itself.

Every expected value here is produced by ``oracle/_ref/libtulips_ref.so``,
i.e. the reference's own ``src/stack`` translation units (Utils.cpp, IPv4.cpp,
ICMPv4.cpp, tcpv4/Processor.cpp, ...) compiled by ``oracle/Makefile`` from
``/root/reference``. Run it in the build container (where /root/reference
exists):

    make -C oracle && python tests/golden/make_golden.py

Outputs (small, committed):
  kat.json          single-call known answers for a1/a2/a5/a6
  adversarial.npz   a 192 KiB random arena + edge-case segments (every length
                    class, every start alignment 0..15, odd offsets, seeds,
                    overlapping segments) with the reference's outputs per mode
  digests.json      FNV-1a-64 / sum digests of the SURVEY.md §8c batches
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from oracle import (DATA_SEED, MODE_INET, MODE_RAW, MODE_TCP,  # noqa: E402
                    FLAG_COMPLEMENT, Oracle, Reference, fixed_offsets, ip4,
                    packed_offsets)

NTHREADS = min(8, os.cpu_count() or 1)


def kat(ref: Reference) -> list:
    rows = []

    def a1(seed, data):
        rows.append({"fn": "checksum", "seed": seed, "data": data.hex(),
                     "expect": ref.checksum(seed, data)})

    # SURVEY.md §8a known answers (re-derived here from the reference)
    a1(0, bytes.fromhex("0001f203f4f5f6f7"))          # RFC 1071 example
    a1(0x1234, b"")
    a1(0, bytes.fromhex("0001f2"))
    a1(0, bytes.fromhex("ffff0001"))
    a1(0, bytes.fromhex("ffff"))
    a1(0, bytes.fromhex("ffffffff"))
    a1(0xFFFF, bytes(4))
    a1(0, bytes(4))
    a1(1, bytes.fromhex("ffff"))
    a1(0, b"")
    a1(0xFFFF, b"")
    a1(0, b"\x80")
    a1(0xFFFF, b"\xff")
    a1(0x0001, b"\xff\xfe")
    rng = np.random.default_rng(1071)
    for L in list(range(0, 40)) + [63, 64, 65, 127, 128, 129, 1499, 1500, 1501]:
        for seed in (0, 1, 0x7FFF, 0xFFFE, 0xFFFF, int(rng.integers(0, 65536))):
            a1(seed, rng.integers(0, 256, L, dtype=np.uint8).tobytes())
    for L in (2, 3, 8, 9, 20):
        a1(0, b"\xff" * L)
        a1(0xFFFF, b"\xff" * L)
        a1(0, b"\x00" * L)

    ip = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
    rows.append({"fn": "ipv4", "data": ip.hex(), "expect": ref.ipv4_checksum(ip)})
    v = ref.ipv4_checksum(ip)
    stored = (~v) & 0xFFFF  # ipv4/Producer.cpp:81 writes ~checksum
    ip2 = ip[:10] + stored.to_bytes(2, "little") + ip[12:]
    rows.append({"fn": "ipv4", "data": ip2.hex(), "expect": ref.ipv4_checksum(ip2)})
    for _ in range(16):
        h = rng.integers(0, 256, 20, dtype=np.uint8).tobytes()
        rows.append({"fn": "ipv4", "data": h.hex(), "expect": ref.ipv4_checksum(h)})

    icmp = bytes.fromhex("0800000012340001")
    rows.append({"fn": "icmpv4", "data": icmp.hex(), "expect": ref.icmpv4_checksum(icmp)})
    for _ in range(16):
        h = rng.integers(0, 256, 8, dtype=np.uint8).tobytes()
        rows.append({"fn": "icmpv4", "data": h.hex(), "expect": ref.icmpv4_checksum(h)})

    syn = bytes.fromhex("22b8270f000000010000000050022000" "00000000")
    src, dst = ip4(10, 1, 0, 1), ip4(10, 1, 0, 2)
    rows.append({"fn": "tcp", "src": src, "dst": dst, "data": syn.hex(),
                 "expect": ref.tcp_checksum(src, dst, syn)})
    for L in (0, 1, 20, 21, 40, 61, 1460, 1480):
        for _ in range(3):
            s = int(rng.integers(0, 2**32)); d = int(rng.integers(0, 2**32))
            seg = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
            rows.append({"fn": "tcp", "src": s, "dst": d, "data": seg.hex(),
                         "expect": ref.tcp_checksum(s, d, seg)})
    # the uint16 `len + 6` wrap of Processor.cpp:346 (len > 65529)
    # (segment bytes given by the SplitMix64 stream spec to keep the file small)
    orc = Oracle()
    for L in (65529, 65530, 65531, 65535):
        seg = orc.splitmix_bytes(L, seed=L).tobytes()
        s = int(rng.integers(0, 2**32)); d = int(rng.integers(0, 2**32))
        rows.append({"fn": "tcp", "src": s, "dst": d, "data_splitmix": [L, L],
                     "expect": ref.tcp_checksum(s, d, seg)})
    return rows


EDGE_LENGTHS = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65,
                127, 128, 129, 255, 256, 257, 1023, 1024, 1025, 1499, 1500,
                1501, 4095, 4096, 4097, 8999, 9000, 9001, 16383, 16384, 16385,
                65534, 65535]


def adversarial(ref: Reference, orc: Oracle) -> dict:
    rng = np.random.default_rng(8937)
    arena_n = 192 * 1024
    arena = orc.splitmix_bytes(arena_n, seed=0xADE5A11)
    offs, lens = [], []
    for L in EDGE_LENGTHS:
        for start in range(0, 18):          # every alignment mod 16, plus 16, 17
            base = int(rng.integers(0, arena_n - L - 64)) & ~63
            offs.append(base + start)
            lens.append(L)
    for _ in range(2000):                   # random segments, random alignment
        L = int(rng.integers(0, 20000))
        offs.append(int(rng.integers(0, arena_n - L)))
        lens.append(L)
    offs = np.array(offs, dtype=np.uint64)
    lens = np.array(lens, dtype=np.uint16)
    n = len(offs)
    seeds = rng.integers(0, 65536, n, dtype=np.uint16)
    seeds[:64] = 0
    seeds[64:128] = 0xFFFF
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    out = {}
    kw = dict(nthreads=NTHREADS)
    out["raw_noseed"] = ref.batch(arena, offs, lens, mode=MODE_RAW, **kw)
    out["raw_seed"] = ref.batch(arena, offs, lens, seeds=seeds, mode=MODE_RAW, **kw)
    out["inet_seed"] = ref.batch(arena, offs, lens, seeds=seeds, mode=MODE_INET, **kw)
    out["tcp"] = ref.batch(arena, offs, lens, src=src, dst=dst, mode=MODE_TCP, **kw)
    out["tcp_complement"] = ref.batch(arena, offs, lens, src=src, dst=dst,
                                      mode=MODE_TCP | FLAG_COMPLEMENT, **kw)
    # constant arenas: the 0x0000 / 0xffff representation paths
    zeros = np.zeros(arena_n, dtype=np.uint8)
    ones = np.full(arena_n, 0xFF, dtype=np.uint8)
    out["zeros_raw_seed"] = ref.batch(zeros, offs, lens, seeds=seeds, mode=MODE_RAW, **kw)
    out["zeros_inet_noseed"] = ref.batch(zeros, offs, lens, mode=MODE_INET, **kw)
    out["ones_raw_seed"] = ref.batch(ones, offs, lens, seeds=seeds, mode=MODE_RAW, **kw)
    out["ones_tcp"] = ref.batch(ones, offs, lens, src=src, dst=dst, mode=MODE_TCP, **kw)
    return dict(arena=arena, offsets=offs, lengths=lens, seeds=seeds, src=src,
                dst=dst, **{"expect_" + k: v for k, v in out.items()})


def digest(orc, v):
    return {"fnv1a64": f"{orc.fnv1a_u16(v):016x}", "sum": int(v.astype(np.int64).sum())}


def digests(ref: Reference, orc: Oracle) -> dict:
    N = 65536
    d = {"spec": "SURVEY.md §8c: SplitMix64 arena seed 0x54554C495053, packed; "
                 "FNV-1a-64 over u16 outputs (LE bytes); TCP src 10.1.0.1 dst 10.1.0.2",
         "batches": {}}
    src = np.full(N, ip4(10, 1, 0, 1), dtype=np.uint32)
    dst = np.full(N, ip4(10, 1, 0, 2), dtype=np.uint32)
    kw = dict(nthreads=NTHREADS)
    for L, stride in ((1500, 1500), (1500, 2048), (9000, 9000), (9000, 9216), (64, 64)):
        arena = orc.splitmix_bytes(N * stride)
        v = ref.batch(arena, stride=stride, fixed_len=L, n=N, mode=MODE_RAW, **kw)
        name = f"F{L}" + ("" if stride == L else f"s{stride}")
        d["batches"][name] = dict(n=N, length=L, stride=stride, mode="raw", **digest(orc, v))
        if stride == L and L in (1500, 9000):
            v = ref.batch(arena, stride=stride, fixed_len=L, n=N, mode=MODE_TCP,
                          src=src, dst=dst, **kw)
            d["batches"][name + "-tcp"] = dict(n=N, length=L, stride=stride, mode="tcp",
                                               **digest(orc, v))
    lens = orc.zipf_lengths(N)
    offs = packed_offsets(lens)
    arena = orc.splitmix_bytes(int(lens.astype(np.int64).sum()))
    d["zipf_lengths"] = {"fnv1a64": f"{orc.fnv1a_u16(lens):016x}",
                         "total": int(lens.astype(np.int64).sum()),
                         "min": int(lens.min()), "max": int(lens.max()),
                         "odd": int((lens & 1).sum()), "first4": [int(x) for x in lens[:4]]}
    v = ref.batch(arena, offs, lens, mode=MODE_RAW, **kw)
    d["batches"]["ZIPF"] = dict(n=N, mode="raw", **digest(orc, v))
    v = ref.batch(arena, offs, lens, mode=MODE_TCP, src=src, dst=dst, **kw)
    d["batches"]["ZIPF-tcp"] = dict(n=N, mode="tcp", **digest(orc, v))
    # M8x1500: 8 contiguous shards of 1,048,576 segments (8.4 M total)
    shard_n, L = 1 << 20, 1500
    shard_digests, all_out = [], []
    for r in range(8):
        arena = orc.splitmix_bytes(shard_n * L, byte_off=r * shard_n * L)
        v = ref.batch(arena, stride=L, fixed_len=L, n=shard_n, mode=MODE_RAW, **kw)
        shard_digests.append(dict(digest(orc, v), batches=m8_batch_digests(orc, v)))
        all_out.append(v)
        del arena
    full = np.concatenate(all_out)
    d["batches"]["M8x1500"] = dict(n=8 * shard_n, length=L, stride=L, mode="raw",
                                   shards=shard_digests, **digest(orc, full))
    d["rotations"] = rotation_digests(ref, orc)
    return d


def rotation_digests(ref, orc, n9=4, nz=24):
    """Digests of the distinct batches bench.py rotates over so that its
    side measurements stream from HBM: F9000 batch b = SplitMix64 stream
    bytes [b * 589,824,000, ...) (stride 9000), ZIPF copy c = the golden Zipf
    lengths over stream bytes [c * 43,772,673, ...). Batch/copy 0 are the
    F9000 / ZIPF digests."""
    N = 65536
    out = {"F9000": [], "ZIPF": []}
    b9 = N * 9000
    for b in range(n9):
        arena = orc.splitmix_bytes(b9, byte_off=b * b9)
        v = ref.batch(arena, stride=9000, fixed_len=9000, n=N, mode=MODE_RAW,
                      nthreads=NTHREADS)
        out["F9000"].append(f"{orc.fnv1a_u16(v):016x}")
        del arena
    lens = orc.zipf_lengths(N)
    offs = packed_offsets(lens)
    zb = int(lens.astype(np.int64).sum())
    for c in range(nz):
        arena = orc.splitmix_bytes(zb, byte_off=c * zb)
        v = ref.batch(arena, offs, lens, mode=MODE_RAW, nthreads=NTHREADS)
        out["ZIPF"].append(f"{orc.fnv1a_u16(v):016x}")
    return out


def patch_rotations():
    """Add rotation_digests() to an existing digests.json."""
    ref, orc = Reference(), Oracle()
    path = os.path.join(HERE, "digests.json")
    with open(path) as f:
        d = json.load(f)
    d["rotations"] = rotation_digests(ref, orc)
    assert d["rotations"]["F9000"][0] == d["batches"]["F9000"]["fnv1a64"]
    assert d["rotations"]["ZIPF"][0] == d["batches"]["ZIPF"]["fnv1a64"]
    with open(path, "w") as f:
        json.dump(d, f, indent=1)


def m8_batch_digests(orc, shard_out):
    """FNV-1a-64 of each 65,536-segment batch of one M8 shard's results:
    bench.py's rotating F1500 steps (a step writes one batch), so a timed run
    of fewer than 16 steps still has a reference digest per batch written."""
    return [f"{orc.fnv1a_u16(shard_out[b * 65536:(b + 1) * 65536]):016x}"
            for b in range(len(shard_out) // 65536)]


def patch_m8_batches():
    """Add the per-batch digests to an existing digests.json (same reference
    build, same arenas as digests())."""
    ref, orc = Reference(), Oracle()
    path = os.path.join(HERE, "digests.json")
    with open(path) as f:
        d = json.load(f)
    shard_n, L = 1 << 20, 1500
    m8 = d["batches"]["M8x1500"]
    for r in range(8):
        arena = orc.splitmix_bytes(shard_n * L, byte_off=r * shard_n * L)
        v = ref.batch(arena, stride=L, fixed_len=L, n=shard_n, mode=MODE_RAW,
                      nthreads=NTHREADS)
        assert f"{orc.fnv1a_u16(v):016x}" == m8["shards"][r]["fnv1a64"]
        m8["shards"][r]["batches"] = m8_batch_digests(orc, v)
        del arena
    with open(path, "w") as f:
        json.dump(d, f, indent=1)


RSS_KEYS = {
    # tests/stack/utils.cpp:11-23 (DYNAMIC_KEY / STATIC_KEY, 40 bytes)
    "dynamic40": bytes.fromhex("008be05ed4a554f83cf808"
                               "75072c4e8b6f1dbf103b043b41b3a4a4ae56c9a4ec1376a0af04108166"),
    "static40": bytes.fromhex("beac01fa6a42b73b8030f20c77cb2da3ae7b30b4d0ca2bcb43a38fb041"
                              "67253d255b0ec26d5a56da"),
}


def rss(ref: Reference) -> dict:
    """Toeplitz RSS (src/stack/Utils.cpp:86-133) fixtures: the reference's two
    KATs (tests/stack/utils.cpp:37,54) plus 4096 random tuples per key for
    keys of 4..52 bytes (short keys exercise the wrap-around quirk)."""
    rng = np.random.default_rng(9899)
    keys = dict(RSS_KEYS)
    for L in (4, 5, 7, 12, 15, 16, 17, 52):
        keys[f"rand{L}"] = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
    n = 4096
    sa = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    da = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    sp = rng.integers(0, 65536, n, dtype=np.uint16)
    dp = rng.integers(0, 65536, n, dtype=np.uint16)
    sa[0], da[0], sp[0], dp[0] = ip4(10, 1, 0, 1), ip4(10, 1, 0, 2), 8888, 9999
    out = {"saddr": sa, "daddr": da, "sport": sp, "dport": dp}
    names = sorted(keys)
    out["key_names"] = np.array(names)
    for i, name in enumerate(names):
        k = keys[name]
        out[f"key_{i}"] = np.frombuffer(k, dtype=np.uint8)
        for init, tag in ((0, "init0"), (0xFFFFFFFF, "initff")):
            out[f"expect_{i}_{tag}"] = np.array(
                [ref.toeplitz(int(sa[j]), int(da[j]), int(sp[j]), int(dp[j]), k, init)
                 for j in range(n)], dtype=np.uint32)
    return out


def _ref_frame_flags(ref: Reference, f: bytes) -> int:
    """Expected TULIPS_FRAME_* flags: the receive chain's checks
    (ethernet/Processor.cpp:69,91; ipv4/Processor.cpp:67-122;
    tcpv4/Processor.cpp:121-131) evaluated with the REFERENCE's own
    ipv4::checksum and tcpv4::Processor::checksum."""
    if len(f) < 14 or (f[12] << 8 | f[13]) != 0x0800:
        return 0
    if len(f) < 34:
        return 0x10
    ip = f[14:]
    if ip[0] != 0x45:
        return 0
    fl = 0x01 | (0x02 if ref.ipv4_checksum(ip[:20]) == 0xFFFF else 0)
    if (ip[6] & 0x3F) != 0 or ip[7] != 0 or ip[9] != 6:
        return fl
    fl |= 0x04
    total = ip[2] << 8 | ip[3]
    tcplen = (total - 20) & 0xFFFF
    if total < 20 or 34 + tcplen > len(f):
        return fl | 0x10
    src = int.from_bytes(ip[12:16], "little")
    dst = int.from_bytes(ip[16:20], "little")
    if ref.tcp_checksum(src, dst, ip[20:20 + tcplen]) == 0xFFFF:
        fl |= 0x08
    return fl


def _make_frame(ref: Reference, rng, payload: int, pad_to: int = 0) -> bytearray:
    """A well-formed Ethernet/IPv4/TCP frame, checksums generated as the send
    path writes them (ipv4/Producer.cpp:79-82, tcpv4/Send.cpp:441-449)."""
    eth = rng.integers(0, 256, 12, dtype=np.uint8).tobytes() + b"\x08\x00"
    src, dst = rng.integers(0, 256, 4, dtype=np.uint8), rng.integers(0, 256, 4, dtype=np.uint8)
    tcp = bytearray(rng.integers(0, 256, 20, dtype=np.uint8).tobytes())
    tcp[12] = 0x50
    tcp[16:18] = b"\0\0"
    seg = bytes(tcp) + rng.integers(0, 256, payload, dtype=np.uint8).tobytes()
    s32, d32 = int.from_bytes(bytes(src), "little"), int.from_bytes(bytes(dst), "little")
    c = (~ref.tcp_checksum(s32, d32, seg)) & 0xFFFF
    seg = seg[:16] + c.to_bytes(2, "little") + seg[18:]
    total = 20 + len(seg)
    ip = bytearray(b"\x45\x00" + total.to_bytes(2, "big") +
                   rng.integers(0, 256, 2, dtype=np.uint8).tobytes() + b"\x40\x00\x40\x06\x00\x00" +
                   bytes(src) + bytes(dst))
    c = (~ref.ipv4_checksum(bytes(ip))) & 0xFFFF
    ip[10:12] = c.to_bytes(2, "little")
    f = bytearray(eth + bytes(ip) + seg)
    if len(f) < pad_to:
        f += bytes(pad_to - len(f))        # Ethernet minimum-size padding
    return f


def frames(ref: Reference, orc: Oracle) -> dict:
    rng = np.random.default_rng(2020)
    out = []
    for i in range(3000):
        kind = i % 16
        payload = int(rng.choice([0, 1, 2, 7, 8, 31, 64, 100, 512, 1459, 1460,
                                  int(rng.integers(0, 1461))]))
        f = _make_frame(ref, rng, payload, pad_to=60)
        if kind == 1:                                   # IP header bit flip
            b = 14 + int(rng.integers(0, 20))
            f[b] ^= 1 << int(rng.integers(0, 8))
        elif kind == 2 and len(f) > 34:                 # TCP bit flip
            b = 34 + int(rng.integers(0, len(f) - 34))
            f[b] ^= 1 << int(rng.integers(0, 8))
        elif kind == 3:
            f[14] = 0x46                                # IP options: unsupported
        elif kind == 4:
            f[20] |= 0x01                               # fragment offset
        elif kind == 5:
            f[23] = 17                                  # UDP
        elif kind == 6:
            f[12:14] = b"\x08\x06"                      # ARP
        elif kind == 7:
            f = f[:max(34, len(f) - int(rng.integers(1, 40)))]   # truncated
        elif kind == 8:
            f[16:18] = (10).to_bytes(2, "big")          # total length < 20
        elif kind == 9:
            f = f[:int(rng.integers(0, 34))]            # runt
        elif kind == 10:
            f[21] = 1                                   # fragment (low offset byte)
        elif kind == 11:
            f[20] = 0x80 | (f[20] & 0x3F)               # reserved flag bit only
        if kind in (4, 5, 8, 10, 11) and i % 32 < 16:   # re-seal the IP header
            f[24:26] = b"\0\0"
            c = (~ref.ipv4_checksum(bytes(f[14:34]))) & 0xFFFF
            f[24:26] = c.to_bytes(2, "little")
        out.append(bytes(f))
    lens = np.array([len(f) for f in out], dtype=np.uint16)
    gaps = rng.integers(0, 16, len(out))
    offs, pos, chunks = [], 3, [rng.integers(0, 256, 3, dtype=np.uint8).tobytes()]
    for f, g in zip(out, gaps):
        offs.append(pos)
        chunks.append(f + rng.integers(0, 256, int(g), dtype=np.uint8).tobytes())
        pos += len(f) + int(g)
    arena = np.frombuffer(b"".join(chunks) + bytes(64), dtype=np.uint8)
    offs = np.array(offs, dtype=np.uint64)
    expect = np.array([_ref_frame_flags(ref, f) for f in out], dtype=np.uint8)
    np.testing.assert_array_equal(orc.validate_frames(arena, offs, lens), expect)
    return dict(arena=arena, offsets=offs, lengths=lens, expect=expect)


def main():
    ref = Reference()
    orc = Oracle()
    fr = frames(ref, orc)
    np.savez_compressed(os.path.join(HERE, "frames.npz"), **fr)
    np.savez_compressed(os.path.join(HERE, "rss.npz"), **rss(ref))
    rows = kat(ref)
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump({"source": "oracle/_ref/libtulips_ref.so (reference src/stack compiled)",
                   "cases": rows}, f, indent=0)
    adv = adversarial(ref, orc)
    np.savez_compressed(os.path.join(HERE, "adversarial.npz"), **adv)
    dg = digests(ref, orc)
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(dg, f, indent=1)
    print(f"kat: {len(rows)} cases; adversarial: {len(adv['offsets'])} segments; "
          f"digests: {sorted(dg['batches'])}")


if __name__ == "__main__":
    import sys
    if sys.argv[1:] == ["--m8-batches"]:
        patch_m8_batches()
    elif sys.argv[1:] == ["--rotations"]:
        patch_rotations()
    else:
        main()
