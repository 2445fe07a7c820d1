"""Pin the CPU restatement (oracle/csum_oracle.c) to the reference.

The reference's own tests hold no absolute checksum value, so
the pins are the fixtures that tests/golden/make_golden.py computed with the
reference's compiled src/stack, plus a live cross-check against that build
where it is present (oracle/_ref/libtulips_ref.so).
"""
import numpy as np
import pytest

from oracle import (MODE_INET, MODE_RAW, MODE_TCP, FLAG_COMPLEMENT, REF_CLANG_SO, Reference,
                    fixed_offsets, ip4, packed_offsets)


def test_kat(oracle, golden):
    for c in golden.kat():
        data = golden.kat_data(c, oracle)
        fn = c["fn"]
        if fn == "checksum":
            got = oracle.checksum(c["seed"], data)
        elif fn == "ipv4":
            got = oracle.ipv4_checksum(data)
        elif fn == "icmpv4":
            got = oracle.icmpv4_checksum(data)
        else:
            got = oracle.tcp_checksum(c["src"], c["dst"], data)
        assert got == c["expect"], c


def test_survey_known_answers(oracle):
    # SURVEY.md §8a list (independently of the fixture file)
    assert oracle.checksum(0, bytes.fromhex("0001f203f4f5f6f7")) == 0xDDF2
    assert oracle.checksum(0x1234, b"") == 0x1234
    assert oracle.checksum(0, bytes.fromhex("0001f2")) == 0xF201
    assert oracle.checksum(0, bytes.fromhex("ffff0001")) == 0x0001
    assert oracle.checksum(0, b"\xff\xff") == 0xFFFF
    assert oracle.checksum(0, b"\xff" * 4) == 0xFFFF
    assert oracle.checksum(0xFFFF, bytes(4)) == 0xFFFF
    assert oracle.checksum(0, bytes(4)) == 0
    assert oracle.checksum(1, b"\xff\xff") == 1
    ip = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
    assert oracle.checksum(0, ip) == 0x479E
    assert oracle.ipv4_checksum(ip) == 0x9E47
    stored = (~oracle.ipv4_checksum(ip)) & 0xFFFF
    assert stored.to_bytes(2, "little") == bytes.fromhex("b861")
    ip2 = ip[:10] + stored.to_bytes(2, "little") + ip[12:]
    assert oracle.ipv4_checksum(ip2) == 0xFFFF
    syn = bytes.fromhex("22b8270f00000001000000005002200000000000")
    src, dst = ip4(10, 1, 0, 1), ip4(10, 1, 0, 2)
    v = oracle.tcp_checksum(src, dst, syn)
    assert v == 0xE9CD
    syn2 = syn[:16] + ((~v) & 0xFFFF).to_bytes(2, "little") + syn[18:]
    assert oracle.tcp_checksum(src, dst, syn2) == 0xFFFF
    icmp = bytes.fromhex("0800000012340001")
    s = (~oracle.icmpv4_checksum(icmp)) & 0xFFFF
    assert s.to_bytes(2, "little") == bytes.fromhex("e5ca")
    icmp2 = icmp[:2] + s.to_bytes(2, "little") + icmp[4:]
    assert oracle.icmpv4_checksum(icmp2) == 0xFFFF


def test_adversarial(oracle, golden):
    adv = golden.adversarial()
    for name, (kind, mode, use_seeds) in golden.ADV_CASES.items():
        got = oracle.batch(golden.adv_arena(adv, kind), adv["offsets"], adv["lengths"],
                           seeds=adv["seeds"] if use_seeds else None,
                           src=adv["src"], dst=adv["dst"], mode=mode, nthreads=4)
        np.testing.assert_array_equal(got, adv["expect_" + name], err_msg=name)


def test_generators_match_spec(oracle, golden):
    d = golden.digests()
    assert oracle.splitmix_bytes(8).tobytes().hex() == "51b4617a118d3a1f"
    # byte_off continuity: any window equals the slice of the stream
    full = oracle.splitmix_bytes(4096)
    for off in (0, 1, 7, 8, 9, 1000, 4000):
        np.testing.assert_array_equal(oracle.splitmix_bytes(64, byte_off=off)[: 4096 - off][:64],
                                      full[off:off + 64])
    z = oracle.zipf_lengths(65536)
    zl = d["zipf_lengths"]
    assert f"{oracle.fnv1a_u16(z):016x}" == zl["fnv1a64"]
    assert int(z.astype(np.int64).sum()) == zl["total"]
    assert [int(x) for x in z[:4]] == zl["first4"]
    assert int((z & 1).sum()) == zl["odd"]


@pytest.mark.parametrize("name", ["F1500", "F1500-tcp", "F9000", "F1500s2048", "F64",
                                  "ZIPF", "ZIPF-tcp"])
def test_batch_digests(oracle, golden, name):
    b = golden.digests()["batches"][name]
    n = b["n"]
    src = np.full(n, ip4(10, 1, 0, 1), dtype=np.uint32)
    dst = np.full(n, ip4(10, 1, 0, 2), dtype=np.uint32)
    mode = MODE_TCP if b["mode"] == "tcp" else MODE_RAW
    if name.startswith("ZIPF"):
        lens = oracle.zipf_lengths(n)
        offs = packed_offsets(lens)
        arena = oracle.splitmix_bytes(int(lens.astype(np.int64).sum()))
        out = oracle.batch(arena, offs, lens, src=src, dst=dst, mode=mode, nthreads=8)
    else:
        arena = oracle.splitmix_bytes(n * b["stride"])
        out = oracle.batch(arena, stride=b["stride"], fixed_len=b["length"], n=n,
                           src=src, dst=dst, mode=mode, nthreads=8)
    assert f"{oracle.fnv1a_u16(out):016x}" == b["fnv1a64"]
    assert int(out.astype(np.int64).sum()) == b["sum"]


@pytest.mark.slow
def test_m8_shard0_digest(oracle, golden):
    b = golden.digests()["batches"]["M8x1500"]
    shard_n = b["n"] // 8
    arena = oracle.splitmix_bytes(shard_n * 1500)
    out = oracle.batch(arena, stride=1500, fixed_len=1500, n=shard_n, nthreads=8)
    assert f"{oracle.fnv1a_u16(out):016x}" == b["shards"][0]["fnv1a64"]


def test_batch_rejects_bad_mode(oracle):
    with pytest.raises(ValueError):
        oracle.batch(np.zeros(16, np.uint8), stride=1, fixed_len=1, n=1, mode=7)


@pytest.mark.skipif(not Reference.available(), reason="oracle/_ref not built here")
def test_live_reference_fuzz(oracle):
    """Restatement == reference build on fresh random cases (build container)."""
    ref = Reference()
    rng = np.random.default_rng(20241220)
    arena = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    n = 20000
    lens = rng.integers(0, 9100, n).astype(np.uint16)
    lens[:100] = rng.integers(60000, 65536, 100)
    offs = np.array([rng.integers(0, len(arena) - int(L)) for L in lens], dtype=np.uint64)
    seeds = rng.integers(0, 65536, n, dtype=np.uint16)
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    for mode in (MODE_RAW, MODE_INET, MODE_TCP, MODE_TCP | FLAG_COMPLEMENT):
        a = oracle.batch(arena, offs, lens, seeds=seeds, src=src, dst=dst, mode=mode, nthreads=8)
        b = ref.batch(arena, offs, lens, seeds=seeds, src=src, dst=dst, mode=mode, nthreads=8)
        np.testing.assert_array_equal(a, b)
    for _ in range(200):
        L = int(rng.integers(0, 64))
        d = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        s = int(rng.integers(0, 65536))
        assert oracle.checksum(s, d) == ref.checksum(s, d)


@pytest.mark.skipif(not Reference.available(REF_CLANG_SO), reason="clang build of oracle/_ref absent")
def test_clang_reference_build_matches_golden(golden):
    """The clang build of the reference (bench.py's second CPU baseline) gives
    the reference's results: every known answer and the F1500 digest."""
    from oracle import Oracle
    ref, orc = Reference(REF_CLANG_SO), Oracle()
    for c in golden.kat():
        if c["fn"] == "checksum":
            d = golden.kat_data(c, orc)
            assert ref.checksum(c["seed"], d) == c["expect"], c
    arena = orc.splitmix_bytes(65536 * 1500)
    out = ref.batch(arena, stride=1500, fixed_len=1500, n=65536, nthreads=8)
    gold = golden.digests()["batches"]["F1500"]["fnv1a64"]
    assert f"{orc.fnv1a_u16(out):016x}" == gold
