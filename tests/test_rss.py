"""Toeplitz RSS hash: src/stack/Utils.cpp:86-133.

Pins: the reference's own KATs (tests/stack/utils.cpp:37,54), and
tests/golden/rss.npz (4096 random tuples x 10 keys x 2 inits, computed by the
reference build, keys of 4..52 bytes so that the short-key wrap-around quirk
of Utils.cpp:123-125 is exercised).
"""
import ctypes as C
import os

import numpy as np
import pytest

from oracle import ip4

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rss.npz")


def rss_fixture():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def keys(fx):
    for i, name in enumerate(fx["key_names"]):
        yield i, str(name), fx[f"key_{i}"].tobytes()


def test_reference_kats_in_fixture():
    fx = rss_fixture()
    names = [str(x) for x in fx["key_names"]]
    i = names.index("dynamic40")
    assert int(fx[f"expect_{i}_init0"][0]) == 0xD90A078C     # tests/stack/utils.cpp:37
    i = names.index("static40")
    assert int(fx[f"expect_{i}_initff"][0]) == 0x108AD839    # tests/stack/utils.cpp:54
    assert int(fx["saddr"][0]) == ip4(10, 1, 0, 1) and int(fx["sport"][0]) == 8888


def test_oracle_matches_reference_fixture(oracle):
    fx = rss_fixture()
    for i, name, key in keys(fx):
        for init, tag in ((0, "init0"), (0xFFFFFFFF, "initff")):
            exp = fx[f"expect_{i}_{tag}"]
            for j in range(0, len(exp), 37):          # a sample per key
                got = oracle.toeplitz(int(fx["saddr"][j]), int(fx["daddr"][j]),
                                      int(fx["sport"][j]), int(fx["dport"][j]), key, init)
                assert got == int(exp[j]), (name, tag, j)


def test_host_dropin_matches_reference_fixture():
    from tulips_amd import csum
    fx = rss_fixture()
    for i, name, key in keys(fx):
        for init, tag in ((0, "init0"), (0xFFFFFFFF, "initff")):
            exp = fx[f"expect_{i}_{tag}"]
            for j in range(0, len(exp), 11):
                got = csum.toeplitz(int(fx["saddr"][j]), int(fx["daddr"][j]),
                                    int(fx["sport"][j]), int(fx["dport"][j]), key, init)
                assert got == int(exp[j]), (name, tag, j)


def test_cxx_symbol_matches_reference():
    """The exported tulips::stack::utils::toeplitz, called with pointers to the
    4-byte address words, as the reference's call sites pass them."""
    from tulips_amd import csum
    f = getattr(csum.lib, "_ZN6tulips5stack5utils8toeplitzERKNS0_4ipv47AddressES5_ttmPKhj")
    f.restype = C.c_uint32
    f.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_uint16, C.c_uint16,
                  C.c_size_t, C.POINTER(C.c_uint8), C.c_uint32]
    fx = rss_fixture()
    for i, name, key in keys(fx):
        kb = (C.c_uint8 * len(key)).from_buffer_copy(key)
        exp = fx[f"expect_{i}_initff"]
        for j in range(0, len(exp), 101):
            s, d = C.c_uint32(int(fx["saddr"][j])), C.c_uint32(int(fx["daddr"][j]))
            got = f(C.byref(s), C.byref(d), int(fx["sport"][j]), int(fx["dport"][j]),
                    len(key), C.cast(kb, C.POINTER(C.c_uint8)), 0xFFFFFFFF)
            assert got == int(exp[j]), (name, j)


def test_host_rejects_short_key():
    from tulips_amd import csum
    with pytest.raises(csum.InvalidArgument):
        csum.toeplitz(1, 2, 3, 4, b"\x01\x02\x03")
    assert csum.lib.tulips_rss_toeplitz_batch(None, None, None, None, 0, None, 0, 0, None,
                                              None) == 0
    assert csum.lib.tulips_rss_toeplitz_batch(0x1000, 0x1000, 0x1000, 0x1000, 4, None, 40,
                                              0, 0x1000, None) == 1


@pytest.mark.gpu
def test_gpu_batch_matches_reference_fixture():
    torch = pytest.importorskip("torch")
    from tulips_amd import csum
    fx = rss_fixture()
    dev = "cuda:0"
    t = {k: torch.from_numpy(np.array(fx[k], copy=True, order="C")).to(dev)
         for k in ("saddr", "daddr", "sport", "dport")}
    for i, name, key in keys(fx):
        for init, tag in ((0, "init0"), (0xFFFFFFFF, "initff")):
            out = csum.rss_batch(t["saddr"], t["daddr"], t["sport"], t["dport"], key, init)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            np.testing.assert_array_equal(got, fx[f"expect_{i}_{tag}"], err_msg=name)


@pytest.mark.gpu
def test_gpu_batch_large_vs_host():
    """4M tuples (16 grid-stride rounds per workgroup) against the host path."""
    torch = pytest.importorskip("torch")
    from tulips_amd import csum
    rng = np.random.default_rng(77)
    n = 1 << 22
    arrs = dict(saddr=rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32),
                daddr=rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32),
                sport=rng.integers(0, 65536, n, dtype=np.uint16),
                dport=rng.integers(0, 65536, n, dtype=np.uint16))
    key = rng.integers(0, 256, 40, dtype=np.uint8).tobytes()
    t = {k: torch.from_numpy(v).to("cuda:0") for k, v in arrs.items()}
    out = csum.rss_batch(t["saddr"], t["daddr"], t["sport"], t["dport"], key, 0x5A5A5A5A)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    for j in list(range(0, n, n // 512)) + [n - 1]:
        exp = csum.toeplitz(int(arrs["saddr"][j]), int(arrs["daddr"][j]),
                            int(arrs["sport"][j]), int(arrs["dport"][j]), key, 0x5A5A5A5A)
        assert int(got[j]) == exp, j


@pytest.mark.gpu
@pytest.mark.parametrize("n,shift", [(1, 0), (3, 0), (4097, 0), (4099, 1), (10001, 2)])
def test_gpu_batch_tails_and_alignment(n, shift):
    """The 4-tuples-per-thread path (aligned arrays, n / 4 vector groups plus
    an n % 4 tail) and the one-tuple path (arrays not 16-B aligned: views
    starting `shift` elements in), against the host path."""
    torch = pytest.importorskip("torch")
    from tulips_amd import csum
    rng = np.random.default_rng(n + shift)
    m = n + shift
    arrs = dict(saddr=rng.integers(0, 2**32, m, dtype=np.uint64).astype(np.uint32),
                daddr=rng.integers(0, 2**32, m, dtype=np.uint64).astype(np.uint32),
                sport=rng.integers(0, 65536, m, dtype=np.uint16),
                dport=rng.integers(0, 65536, m, dtype=np.uint16))
    key = rng.integers(0, 256, 52, dtype=np.uint8).tobytes()
    t = {k: torch.from_numpy(v).to("cuda:0")[shift:] for k, v in arrs.items()}
    out = csum.rss_batch(t["saddr"], t["daddr"], t["sport"], t["dport"], key, 0x1234567)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    for j in range(n):
        exp = csum.toeplitz(int(arrs["saddr"][shift + j]), int(arrs["daddr"][shift + j]),
                            int(arrs["sport"][shift + j]), int(arrs["dport"][shift + j]),
                            key, 0x1234567)
        assert int(got[j]) == exp, j
