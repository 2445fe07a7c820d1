"""transport::gpucsum::Device — the batched receive-validation decorator
(integration/include/tulips/transport/gpucsum/Device.h).

integration/_build/libgpucsum_test.so (integration/Makefile) is the decorator
compiled against the reference's headers, wrapping the reference's own
list::Device (src/transport/list/Device.cpp). The frames of
tests/golden/frames.npz are committed on a peer list device, polled through
the decorator, and the frames reaching the stack's Processor must be exactly
those whose reference-derived flags pass the VALIDATE_IP_CSUM /
VALIDATE_L4_CSUM hints, in arrival order (the drop rules of
src/transport/ofed/Device.cpp:528-545 and src/transport/ena/Device.cpp:316-340).
"""
import ctypes as C
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "integration", "_build", "libgpucsum_test.so")
GOLDEN = os.path.join(ROOT, "tests", "golden", "frames.npz")

VALIDATE_IP_CSUM, VALIDATE_L4_CSUM = 0x1, 0x2   # include/tulips/transport/Device.h:29-30

needs_harness = pytest.mark.skipif(not os.path.exists(HARNESS),
                                   reason="integration/_build not built (no reference tree)")


def harness():
    from tulips_amd import csum  # noqa: F401  (torch's HIP runtime first, then ours)
    lib = C.CDLL(HARNESS)
    f = lib.gpucsum_run
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint16,
                  C.c_int, C.c_void_p, C.c_void_p]
    return f


def fixture():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def expected_forwarded(flags, hints):
    f = flags.astype(np.int64)
    bad_ip = ((hints & VALIDATE_IP_CSUM) != 0) & ((f & 0x01) != 0) & ((f & 0x02) == 0)
    bad_l4 = ((hints & VALIDATE_L4_CSUM) != 0) & ((f & 0x04) != 0) & ((f & 0x08) == 0)
    bad_l4 &= ~bad_ip
    return (~(bad_ip | bad_l4)).astype(np.uint8), int(bad_ip.sum()), int(bad_l4.sum())


def run(fx, burst, hints, use_wait, n=None):
    f = harness()
    n = len(fx["offsets"]) if n is None else n
    arena = np.ascontiguousarray(fx["arena"])
    offs = np.ascontiguousarray(fx["offsets"][:n])
    lens = np.ascontiguousarray(fx["lengths"][:n])
    fwd = np.zeros(n, dtype=np.uint8)
    stats = np.zeros(5, dtype=np.uint64)
    rc = f(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, n, burst, hints,
           int(use_wait), fwd.ctypes.data, stats.ctypes.data)
    assert rc == 0, f"gpucsum_run rc={rc}"
    return fwd, stats


@needs_harness
def test_harness_exports():
    from tulips_amd import csum  # noqa: F401  (loading needs torch's runtime first)
    lib = C.CDLL(HARNESS)
    assert hasattr(lib, "gpucsum_run")
    # the decorator's vtable is in the library (C++ symbol of its poll override)
    assert hasattr(lib, "_ZN6tulips9transport7gpucsum6Device4pollERNS0_9ProcessorE")


@needs_harness
@pytest.mark.gpu
@pytest.mark.parametrize("hints", [3, 1, 2, 0])
@pytest.mark.parametrize("use_wait", [False, True])
def test_forwarded_frames_follow_hints(hints, use_wait):
    fx = fixture()
    fwd, st = run(fx, 256, hints, use_wait)
    exp, bad_ip, bad_l4 = expected_forwarded(fx["expect"], hints)
    np.testing.assert_array_equal(fwd, exp)
    n = len(exp)
    assert int(st[0]) == n and int(st[1]) == int(exp.sum())
    assert (int(st[2]), int(st[3])) == (bad_ip, bad_l4)
    assert int(st[4]) >= (n + 255) // 256


@needs_harness
@pytest.mark.gpu
@pytest.mark.parametrize("burst", [1, 7, 4096])
def test_burst_sizes(burst):
    fx = fixture()
    n = 600 if burst == 1 else None
    fwd, st = run(fx, burst, 3, False, n=n)
    exp, _, _ = expected_forwarded(fx["expect"][:len(fwd)], 3)
    np.testing.assert_array_equal(fwd, exp)
    if burst == 4096:
        assert int(st[4]) == 1          # the whole poll burst in one launch
