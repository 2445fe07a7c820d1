"""CPU-side tests of the product library: it loads, exports every symbol the
headers declare (plus the reference's C++ symbols), validates arguments
without touching a GPU, and its host scalar drop-ins match the reference."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import tulips_amd
from tulips_amd import csum
from oracle import ip4

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRODUCT_H = os.path.join(ROOT, "include", "tulips_csum.h")
BENCH_H = os.path.join(ROOT, "include", "tulips_csum_bench.h")


def declared_functions(header=PRODUCT_H):
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(tulips_(?:csum|rss)_\w+)\s*\(", text)))


def exported(path):
    """Defined dynamic symbols of a shared library (binutils nm -D)."""
    import shutil
    import subprocess
    nm = shutil.which("nm")
    if nm is None:
        pytest.skip("nm not installed")
    out = subprocess.run([nm, "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    return sorted(line.split()[-1] for line in out.splitlines() if line.strip())


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 15, names
    for n in names:
        assert hasattr(csum.lib, n), f"{n} declared in include/ but not exported"
        assert n in csum._SIGNATURES, f"{n} has no ctypes signature"


def test_product_exports_exactly_the_header_and_reference_symbols():
    """The product .so exports include/tulips_csum.h and the reference's own
    C++ symbols (include/tulips/stack/Utils.h:10-11 & co.), nothing else:
    no measurement entry points, internal C++ or HIP registration symbols
    (tulips_amd/csrc/libtulips_csum.map)."""
    assert exported(csum.LIB_PATH) == sorted(declared_functions() + list(csum.CXX_SYMBOLS))


def test_bench_library_exports_exactly_its_header():
    import benchlib
    got = exported(benchlib.LIB_PATH)
    assert got == declared_functions(BENCH_H)
    assert not set(got) & set(exported(csum.LIB_PATH))


def test_reference_cxx_symbols_exported():
    for sym in csum.CXX_SYMBOLS:
        assert hasattr(csum.lib, sym), sym


def test_version_and_status_strings():
    assert "gfx950" in csum.version()
    assert csum.lib.tulips_csum_status_string(0) == b"Ok"
    assert csum.lib.tulips_csum_status_string(1) == b"InvalidArgument"
    assert csum.lib.tulips_csum_status_string(7) == b"Unknown"


def _kat_check(golden, oracle, fns):
    for c in golden.kat():
        data = golden.kat_data(c, oracle)
        got = fns[c["fn"]](c, data)
        assert got == c["expect"], c


def test_host_c_abi_matches_reference_kat(golden, oracle):
    _kat_check(golden, oracle, {
        "checksum": lambda c, d: tulips_amd.checksum(c["seed"], d),
        "ipv4": lambda c, d: tulips_amd.ipv4_checksum(d),
        "icmpv4": lambda c, d: tulips_amd.icmpv4_checksum(d),
        "tcp": lambda c, d: tulips_amd.tcp_checksum(c["src"], c["dst"], d),
    })


def test_host_cxx_symbols_match_reference_kat(golden, oracle):
    lib = csum.lib
    u8p = C.POINTER(C.c_uint8)
    a1 = getattr(lib, "_ZN6tulips5stack5utils8checksumEtPKht")
    a1.restype, a1.argtypes = C.c_uint16, [C.c_uint16, u8p, C.c_uint16]
    a5 = getattr(lib, "_ZN6tulips5stack4ipv48checksumEPKh")
    a5.restype, a5.argtypes = C.c_uint16, [u8p]
    a6 = getattr(lib, "_ZN6tulips5stack6icmpv48checksumEPKh")
    a6.restype, a6.argtypes = C.c_uint16, [u8p]
    # tcpv4::Processor::checksum (private static): Address const& -> pointer
    a2 = getattr(lib, "_ZN6tulips5stack5tcpv49Processor8checksumERKNS0_4ipv47AddressES6_tPKh")
    a2.restype = C.c_uint16
    a2.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_uint16, u8p]

    def buf(d):
        b = (C.c_uint8 * max(1, len(d))).from_buffer_copy(d or b"\0")
        return C.cast(b, u8p), b

    def call(f, *args, data):
        p, keep = buf(data)
        return f(*args[:-1], p, *args[-1:]) if args else f(p)

    seen_tcp = False
    for c in golden.kat():
        d = golden.kat_data(c, oracle)
        p, _k = buf(d)
        if c["fn"] == "checksum":
            assert a1(c["seed"], p, len(d)) == c["expect"], c
        elif c["fn"] == "ipv4":
            assert a5(p) == c["expect"], c
        elif c["fn"] == "icmpv4":
            assert a6(p) == c["expect"], c
        elif c["fn"] == "tcp":
            src, dst = C.c_uint32(c["src"]), C.c_uint32(c["dst"])
            assert a2(C.byref(src), C.byref(dst), len(d), p) == c["expect"], c
            seen_tcp = True
    assert seen_tcp


def test_host_scalar_fuzz_vs_oracle(oracle):
    rng = np.random.default_rng(7)
    for _ in range(3000):
        L = int(rng.integers(0, 200))
        d = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        if rng.random() < 0.1:
            d = bytes([0xFF]) * L
        s = int(rng.choice([0, 0xFFFF, rng.integers(0, 65536)]))
        assert tulips_amd.checksum(s, d) == oracle.checksum(s, d)
        a, b = int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32))
        assert tulips_amd.tcp_checksum(a, b, d) == oracle.tcp_checksum(a, b, d)


def test_host_scalar_len_bounds():
    with pytest.raises(ValueError):
        tulips_amd.checksum(0, b"\0" * 10, 11)
    with pytest.raises(ValueError):
        tulips_amd.ipv4_checksum(b"\0" * 19)


# -- argument validation: these calls return before any HIP API is used -----
def _vp(x):
    return C.c_void_p(x)


FAKE = 0x10000  # never dereferenced: validation fails first


def test_batch_validation_without_gpu():
    lib = csum.lib
    # n == 0 is a no-op
    assert lib.tulips_csum_batch(None, None, None, None, None, None, None, 0, 0, None) == 0
    assert lib.tulips_csum_batch_fixed(None, 0, 0, None, None, None, None, 0, 0, None) == 0
    # null base / arrays / out
    assert lib.tulips_csum_batch(None, FAKE, FAKE, None, None, None, FAKE, 4, 0, None) == 1
    assert lib.tulips_csum_batch(FAKE, None, FAKE, None, None, None, FAKE, 4, 0, None) == 1
    assert lib.tulips_csum_batch(FAKE, FAKE, FAKE, None, None, None, None, 4, 0, None) == 1
    # TCP needs addresses
    assert lib.tulips_csum_batch(FAKE, FAKE, FAKE, None, None, None, FAKE, 4, 2, None) == 1
    assert lib.tulips_csum_batch(FAKE, FAKE, FAKE, None, FAKE, None, FAKE, 4, 2, None) == 1
    # unknown mode / flag bits
    assert lib.tulips_csum_batch(FAKE, FAKE, FAKE, None, None, None, FAKE, 4, 3, None) == 1
    assert lib.tulips_csum_batch(FAKE, FAKE, FAKE, None, None, None, FAKE, 4, 0x200, None) == 1
    # segment longer than the reference's uint16 len
    assert lib.tulips_csum_batch_fixed(FAKE, 70000, 65536, None, None, None, FAKE, 4, 0, None) == 1
    # verify needs INET/TCP and a counter
    assert lib.tulips_csum_verify(FAKE, FAKE, FAKE, FAKE, FAKE, None, None, 4, 2, None) == 1
    assert lib.tulips_csum_verify(FAKE, FAKE, FAKE, FAKE, FAKE, None, FAKE, 4, 0, None) == 1
    # bad tuning
    t = csum.Tuning(group=48, unroll=4, nontemporal=0, max_blocks=0)
    assert lib.tulips_csum_batch_fixed_tuned(FAKE, 1500, 1500, None, None, None, FAKE, 4, 0,
                                             C.byref(t), None) == 1
    t = csum.Tuning(group=64, unroll=3, nontemporal=0, max_blocks=0)
    assert lib.tulips_csum_batch_tuned(FAKE, FAKE, FAKE, None, None, None, FAKE, 4, 0,
                                       C.byref(t), None) == 1
    # in-order arenas: same checks, plus the tuning must be SPAN/DEFAULT with a
    # known unroll and halo
    assert lib.tulips_csum_batch_arena(None, 0, None, None, None, None, None, None, 0, 0,
                                       None) == 0
    assert lib.tulips_csum_batch_arena(None, 16, FAKE, FAKE, None, None, None, FAKE, 4, 0,
                                       None) == 1
    assert lib.tulips_csum_batch_arena(FAKE, 16, FAKE, FAKE, None, None, None, None, 4, 0,
                                       None) == 1
    assert lib.tulips_csum_batch_arena(FAKE, 16, FAKE, FAKE, None, None, None, FAKE, 4, 2,
                                       None) == 1
    assert lib.tulips_csum_verify_arena(FAKE, 16, FAKE, FAKE, FAKE, FAKE, None, None, 4, 2,
                                        None) == 1
    assert lib.tulips_csum_verify_arena(FAKE, 16, FAKE, FAKE, None, None, None, FAKE, 4, 0,
                                        None) == 1
    for kind, unroll, halo in ((csum.KIND_PACKED, 4, 0), (csum.KIND_SPAN, 3, 0),
                               (csum.KIND_SPAN, 10, 1), (csum.KIND_SPAN, 5, 9), (csum.KIND_SPAN, 2, 0),
                               (csum.KIND_SPAN, 2, 4), (csum.KIND_SPAN, 9, 6),
                               (csum.KIND_SPAN, 13, 0), (csum.KIND_SPAN, 6, 6),
                               (csum.KIND_SPAN, 8, 2), (csum.KIND_SPAN, 6, 3)):
        t = csum.Tuning(kind=kind, unroll=unroll, group=halo)
        assert lib.tulips_csum_batch_arena_tuned(FAKE, 16, FAKE, FAKE, None, None, None, FAKE,
                                                 4, 0, C.byref(t), None) == 1, (kind, unroll)
    # host ctx
    assert lib.tulips_csum_ctx_create(0, 0, None) == 1
    assert lib.tulips_csum_ctx_destroy(None) == 1
    assert lib.tulips_csum_batch_host(None, FAKE, FAKE, FAKE, None, None, None, FAKE, 4, 0) == 1


def test_python_binding_raises_typed_errors():
    with pytest.raises(csum.InvalidArgument):
        csum._check(1, "x")
    with pytest.raises(csum.CsumError):
        csum._check(2, "x")


def test_default_tuning():
    t = csum.default_tuning(9000)
    assert t.group == 64
    t = csum.default_tuning(1500)
    assert (t.group, t.unroll) == (32, 3)      # 96 chunks: a 1500 B segment in one batch
    t = csum.default_tuning(0, variable=True)
    assert t.kind == csum.KIND_PACKED and t.group == 8 and t.unroll == 4 and t.sps == 2
    # packed geometries are for variable-length batches only; kinds 2 and 4
    # (hybrid, workgroup-balanced) live in tools/sessions/variants, not the library
    for kind in (2, 4, csum.KIND_PACKED):
        bad = csum.Tuning(kind=kind, group=16, unroll=4, nontemporal=1)
        assert csum.lib.tulips_csum_batch_fixed_tuned(FAKE, 1500, 1500, None, None, None,
                                                      FAKE, 4, 0, C.byref(bad), None) == 1
    for kind, g, u, s in ((2, 16, 2, 1), (2, 8, 4, 2), (4, 8, 4, 2),
                          (csum.KIND_PACKED, 8, 8, 2), (csum.KIND_PACKED, 5, 4, 2),
                          (csum.KIND_PACKED, 64, 4, 2), (csum.KIND_PACKED, 16, 4, 5),
                          (csum.KIND_PACKED, 8, 4, 1), (csum.KIND_PACKED, 8, 4, 3),
                          (csum.KIND_PACKED, 8, 4, 4), (csum.KIND_SUBGROUP, 8, 4, 0),
                          (csum.KIND_SUBGROUP, 16, 4, 2), (csum.KIND_SUBGROUP, 32, 5, 0),
                          (7, 16, 4, 0)):
        bad = csum.Tuning(kind=kind, group=g, unroll=u, nontemporal=1, sps=s)
        assert csum.lib.tulips_csum_batch_tuned(FAKE, FAKE, FAKE, None, None, None, FAKE, 4,
                                                0, C.byref(bad), None) == 1
    with pytest.raises(csum.InvalidArgument):
        csum.default_tuning(70000)


def test_missing_library_fails_loudly(tmp_path):
    """No CPU fallback: the package without its built .so refuses to import."""
    import shutil
    import subprocess
    import sys
    pkg = tmp_path / "tulips_amd"
    pkg.mkdir()
    for f in ("__init__.py", "csum.py", "shard.py"):
        shutil.copy(os.path.join(ROOT, "tulips_amd", f), pkg / f)
    r = subprocess.run([sys.executable, "-c", "import tulips_amd"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "no CPU fallback" in r.stderr


def test_crash_backtrace_names_native_frames(tmp_path):
    """tulips_csum_debug_crash_backtrace (benchlib; bench.py installs it): a SIGSEGV in
    native code prints the native call stack, then Python's faulthandler (the
    handler installed before) prints the interpreter's, and the process still
    dies of the signal."""
    import subprocess
    import sys
    prog = ("import faulthandler, sys, ctypes; faulthandler.enable(); "
            f"sys.path.insert(0, {ROOT!r}); import benchlib; "
            "assert benchlib.lib.tulips_csum_debug_crash_backtrace(1) == 0; "
            "assert benchlib.lib.tulips_csum_debug_crash_backtrace(2) == 1; "
            "ctypes.string_at(16)")
    r = subprocess.run([sys.executable, "-c", prog], capture_output=True, text=True,
                       timeout=300, cwd=tmp_path)
    assert r.returncode == -11, r.stderr[-2000:]
    assert "tulips_csum: fatal signal 11 (SIGSEGV) at address 0x0000000000000010" in r.stderr
    assert "native stack:" in r.stderr
    assert "Fatal Python error: Segmentation fault" in r.stderr   # faulthandler, chained


READELF = "/opt/rocm/llvm/bin/llvm-readelf"


@pytest.mark.skipif(not os.path.exists(READELF), reason="llvm-readelf not installed")
def test_no_kernel_spills_to_scratch(tmp_path):
    """Every gfx950 kernel in the library keeps its registers on chip: a
    scratch spill turns a bandwidth-bound kernel into a scratch-bound one
    (a frame geometry spilling 200 B per lane ran 4x slower,
    profiles/probe_frames_r03.txt). Reads the AMDGPU metadata of the code
    objects embedded in libtulips_csum.so (clang offload bundles); no GPU."""
    import struct
    import subprocess
    data = open(csum.LIB_PATH, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    objs, pos = [], 0
    while True:
        i = data.find(magic, pos)
        if i < 0:
            break
        n = struct.unpack_from("<Q", data, i + 24)[0]
        off = i + 32
        for _ in range(n):
            eo, es, ts = struct.unpack_from("<QQQ", data, off)
            off += 24
            triple = data[off:off + ts].decode()
            off += ts
            if "gfx950" in triple and es:
                objs.append(data[i + eo:i + eo + es])
        pos = i + len(magic)
    assert objs, "no gfx950 code object in the library"
    kernels, spilling = 0, []
    for k, co in enumerate(objs):
        p = tmp_path / f"co{k}.o"
        p.write_bytes(co)
        out = subprocess.run([READELF, "--notes", str(p)], capture_output=True, text=True,
                             check=True).stdout
        for block in out.split(".private_segment_fixed_size:")[1:]:
            kernels += 1
            size = int(block.split()[0])
            if size:
                name = re.search(r"\.name:\s+(\S+)", block)
                spilling.append((name.group(1) if name else "?", size))
    assert kernels >= 100, kernels
    assert not spilling, spilling


def test_bench_library_rejects_bad_arguments():
    """The measurement library's ceiling kernels (include/tulips_csum_bench.h)
    validate their arguments before any launch (no GPU call is made)."""
    import benchlib
    lib = benchlib.lib
    assert lib.tulips_csum_stream_read(FAKE + 1, 16, FAKE, 0, None) == 1
    assert lib.tulips_csum_stream_read_tiles(FAKE, 0, 4, FAKE, None) == 1
    assert lib.tulips_csum_stream_read_slots(FAKE, 2048, 0, 4, FAKE, None) == 1
    assert lib.tulips_csum_stream_read_slots(FAKE, 1000, 1514, 4, FAKE, None) == 1
    assert lib.tulips_csum_stream_read_slots(FAKE, 70000, 65536, 4, FAKE, None) == 1
    assert lib.tulips_csum_stream_read_slots(None, 2048, 1514, 0, None, None) == 0
    g = lib.tulips_csum_stream_read_slots_geom
    assert g(FAKE, 1500, 1500, 4, 32, 4, FAKE, None) == 1                 # geometry
    assert g(FAKE, 1500, 1500, 4, 64, 12, FAKE, None) == 1
    assert g(FAKE, 1000, 1500, 4, 32, 3, FAKE, None) == 1                 # slot < read
    assert g(None, 0, 0, 0, 32, 3, None, None) == 0                       # nothing to do
    cp = lib.tulips_csum_stream_copy_slots
    assert cp(FAKE, 65536, 0, 1460, 1514, 4, FAKE, 1536, None) == 1       # per_group 0
    assert cp(FAKE, 65536, 44, 1460, 0, 4, FAKE, 1536, None) == 1         # no bytes
    assert cp(FAKE, 65536, 44, 1460, 70000, 4, FAKE, 70016, None) == 1    # > 65535
    assert cp(FAKE, 65536, 44, 1460, 1514, 4, FAKE + 8, 1536, None) == 1  # misaligned out
    assert cp(FAKE, 65536, 44, 1460, 1514, 4, FAKE, 1528, None) == 1      # stride % 16
    assert cp(FAKE, 65536, 44, 1460, 1514, 4, FAKE, 1504, None) == 1      # stride < bytes
    assert cp(None, 65536, 44, 1460, 1514, 4, FAKE, 1536, None) == 1
    assert cp(None, 0, 0, 0, 0, 0, None, 0, None) == 0                    # nothing to do
