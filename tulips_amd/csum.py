"""Python binding of the MI355X checksum library (``libtulips_csum.so``).

The product is the C ABI in ``include/tulips_csum.h``; this module is the thin
ctypes layer tests and ``bench.py`` use to drive it. Device buffers are
passed as torch tensors on a ROCm device (PyTorch is the allocator/stream
plumbing here, nothing more) or as raw integer device addresses.

There is deliberately no CPU fallback: if the shared library is missing,
importing this module raises, and every batch call goes to the gfx950
kernels.

Names mirror the reference (xenogenics/tulips @ 2024-12-20):
  checksum(seed, data)          tulips::stack::utils::checksum   src/stack/Utils.cpp:14-42
  ipv4_checksum(header)         tulips::stack::ipv4::checksum    src/stack/IPv4.cpp:75-82
  icmpv4_checksum(header)       tulips::stack::icmpv4::checksum  src/stack/ICMPv4.cpp:10-15
  tcp_checksum(src, dst, seg)   tcpv4::Processor::checksum       src/stack/tcpv4/Processor.cpp:337-357
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libtulips_csum.so")

# include/tulips_csum.h
STATUS_OK = 0
STATUS_INVALID_ARGUMENT = 1
STATUS_HARDWARE_ERROR = 2
STATUS_NO_MORE_RESOURCES = 3
RAW, INET, TCP = 0, 1, 2
COMPLEMENT = 0x100
MAX_SEGMENT = 65535

_STATUS_NAMES = {0: "Ok", 1: "InvalidArgument", 2: "HardwareError",
                 3: "NoMoreResources", 18: "UnsupportedOperation"}


class CsumError(RuntimeError):
    """A non-Ok tulips::Status from the library."""

    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(f"{what}: {_STATUS_NAMES.get(status, status)}")


class InvalidArgument(CsumError, ValueError):
    pass


def _check(rc: int, what: str) -> None:
    if rc == STATUS_OK:
        return
    if rc == STATUS_INVALID_ARGUMENT:
        raise InvalidArgument(rc, what)
    detail = lib.tulips_csum_last_error().decode(errors="replace")
    raise CsumError(rc, f"{what} [{detail}]" if detail else what)


KIND_DEFAULT, KIND_SUBGROUP, KIND_PACKED = 0, 1, 3
KIND_SPAN = 5


class Tuning(C.Structure):
    """tulips_csum_tuning (include/tulips_csum.h).

    kind SUBGROUP: `group` lanes (16/32/64) per segment, `unroll` chunks per
    lane in flight; PACKED (variable only): one wave per `group` segments
    (8/16), their chunks packed end to end, `unroll` 64-chunk windows per
    double-buffered batch; SPAN (in-order arenas only): `unroll` 4..8 chunks
    per lane (4 KiB of arena per workgroup each). A positive `group` with
    kind left at DEFAULT means SUBGROUP.
    """
    _fields_ = [("kind", C.c_int32), ("group", C.c_int32), ("unroll", C.c_int32),
                ("nontemporal", C.c_int32), ("max_blocks", C.c_uint32),
                ("block", C.c_int32), ("sps", C.c_int32)]

    def __init__(self, group=0, unroll=0, nontemporal=-1, max_blocks=0, block=0,
                 kind=None, sps=0):
        if kind is None:
            kind = KIND_SUBGROUP if group else KIND_DEFAULT
        super().__init__(kind, group, unroll, nontemporal, max_blocks, block, sps)

    def __repr__(self):
        return (f"Tuning(kind={self.kind}, group={self.group}, unroll={self.unroll}, "
                f"nontemporal={self.nontemporal}, max_blocks={self.max_blocks}, "
                f"block={self.block}, sps={self.sps})")


_vp = C.c_void_p
_u8p = C.POINTER(C.c_uint8)

_SIGNATURES = {
    "tulips_csum_host": (C.c_uint16, [C.c_uint16, _u8p, C.c_uint16]),
    "tulips_csum_ipv4_host": (C.c_uint16, [_u8p]),
    "tulips_csum_icmpv4_host": (C.c_uint16, [_u8p]),
    "tulips_csum_tcp_host": (C.c_uint16, [C.c_uint32, C.c_uint32, C.c_uint16, _u8p]),
    "tulips_csum_batch": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                    C.c_uint32, C.c_uint32, _vp]),
    "tulips_csum_batch_fixed": (C.c_int, [_vp, C.c_uint64, C.c_uint32, _vp, _vp,
                                          _vp, _vp, C.c_uint32, C.c_uint32, _vp]),
    "tulips_csum_verify": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                     C.c_uint32, C.c_uint32, _vp]),
    "tulips_csum_batch_arena": (C.c_int, [_vp, C.c_uint64, _vp, _vp, _vp, _vp, _vp, _vp,
                                          C.c_uint32, C.c_uint32, _vp]),
    "tulips_csum_verify_arena": (C.c_int, [_vp, C.c_uint64, _vp, _vp, _vp, _vp, _vp, _vp,
                                           C.c_uint32, C.c_uint32, _vp]),
    "tulips_csum_batch_arena_tuned": (C.c_int, [_vp, C.c_uint64, _vp, _vp, _vp, _vp, _vp,
                                                _vp, C.c_uint32, C.c_uint32,
                                                C.POINTER(Tuning), _vp]),
    "tulips_csum_ctx_create": (C.c_int, [C.c_int, C.c_uint64, C.POINTER(_vp)]),
    "tulips_csum_ctx_destroy": (C.c_int, [_vp]),
    "tulips_csum_batch_host": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                         C.c_uint32, C.c_uint32]),
    "tulips_csum_status_string": (C.c_char_p, [C.c_int]),
    "tulips_csum_version": (C.c_char_p, []),
    "tulips_csum_last_error": (C.c_char_p, []),
    "tulips_csum_default_tuning": (C.c_int, [C.c_uint32, C.c_int, C.POINTER(Tuning)]),
    "tulips_csum_batch_fixed_tuned": (C.c_int, [_vp, C.c_uint64, C.c_uint32, _vp,
                                                _vp, _vp, _vp, C.c_uint32,
                                                C.c_uint32, C.POINTER(Tuning), _vp]),
    "tulips_csum_batch_tuned": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                          C.c_uint32, C.c_uint32,
                                          C.POINTER(Tuning), _vp]),
    "tulips_rss_toeplitz_host": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint16,
                                           _u8p, C.c_size_t, C.c_uint32,
                                           C.POINTER(C.c_uint32)]),
    "tulips_rss_toeplitz_batch": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint32, _u8p,
                                            C.c_size_t, C.c_uint32, _vp, _vp]),
    "tulips_csum_host_alloc": (C.c_int, [C.c_size_t, C.POINTER(_vp)]),
    "tulips_csum_host_free": (C.c_int, [_vp]),
    "tulips_csum_validate_frames": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, _vp, _vp]),
    "tulips_csum_generate_frames": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, _vp]),
    "tulips_csum_generate_fields": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, _vp, _vp]),
    "tulips_csum_segment_frames": (C.c_int, [_vp, _vp, _vp, C.c_uint32, C.c_uint32, _vp,
                                             C.c_uint64, C.c_uint32, _vp, _vp, _vp]),
    "tulips_csum_segment_frames_planned": (C.c_int, [_vp, _vp, _vp, C.c_uint32, C.c_uint32,
                                                     _vp, _vp, C.c_uint64, C.c_uint32, _vp,
                                                     _vp]),
    "tulips_csum_segment_plan_host": (C.c_int, [_vp, _vp, _vp, C.c_uint32, C.c_uint32, _vp]),
    "tulips_csum_frames_tuned": (C.c_int, [C.c_int, _vp, _vp, _vp, C.c_uint32, _vp, _vp,
                                           C.POINTER(Tuning), _vp]),
    "tulips_csum_validate_frames_host": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint32, _vp,
                                                   _vp]),
    "tulips_csum_release_stream": (C.c_int, [_vp]),
    "tulips_csum_shard_plan": (C.c_int, [_vp, C.c_uint32, C.c_uint32, _vp]),
    "tulips_csum_mctx_create": (C.c_int, [_vp, C.c_uint32, C.c_uint64, C.POINTER(_vp)]),
    "tulips_csum_mctx_destroy": (C.c_int, [_vp]),
    "tulips_csum_mctx_batch_host": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                              C.c_uint32, C.c_uint32]),
    "tulips_csum_mctx_validate_frames_host": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint32,
                                                        _vp, _vp]),
    "tulips_csum_mctx_shard_bounds": (C.c_int, [_vp, _vp]),
    "tulips_csum_mctx_validate_frames_rss_host": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint32,
                                                            _vp, C.c_size_t, C.c_uint32, _vp,
                                                            C.c_uint32, _vp, _vp, _vp]),
    "tulips_csum_mctx_batch_fixed_device": (C.c_int, [_vp, _vp, C.c_uint64, C.c_uint32, _vp,
                                                      _vp, _vp, _vp, C.c_uint32, C.c_uint32,
                                                      _vp]),
    "tulips_csum_mctx_batch_arena_device": (C.c_int, [_vp, _vp, C.c_uint64, _vp, _vp, _vp,
                                                      _vp, _vp, _vp, C.c_uint32, C.c_uint32,
                                                      _vp]),
    "tulips_csum_generate_frames_host": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint32, _vp]),
    "tulips_csum_validate_frames_zc": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint32, _vp, _vp]),
    "tulips_csum_ctx_set_lowlat": (C.c_int, [_vp, C.c_int]),
    "tulips_csum_segment_frames_host": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint32, C.c_uint32,
                                                  _vp, C.c_uint64, C.c_uint32, _vp, _vp]),
    "tulips_csum_validate_frames_cpu": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, _vp]),
    "tulips_csum_burst_prefers_cpu": (C.c_int, [C.c_uint32, C.c_uint64]),
    "tulips_csum_mctx_validate_frames_rss_device": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint32,
                                                              _vp, C.c_size_t, C.c_uint32,
                                                              _vp, C.c_uint32, _vp, _vp, _vp,
                                                              _vp]),
    "tulips_csum_mctx_set_peer_mode": (C.c_int, [_vp, C.c_int]),
}

# include/tulips_csum.h TULIPS_FRAME_* (per-frame validation flags)
FRAME_IPV4 = 0x01
FRAME_IP_CSUM_OK = 0x02
FRAME_TCP = 0x04
FRAME_L4_CSUM_OK = 0x08
FRAME_TRUNCATED = 0x10

# Exported C++ symbols of the reference surface (host scalar drop-ins).
CXX_SYMBOLS = (
    "_ZN6tulips5stack5utils8checksumEtPKht",
    "_ZN6tulips5stack4ipv48checksumEPKh",
    "_ZN6tulips5stack6icmpv48checksumEPKh",
    "_ZN6tulips5stack5tcpv49Processor8checksumERKNS0_4ipv47AddressES6_tPKh",
    "_ZN6tulips5stack5utils8toeplitzERKNS0_4ipv47AddressES5_ttmPKhj",
)


def _load():
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64
    # (SONAME libamdhip64.so.7, loaded via RPATH as "libamdhip64.so"). If our
    # library were loaded first it would pull /opt/rocm's copy and torch would
    # then load a second runtime, which finds no device. Importing torch
    # first makes our NEEDED libamdhip64.so.7 resolve to torch's copy.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make lib` or "
            "`python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


# ---------------------------------------------------------------------------
# host scalar drop-ins
# ---------------------------------------------------------------------------
def _buf(data: bytes):
    data = bytes(data)
    b = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    return C.cast(b, _u8p), b


def checksum(seed: int, data: bytes, length: int | None = None) -> int:
    """utils::checksum(seed, data, len) on the host (no GPU)."""
    length = len(data) if length is None else length
    if not 0 <= length <= MAX_SEGMENT or length > len(data):
        raise ValueError("length out of range")
    p, _keep = _buf(data)
    return lib.tulips_csum_host(seed & 0xFFFF, p, length)


def ipv4_checksum(header: bytes) -> int:
    if len(header) < 20:
        raise ValueError("IPv4 header is 20 bytes")
    p, _keep = _buf(header)
    return lib.tulips_csum_ipv4_host(p)


def icmpv4_checksum(header: bytes) -> int:
    if len(header) < 8:
        raise ValueError("ICMPv4 header is 8 bytes")
    p, _keep = _buf(header)
    return lib.tulips_csum_icmpv4_host(p)


def tcp_checksum(src: int, dst: int, segment: bytes, length: int | None = None) -> int:
    length = len(segment) if length is None else length
    if not 0 <= length <= MAX_SEGMENT or length > len(segment):
        raise ValueError("length out of range")
    p, _keep = _buf(segment)
    return lib.tulips_csum_tcp_host(src, dst, length, p)


# ---------------------------------------------------------------------------
# device batches
# ---------------------------------------------------------------------------
def _addr(x) -> int | None:
    """Device address of a torch tensor (or pass-through int / None)."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if not x.is_cuda:
        raise ValueError("device batch arguments must be ROCm device tensors")
    if not x.is_contiguous():
        raise ValueError("device tensors must be contiguous")
    return x.data_ptr()


def _stream(stream) -> int | None:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def _check_sizes(n: int, **arrays) -> None:
    for name, a in arrays.items():
        if a is not None and not isinstance(a, int) and int(a.numel()) < n:
            raise ValueError(f"{name} holds {int(a.numel())} entries, batch has {n}")


def _alloc_out(n: int, like):
    import torch
    return torch.empty(n, dtype=torch.uint16, device=like.device)


def batch(arena, offsets, lengths, *, seeds=None, src=None, dst=None,
          mode: int = RAW, out=None, stream=None, tuning: Tuning | None = None):
    """Checksum segment i = arena[offsets[i] : offsets[i] + lengths[i]].

    arena: uint8 device tensor; offsets: uint64/int64; lengths: uint16;
    seeds: uint16 (RAW/INET); src/dst: uint32/int32 address words (TCP).
    Returns the uint16 result tensor (enqueued on `stream`).
    """
    n = int(offsets.numel())
    if int(lengths.numel()) != n:
        raise ValueError("offsets/lengths size mismatch")
    _check_sizes(n, seeds=seeds, src=src, dst=dst, out=out)
    if out is None:
        out = _alloc_out(n, arena)
    args = (_addr(arena), _addr(offsets), _addr(lengths), _addr(seeds),
            _addr(src), _addr(dst), _addr(out), n, mode)
    if tuning is None:
        rc = lib.tulips_csum_batch(*args, _stream(stream))
    else:
        rc = lib.tulips_csum_batch_tuned(*args, C.byref(tuning), _stream(stream))
    _check(rc, "tulips_csum_batch")
    return out


def _arena_bytes(arena, arena_bytes):
    if arena_bytes is not None:
        return int(arena_bytes)
    if isinstance(arena, int):
        raise ValueError("arena_bytes is required with a raw arena address")
    return int(arena.numel()) * arena.element_size()


def batch_arena(arena, offsets, lengths, *, arena_bytes=None, seeds=None, src=None,
                dst=None, mode: int = RAW, out=None, stream=None,
                tuning: Tuning | None = None):
    """batch() for an in-order arena: offsets[i] + lengths[i] <= offsets[i+1],
    all segments inside arena[:arena_bytes] (default: the whole tensor)."""
    n = int(offsets.numel())
    if int(lengths.numel()) != n:
        raise ValueError("offsets/lengths size mismatch")
    _check_sizes(n, seeds=seeds, src=src, dst=dst, out=out)
    if out is None:
        out = _alloc_out(n, offsets)
    args = (_addr(arena), _arena_bytes(arena, arena_bytes), _addr(offsets), _addr(lengths),
            _addr(seeds), _addr(src), _addr(dst), _addr(out), n, mode)
    if tuning is None:
        rc = lib.tulips_csum_batch_arena(*args, _stream(stream))
    else:
        rc = lib.tulips_csum_batch_arena_tuned(*args, C.byref(tuning), _stream(stream))
    _check(rc, "tulips_csum_batch_arena")
    return out


def verify_arena(arena, offsets, lengths, *, arena_bytes=None, src=None, dst=None,
                 mode: int = TCP, out=None, bad=None, stream=None):
    """verify() for an in-order arena (see batch_arena)."""
    import torch
    n = int(offsets.numel())
    if bad is None:
        bad = torch.zeros(1, dtype=torch.int32, device=offsets.device)
    rc = lib.tulips_csum_verify_arena(_addr(arena), _arena_bytes(arena, arena_bytes),
                                      _addr(offsets), _addr(lengths), _addr(src),
                                      _addr(dst), _addr(out), _addr(bad), n, mode,
                                      _stream(stream))
    _check(rc, "tulips_csum_verify_arena")
    return bad


def batch_fixed(arena, stride: int, length: int, n: int, *, seeds=None,
                src=None, dst=None, mode: int = RAW, out=None, stream=None,
                tuning: Tuning | None = None, base_offset: int = 0):
    """Checksum segment i = arena[base_offset + i*stride :][:length]."""
    _check_sizes(n, seeds=seeds, src=src, dst=dst, out=out)
    if n and not isinstance(arena, int):
        end = base_offset + (n - 1) * stride + length
        if end > arena.numel() * arena.element_size():
            raise ValueError(f"segments end at byte {end}, past the arena")
    if out is None:
        out = _alloc_out(n, arena)
    base = _addr(arena) + base_offset
    args = (base, stride, length, _addr(seeds), _addr(src), _addr(dst),
            _addr(out), n, mode)
    if tuning is None:
        rc = lib.tulips_csum_batch_fixed(*args, _stream(stream))
    else:
        rc = lib.tulips_csum_batch_fixed_tuned(*args, C.byref(tuning), _stream(stream))
    _check(rc, "tulips_csum_batch_fixed")
    return out


def verify(arena, offsets, lengths, *, src=None, dst=None, mode: int = TCP,
           out=None, bad=None, stream=None):
    """Count segments whose INET/TCP result is not 0xffff; returns the uint32
    device counter (and fills `out` when given)."""
    import torch
    n = int(offsets.numel())
    if bad is None:
        bad = torch.zeros(1, dtype=torch.int32, device=arena.device)
    rc = lib.tulips_csum_verify(_addr(arena), _addr(offsets), _addr(lengths),
                                _addr(src), _addr(dst), _addr(out), _addr(bad),
                                n, mode, _stream(stream))
    _check(rc, "tulips_csum_verify")
    return bad


def default_tuning(fixed_length: int = 0, variable: bool = False) -> Tuning:
    t = Tuning()
    _check(lib.tulips_csum_default_tuning(fixed_length, int(variable), C.byref(t)),
           "tulips_csum_default_tuning")
    return t


@dataclass
class _Arr:
    ptr: int | None
    keep: object = None


def _host(a, dtype):
    import numpy as np
    if a is None:
        return _Arr(None)
    a = np.ascontiguousarray(a, dtype=dtype)
    return _Arr(a.ctypes.data, a)


class HostContext:
    """tulips_csum_ctx: host-resident batches through pinned staging."""

    def __init__(self, device: int = 0, chunk_bytes: int = 0):
        h = C.c_void_p()
        _check(lib.tulips_csum_ctx_create(device, chunk_bytes, C.byref(h)),
               "tulips_csum_ctx_create")
        self._h = h

    def close(self):
        if self._h:
            lib.tulips_csum_ctx_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def batch(self, arena, offsets, lengths, *, seeds=None, src=None, dst=None,
              mode: int = RAW, out=None):
        import numpy as np
        ar = arena if isinstance(arena, int) else _host(arena, np.uint8)
        base = ar if isinstance(ar, int) else ar.ptr
        off = _host(offsets, np.uint64)
        ln = _host(lengths, np.uint16)
        n = len(off.keep)
        if out is None:
            out = np.empty(n, dtype=np.uint16)
        sd, s, d = _host(seeds, np.uint16), _host(src, np.uint32), _host(dst, np.uint32)
        rc = lib.tulips_csum_batch_host(self._h, base, off.ptr, ln.ptr, sd.ptr,
                                        s.ptr, d.ptr, out.ctypes.data, n, mode)
        _check(rc, "tulips_csum_batch_host")
        return out

    def validate_frames(self, arena, offsets, lengths, *, flags=None,
                        with_counters: bool = False, low_latency: bool = False):
        """Host-resident frames -> uint8 FRAME_* flags (and the 4 counters).
        low_latency: tulips_csum_validate_frames_zc (resident server, frames
        read in place when page-locked)."""
        import numpy as np
        ar = arena if isinstance(arena, int) else _host(arena, np.uint8)
        base = ar if isinstance(ar, int) else ar.ptr
        off = _host(offsets, np.uint64)
        ln = _host(lengths, np.uint16)
        n = len(off.keep)
        if len(ln.keep) != n:
            raise ValueError("offsets/lengths size mismatch")
        if flags is None:
            flags = np.empty(n, dtype=np.uint8)
        cnt = np.zeros(4, dtype=np.uint32)
        fn = lib.tulips_csum_validate_frames_zc if low_latency else \
            lib.tulips_csum_validate_frames_host
        rc = fn(self._h, base, off.ptr, ln.ptr, n, flags.ctypes.data,
                cnt.ctypes.data if with_counters else None)
        _check(rc, "tulips_csum_validate_frames_zc" if low_latency else
               "tulips_csum_validate_frames_host")
        return (flags, cnt) if with_counters else flags

    def set_lowlat(self, resident: bool):
        """Low-latency path form: one launch per burst (False) or a resident
        server (True), tulips_csum_ctx_set_lowlat."""
        _check(lib.tulips_csum_ctx_set_lowlat(self._h, 1 if resident else 0),
               "tulips_csum_ctx_set_lowlat")

    def generate_frames(self, arena, offsets, lengths):
        """Write both checksum fields of host frames in `arena` (a writable
        uint8 numpy array) in place; returns the FRAME_* flags of what was
        written."""
        import numpy as np
        if not (isinstance(arena, np.ndarray) and arena.dtype == np.uint8 and
                arena.flags.c_contiguous and arena.flags.writeable):
            raise ValueError("arena must be a writable contiguous uint8 array")
        off = _host(offsets, np.uint64)
        ln = _host(lengths, np.uint16)
        n = len(off.keep)
        if len(ln.keep) != n:
            raise ValueError("offsets/lengths size mismatch")
        flags = np.empty(n, dtype=np.uint8)
        _check(lib.tulips_csum_generate_frames_host(self._h, arena.ctypes.data, off.ptr,
                                                    ln.ptr, n, flags.ctypes.data),
               "tulips_csum_generate_frames_host")
        return flags

    def segment_frames(self, arena, offsets, lengths, mss: int, *, stride: int = 2048,
                       capacity: int | None = None):
        """Host super-frames -> (out bytes, out_lengths, first)."""
        import numpy as np
        ar = _host(arena, np.uint8)
        off = _host(offsets, np.uint64)
        ln = _host(lengths, np.uint16)
        n = len(off.keep)
        first = np.zeros(n + 1, dtype=np.uint32)
        if capacity is None:
            _check(lib.tulips_csum_segment_frames_host(self._h, ar.ptr, off.ptr, ln.ptr, n,
                                                       mss, None, stride, 0, None,
                                                       first.ctypes.data),
                   "tulips_csum_segment_frames_host")
            capacity = int(first[n])
        out = np.zeros(max(capacity, 1) * stride, dtype=np.uint8)
        olen = np.zeros(max(capacity, 1), dtype=np.uint16)
        _check(lib.tulips_csum_segment_frames_host(self._h, ar.ptr, off.ptr, ln.ptr, n, mss,
                                                   out.ctypes.data, stride, capacity,
                                                   olen.ctypes.data, first.ctypes.data),
               "tulips_csum_segment_frames_host")
        return out, olen[:capacity], first


def shard_plan(lengths, nshards: int):
    """Byte-balanced contiguous shard bounds (tulips_csum_shard_plan)."""
    import numpy as np
    ln = _host(lengths, np.uint16)
    n = len(ln.keep)
    bounds = np.zeros(nshards + 1, dtype=np.uint32)
    _check(lib.tulips_csum_shard_plan(ln.ptr, n, nshards, bounds.ctypes.data),
           "tulips_csum_shard_plan")
    return bounds


class MultiContext(HostContext):
    """tulips_csum_mctx: host-resident batches split byte-balanced over
    several devices (a device may repeat)."""

    def __init__(self, devices, chunk_bytes: int = 0):
        import numpy as np
        devs = np.ascontiguousarray(devices, dtype=np.int32)
        h = C.c_void_p()
        _check(lib.tulips_csum_mctx_create(devs.ctypes.data, len(devs), chunk_bytes,
                                           C.byref(h)), "tulips_csum_mctx_create")
        self._h = h
        self.ndev = len(devs)

    def close(self):
        if self._h:
            lib.tulips_csum_mctx_destroy(self._h)
            self._h = None

    def set_peer_mode(self, staged: bool):
        """Device-resident calls: move pieces by peer DMA where the devices
        allow it (False, the default) or always through page-locked host
        bounce buffers (True), tulips_csum_mctx_set_peer_mode."""
        _check(lib.tulips_csum_mctx_set_peer_mode(self._h, 1 if staged else 0),
               "tulips_csum_mctx_set_peer_mode")

    def bounds(self):
        import numpy as np
        b = np.zeros(self.ndev + 1, dtype=np.uint32)
        _check(lib.tulips_csum_mctx_shard_bounds(self._h, b.ctypes.data), "shard_bounds")
        return b

    def batch(self, arena, offsets, lengths, *, seeds=None, src=None, dst=None,
              mode: int = RAW, out=None):
        import numpy as np
        ar = arena if isinstance(arena, int) else _host(arena, np.uint8)
        base = ar if isinstance(ar, int) else ar.ptr
        off = _host(offsets, np.uint64)
        ln = _host(lengths, np.uint16)
        n = len(off.keep)
        if out is None:
            out = np.empty(n, dtype=np.uint16)
        sd, s, d = _host(seeds, np.uint16), _host(src, np.uint32), _host(dst, np.uint32)
        _check(lib.tulips_csum_mctx_batch_host(self._h, base, off.ptr, ln.ptr, sd.ptr, s.ptr,
                                               d.ptr, out.ctypes.data, n, mode),
               "tulips_csum_mctx_batch_host")
        return out

    def validate_frames(self, arena, offsets, lengths, *, flags=None,
                        with_counters: bool = False):
        import numpy as np
        ar = arena if isinstance(arena, int) else _host(arena, np.uint8)
        base = ar if isinstance(ar, int) else ar.ptr
        off = _host(offsets, np.uint64)
        ln = _host(lengths, np.uint16)
        n = len(off.keep)
        if flags is None:
            flags = np.empty(n, dtype=np.uint8)
        cnt = np.zeros(4, dtype=np.uint32)
        _check(lib.tulips_csum_mctx_validate_frames_host(
            self._h, base, off.ptr, ln.ptr, n, flags.ctypes.data,
            cnt.ctypes.data if with_counters else None),
            "tulips_csum_mctx_validate_frames_host")
        return (flags, cnt) if with_counters else flags

    def validate_frames_rss(self, arena, offsets, lengths, key: bytes, table, *,
                            init: int = 0, with_counters: bool = False):
        """Flow-affine validation (tulips_csum_mctx_validate_frames_rss_host):
        each TCP frame validated on device table[toeplitz(tuple) % len(table)].
        Returns (flags, device_of[, counters])."""
        import numpy as np
        ar = arena if isinstance(arena, int) else _host(arena, np.uint8)
        base = ar if isinstance(ar, int) else ar.ptr
        off = _host(offsets, np.uint64)
        ln = _host(lengths, np.uint16)
        n = len(off.keep)
        tb = np.ascontiguousarray(table, dtype=np.uint16)
        kp, _keep = _buf(key)
        flags = np.empty(n, dtype=np.uint8)
        dev = np.empty(n, dtype=np.uint16)
        cnt = np.zeros(4, dtype=np.uint32)
        _check(lib.tulips_csum_mctx_validate_frames_rss_host(
            self._h, base, off.ptr, ln.ptr, n, kp, len(key), init & 0xFFFFFFFF,
            tb.ctypes.data, len(tb), flags.ctypes.data,
            cnt.ctypes.data if with_counters else None, dev.ctypes.data),
            "tulips_csum_mctx_validate_frames_rss_host")
        return (flags, dev, cnt) if with_counters else (flags, dev)

    def validate_frames_rss_device(self, arena, offsets, lengths, key: bytes, table, *,
                                   init: int = 0, counters=None, want_device_of: bool = True,
                                   stream=None):
        """Flow-affine validation of frames resident on `stream`'s device
        (tulips_csum_mctx_validate_frames_rss_device). Returns (flags,
        device_of) device tensors; `counters` (int32[4] device tensor) is
        zeroed and filled when given."""
        import numpy as np
        import torch
        n = int(offsets.numel())
        if int(lengths.numel()) != n:
            raise ValueError("offsets/lengths size mismatch")
        dev = offsets.device
        flags = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        devof = torch.empty(max(n, 1), dtype=torch.int16, device=dev) if want_device_of else None
        if counters is not None and int(counters.numel()) < 4:
            raise ValueError("counters needs 4 entries")
        tb = np.ascontiguousarray(table, dtype=np.uint16)
        kp, _keep = _buf(key)
        _check(lib.tulips_csum_mctx_validate_frames_rss_device(
            self._h, _addr(arena), _addr(offsets), _addr(lengths), n, kp, len(key),
            init & 0xFFFFFFFF, tb.ctypes.data, len(tb), _addr(flags), _addr(counters),
            _addr(devof), _stream(stream)), "tulips_csum_mctx_validate_frames_rss_device")
        return flags[:n], (devof[:n] if devof is not None else None)

    def batch_fixed_device(self, arena, stride: int, length: int, n: int, *, seeds=None,
                           src=None, dst=None, mode: int = RAW, out=None, stream=None,
                           base_offset: int = 0):
        """Device-resident fixed-stride batch on `stream`'s device, spread
        over the context's devices (tulips_csum_mctx_batch_fixed_device)."""
        _check_sizes(n, seeds=seeds, src=src, dst=dst, out=out)
        if out is None:
            out = _alloc_out(n, arena)
        _check(lib.tulips_csum_mctx_batch_fixed_device(
            self._h, _addr(arena) + base_offset, stride, length, _addr(seeds), _addr(src),
            _addr(dst), _addr(out), n, mode, _stream(stream)),
            "tulips_csum_mctx_batch_fixed_device")
        return out

    def batch_arena_device(self, arena, offsets, lengths, *, arena_bytes=None, seeds=None,
                           src=None, dst=None, mode: int = RAW, out=None, stream=None):
        """Device-resident in-order arena on `stream`'s device, spread over the
        context's devices (tulips_csum_mctx_batch_arena_device)."""
        n = int(offsets.numel())
        if int(lengths.numel()) != n:
            raise ValueError("offsets/lengths size mismatch")
        _check_sizes(n, seeds=seeds, src=src, dst=dst, out=out)
        if out is None:
            out = _alloc_out(n, offsets)
        _check(lib.tulips_csum_mctx_batch_arena_device(
            self._h, _addr(arena), _arena_bytes(arena, arena_bytes), _addr(offsets),
            _addr(lengths), _addr(seeds), _addr(src), _addr(dst), _addr(out), n, mode,
            _stream(stream)), "tulips_csum_mctx_batch_arena_device")
        return out

    def generate_frames(self, *a, **k):
        raise NotImplementedError("use HostContext for generation")

    def segment_frames(self, *a, **k):
        raise NotImplementedError("use HostContext for segmentation")


def toeplitz(saddr: int, daddr: int, sport: int, dport: int, key: bytes,
             init: int = 0) -> int:
    """utils::toeplitz (src/stack/Utils.cpp:86-133) on the host."""
    p, _keep = _buf(key)
    out = C.c_uint32()
    _check(lib.tulips_rss_toeplitz_host(saddr, daddr, sport, dport, p, len(key),
                                        init & 0xFFFFFFFF, C.byref(out)),
           "tulips_rss_toeplitz_host")
    return out.value


def rss_batch(saddr, daddr, sport, dport, key: bytes, init: int = 0, out=None,
              stream=None):
    """Toeplitz hashes of n device-resident tuples (uint32 addresses as
    ipv4::Address::m_data words, uint16 host-order ports) -> uint32 tensor."""
    import torch
    n = int(saddr.numel())
    _check_sizes(n, daddr=daddr, sport=sport, dport=dport, out=out)
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=saddr.device)
    p, _keep = _buf(key)
    _check(lib.tulips_rss_toeplitz_batch(_addr(saddr), _addr(daddr), _addr(sport),
                                         _addr(dport), n, p, len(key), init & 0xFFFFFFFF,
                                         _addr(out), _stream(stream)),
           "tulips_rss_toeplitz_batch")
    return out


def validate_frames(arena, offsets, lengths, *, flags=None, counters=None,
                    want_flags: bool = True, stream=None):
    """Validate Ethernet/IPv4/TCP frames arena[offsets[i]:][:lengths[i]].

    Returns the uint8 FRAME_* flags tensor (None when want_flags is False and
    no `flags` is given); `counters` (int32[4] device tensor, zeroed by the
    call) receives {IPv4, bad IP checksum, TCP, TCP without L4_CSUM_OK}.
    """
    import torch
    n = int(offsets.numel())
    if int(lengths.numel()) != n:
        raise ValueError("offsets/lengths size mismatch")
    _check_sizes(n, flags=flags)
    if flags is None and want_flags:
        flags = torch.empty(n, dtype=torch.uint8, device=arena.device)
    if counters is not None and int(counters.numel()) < 4:
        raise ValueError("counters needs 4 entries")
    _check(lib.tulips_csum_validate_frames(_addr(arena), _addr(offsets), _addr(lengths),
                                           n, _addr(flags), _addr(counters),
                                           _stream(stream)),
           "tulips_csum_validate_frames")
    return flags


def validate_frames_cpu(arena, offsets, lengths, *, with_counters: bool = False):
    """Host-resident frames validated on this thread by the library's host
    code (tulips_csum_validate_frames_cpu; no GPU): the same FRAME_* flags
    (and counters) as validate_frames."""
    import numpy as np
    ar = _host(arena, np.uint8)
    off = _host(offsets, np.uint64)
    ln = _host(lengths, np.uint16)
    n = len(off.keep)
    if len(ln.keep) != n:
        raise ValueError("offsets/lengths size mismatch")
    flags = np.empty(max(n, 1), dtype=np.uint8)
    cnt = np.zeros(4, dtype=np.uint32)
    _check(lib.tulips_csum_validate_frames_cpu(ar.ptr, off.ptr, ln.ptr, n, flags.ctypes.data,
                                               cnt.ctypes.data),
           "tulips_csum_validate_frames_cpu")
    return (flags[:n], cnt) if with_counters else flags[:n]


def generate_frames(arena, offsets, lengths, *, flags=None, want_flags: bool = True,
                    stream=None):
    """Write the IPv4 and TCP checksum fields of frames in `arena` in place
    (ipv4/Producer.cpp:79-82, tcpv4/Send.cpp:441-449). Returns the uint8
    FRAME_* flags of what was written (None when want_flags is False)."""
    import torch
    n = int(offsets.numel())
    if int(lengths.numel()) != n:
        raise ValueError("offsets/lengths size mismatch")
    _check_sizes(n, flags=flags)
    if flags is None and want_flags:
        flags = torch.empty(n, dtype=torch.uint8, device=arena.device)
    _check(lib.tulips_csum_generate_frames(_addr(arena), _addr(offsets), _addr(lengths), n,
                                           _addr(flags), _stream(stream)),
           "tulips_csum_generate_frames")
    return flags


def generate_fields(arena, offsets, lengths, *, fields=None, flags=None,
                    want_flags: bool = True, stream=None):
    """The two checksum field values generate_frames would write, returned
    as uint32 per frame (IPv4 field low 16 bits, TCP field high; each the
    uint16 a little-endian load of the header word gives); the frames are
    only read. Returns (fields, flags)."""
    import torch
    n = int(offsets.numel())
    if int(lengths.numel()) != n:
        raise ValueError("offsets/lengths size mismatch")
    _check_sizes(n, fields=fields, flags=flags)
    if fields is None:
        fields = torch.empty(n, dtype=torch.int32, device=arena.device)
    if flags is None and want_flags:
        flags = torch.empty(n, dtype=torch.uint8, device=arena.device)
    _check(lib.tulips_csum_generate_fields(_addr(arena), _addr(offsets), _addr(lengths), n,
                                           _addr(fields), _addr(flags), _stream(stream)),
           "tulips_csum_generate_fields")
    return fields, flags


def segment_frames(arena, offsets, lengths, mss: int, *, stride: int = 2048,
                   out=None, out_lengths=None, capacity: int | None = None, stream=None):
    """Segmentation offload of device-resident frames.

    Returns (out, out_lengths, first): `first` (int32[n+1]) is the exclusive
    prefix sum of the per-frame segment counts. Without `out` the function
    sizes it itself (one synchronising read of first[n]); segment j occupies
    out[j*stride:][:out_lengths[j]].
    """
    import torch
    n = int(offsets.numel())
    if int(lengths.numel()) != n:
        raise ValueError("offsets/lengths size mismatch")
    dev = arena.device
    first = torch.empty(n + 1, dtype=torch.int32, device=dev)
    st = _stream(stream)
    if out is None:
        _check(lib.tulips_csum_segment_frames(_addr(arena), _addr(offsets), _addr(lengths), n,
                                              mss, None, stride, 0, None, _addr(first), st),
               "tulips_csum_segment_frames")
        total = int(first[n].item())
        out = torch.empty(max(total, 1) * stride, dtype=torch.uint8, device=dev)
        capacity = total
    elif capacity is None:
        capacity = int(out.numel()) // stride
    if out_lengths is None:
        out_lengths = torch.zeros(max(capacity, 1), dtype=torch.int16, device=dev)
    if int(out_lengths.numel()) < capacity or int(out.numel()) < capacity * stride:
        raise ValueError("output smaller than its capacity")
    _check(lib.tulips_csum_segment_frames(_addr(arena), _addr(offsets), _addr(lengths), n, mss,
                                          _addr(out), stride, capacity, _addr(out_lengths),
                                          _addr(first), st),
           "tulips_csum_segment_frames")
    return out, out_lengths, first


def segment_plan(arena, offsets, lengths, mss: int):
    """Host frames -> first (uint32[n+1]), the plan of
    segment_frames_planned (tulips_csum_segment_plan_host)."""
    import numpy as np
    ar = _host(arena, np.uint8)
    off = _host(offsets, np.uint64)
    ln = _host(lengths, np.uint16)
    n = len(off.keep)
    first = np.zeros(n + 1, dtype=np.uint32)
    _check(lib.tulips_csum_segment_plan_host(ar.ptr, off.ptr, ln.ptr, n, mss,
                                             first.ctypes.data),
           "tulips_csum_segment_plan_host")
    return first


def segment_frames_planned(arena, offsets, lengths, mss: int, first, *, stride: int = 2048,
                           out=None, out_lengths=None, capacity: int | None = None,
                           stream=None):
    """Segmentation of device-resident frames with the caller's plan `first`
    (device int32[n+1], tulips_csum_segment_frames_planned). Returns (out,
    out_lengths)."""
    import torch
    n = int(offsets.numel())
    if int(lengths.numel()) != n or int(first.numel()) != n + 1:
        raise ValueError("offsets/lengths/first size mismatch")
    dev = arena.device
    if capacity is None:
        capacity = int(out.numel()) // stride if out is not None else int(first[n].item())
    if out is None:
        out = torch.empty(max(capacity, 1) * stride, dtype=torch.uint8, device=dev)
    if out_lengths is None:
        out_lengths = torch.zeros(max(capacity, 1), dtype=torch.int16, device=dev)
    if int(out_lengths.numel()) < capacity or int(out.numel()) < capacity * stride:
        raise ValueError("output smaller than its capacity")
    _check(lib.tulips_csum_segment_frames_planned(
        _addr(arena), _addr(offsets), _addr(lengths), n, mss, _addr(first), _addr(out), stride,
        capacity, _addr(out_lengths), _stream(stream)), "tulips_csum_segment_frames_planned")
    return out, out_lengths


def release_stream(stream) -> None:
    """Free the library's per-stream state (counter shards, segmentation
    workspace) after waiting for `stream` (include/tulips_csum.h)."""
    _check(lib.tulips_csum_release_stream(_stream(stream)), "release_stream")


def version() -> str:
    return lib.tulips_csum_version().decode()
