"""ctypes binding of the measurement library (benchlib/libtulips_csum_bench.so,
include/tulips_csum_bench.h): the SURVEY.md §8c device data fill, the
ceiling kernels bench.py compares the product kernels with, the GPU sleep
used to gate timed regions, C-timed latency loops and the crash backtrace
hook. Not part of the product: tulips_amd never imports it."""
from __future__ import annotations

import ctypes as C
import os

from tulips_amd import csum  # loads the product (and torch's HIP runtime) first

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libtulips_csum_bench.so")

_vp = C.c_void_p
_SIGNATURES = {
    "tulips_csum_fill_splitmix": (C.c_int, [_vp, C.c_uint64, C.c_uint64, C.c_uint64, _vp]),
    "tulips_csum_gpu_sleep": (C.c_int, [C.c_uint32, _vp]),
    "tulips_csum_debug_crash_backtrace": (C.c_int, [C.c_int]),
    "tulips_csum_stream_read": (C.c_int, [_vp, C.c_uint64, _vp, C.c_uint32, _vp]),
    "tulips_csum_stream_read_tiles": (C.c_int, [_vp, C.c_uint64, C.c_uint32, _vp, _vp]),
    "tulips_csum_stream_read_slots": (C.c_int, [_vp, C.c_uint64, C.c_uint32, C.c_uint32, _vp,
                                                _vp]),
    "tulips_csum_stream_read_slots_geom": (C.c_int, [_vp, C.c_uint64, C.c_uint32, C.c_uint32,
                                                     C.c_int, C.c_int, _vp, _vp]),
    "tulips_csum_stream_copy_slots": (C.c_int, [_vp, C.c_uint64, C.c_uint32, C.c_uint32,
                                                C.c_uint32, C.c_uint32, _vp, C.c_uint64, _vp]),
    "tulips_csum_time_validate": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, C.c_uint32,
                                            C.c_uint32, _vp, _vp]),
    "tulips_csum_time_validate_ring": (C.c_int, [_vp, C.c_int, _vp, C.c_uint64, C.c_uint32,
                                                 _vp, _vp, C.c_uint32, C.c_uint32, _vp, _vp]),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make benchlib` or "
                          "`python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def _check(rc: int, what: str) -> None:
    if rc != csum.STATUS_OK:
        raise csum.CsumError(rc, what)


def fill_splitmix(dst, nbytes: int | None = None, seed: int = 0x54554C495053,
                  byte_off: int = 0, stream=None) -> None:
    """Device fill with the SURVEY.md §8c SplitMix64 byte stream."""
    nbytes = int(dst.numel()) if nbytes is None else nbytes
    _check(lib.tulips_csum_fill_splitmix(csum._addr(dst), nbytes, seed, byte_off,
                                         csum._stream(stream)),
           "tulips_csum_fill_splitmix")


def stream_read(buf, sink, nbytes: int | None = None, max_blocks: int = 0,
                stream=None) -> None:
    """The plain streaming-read ceiling over buf[:nbytes]."""
    nbytes = int(buf.numel()) if nbytes is None else nbytes
    _check(lib.tulips_csum_stream_read(csum._addr(buf), nbytes, csum._addr(sink),
                                       max_blocks, csum._stream(stream)),
           "tulips_csum_stream_read")


def gpu_sleep(us: int, stream=None) -> None:
    _check(lib.tulips_csum_gpu_sleep(us, csum._stream(stream)), "tulips_csum_gpu_sleep")


def crash_backtrace(enable: bool = True) -> None:
    _check(lib.tulips_csum_debug_crash_backtrace(1 if enable else 0),
           "tulips_csum_debug_crash_backtrace")
