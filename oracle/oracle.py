"""TEST INFRASTRUCTURE ONLY — not part of the product.

ctypes bindings for the CPU checkers:

* ``Oracle``  -> ``oracle/liboracle.so``: the C restatement
  (``oracle/csum_oracle.c``) of the reference checksum path plus the golden
  data generators of SURVEY.md §8c.
* ``Reference`` -> ``oracle/_ref/libtulips_ref.so``: the reference's own
  ``src/stack`` sources compiled by ``oracle/Makefile`` with g++ (present
  only where it was built; it travels to the GPU box as a prebuilt ``.so``),
  or ``libtulips_ref_clang.so``, the same sources built with clang.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libtulips_ref.so")
REF_CLANG_SO = os.path.join(HERE, "_ref", "libtulips_ref_clang.so")  # same sources, clang

MODE_RAW, MODE_INET, MODE_TCP = 0, 1, 2
FLAG_COMPLEMENT = 0x100

# SURVEY.md §8c constants
DATA_SEED = 0x54554C495053
ZIPF_SEED = 0x5A495046
ZIPF_RMAX = 8937

_u8p = C.POINTER(C.c_uint8)
_u16p = C.POINTER(C.c_uint16)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)


def _ptr(a, t):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(t)


def build_oracle() -> None:
    """Compile liboracle.so (gcc only; works on the GPU box too)."""
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)


class _Batchable:
    _batch = None

    def batch(self, arena, offsets=None, lengths=None, *, stride=0,
              fixed_len=0, seeds=None, src=None, dst=None, mode=MODE_RAW,
              n=None, nthreads=1):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            n = len(offsets)
        if lengths is not None:
            lengths = np.ascontiguousarray(lengths, dtype=np.uint16)
        if seeds is not None:
            seeds = np.ascontiguousarray(seeds, dtype=np.uint16)
        if src is not None:
            src = np.ascontiguousarray(src, dtype=np.uint32)
        if dst is not None:
            dst = np.ascontiguousarray(dst, dtype=np.uint32)
        assert n is not None
        out = np.zeros(n, dtype=np.uint16)
        rc = self._batch(_ptr(arena, _u8p), _ptr(offsets, _u64p),
                         _ptr(lengths, _u16p), C.c_uint64(stride),
                         C.c_uint32(fixed_len), _ptr(seeds, _u16p),
                         _ptr(src, _u32p), _ptr(dst, _u32p),
                         _ptr(out, _u16p), C.c_uint64(n), C.c_uint32(mode),
                         C.c_int(nthreads))
        if rc != 0:
            raise ValueError(f"batch rejected its arguments (rc={rc})")
        return out

    @staticmethod
    def _bind_batch(fn):
        fn.restype = C.c_int
        fn.argtypes = [_u8p, _u64p, _u16p, C.c_uint64, C.c_uint32, _u16p,
                       _u32p, _u32p, _u16p, C.c_uint64, C.c_uint32, C.c_int]
        return fn


class Oracle(_Batchable):
    """The C restatement (oracle/csum_oracle.c)."""

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build_oracle()
        L = C.CDLL(path)
        self.lib = L
        L.orc_checksum.restype = C.c_uint16
        L.orc_checksum.argtypes = [C.c_uint16, _u8p, C.c_uint16]
        L.orc_ipv4_checksum.restype = C.c_uint16
        L.orc_ipv4_checksum.argtypes = [_u8p]
        L.orc_icmpv4_checksum.restype = C.c_uint16
        L.orc_icmpv4_checksum.argtypes = [_u8p]
        L.orc_tcp_checksum.restype = C.c_uint16
        L.orc_tcp_checksum.argtypes = [C.c_uint32, C.c_uint32, C.c_uint16, _u8p]
        L.orc_tcp_seed.restype = C.c_uint16
        L.orc_tcp_seed.argtypes = [C.c_uint32, C.c_uint32, C.c_uint16]
        L.orc_fill_splitmix.restype = None
        L.orc_fill_splitmix.argtypes = [_u8p, C.c_uint64, C.c_uint64, C.c_uint64]
        L.orc_zipf_lengths.restype = C.c_int
        L.orc_zipf_lengths.argtypes = [_u16p, C.c_uint64, C.c_uint64, C.c_uint32]
        L.orc_fnv1a_u16.restype = C.c_uint64
        L.orc_fnv1a_u16.argtypes = [_u16p, C.c_uint64]
        self._batch = self._bind_batch(L.orc_batch)

    def checksum(self, seed: int, data: bytes) -> int:
        buf = np.frombuffer(bytes(data) or b"\0", dtype=np.uint8).copy()
        return self.lib.orc_checksum(seed, _ptr(buf, _u8p), len(data))

    def ipv4_checksum(self, hdr: bytes) -> int:
        assert len(hdr) >= 20
        buf = np.frombuffer(bytes(hdr), dtype=np.uint8).copy()
        return self.lib.orc_ipv4_checksum(_ptr(buf, _u8p))

    def icmpv4_checksum(self, hdr: bytes) -> int:
        assert len(hdr) >= 8
        buf = np.frombuffer(bytes(hdr), dtype=np.uint8).copy()
        return self.lib.orc_icmpv4_checksum(_ptr(buf, _u8p))

    def tcp_checksum(self, src: int, dst: int, data: bytes, length=None) -> int:
        length = len(data) if length is None else length
        buf = np.frombuffer(bytes(data) or b"\0", dtype=np.uint8).copy()
        return self.lib.orc_tcp_checksum(src, dst, length, _ptr(buf, _u8p))

    def tcp_seed(self, src: int, dst: int, length: int) -> int:
        return self.lib.orc_tcp_seed(src, dst, length)

    def splitmix_bytes(self, nbytes: int, seed: int = DATA_SEED,
                       byte_off: int = 0) -> np.ndarray:
        out = np.empty(nbytes, dtype=np.uint8)
        self.lib.orc_fill_splitmix(_ptr(out, _u8p), nbytes, seed, byte_off)
        return out

    def zipf_lengths(self, n: int, seed: int = ZIPF_SEED,
                     rmax: int = ZIPF_RMAX) -> np.ndarray:
        out = np.empty(n, dtype=np.uint16)
        if self.lib.orc_zipf_lengths(_ptr(out, _u16p), n, seed, rmax) != 0:
            raise ValueError("bad zipf parameters")
        return out

    def fnv1a_u16(self, v: np.ndarray) -> int:
        v = np.ascontiguousarray(v, dtype=np.uint16)
        return int(self.lib.orc_fnv1a_u16(_ptr(v, _u16p), len(v)))

    def validate_frames(self, arena, offsets, lengths) -> np.ndarray:
        """Per-frame TULIPS_FRAME_* flags (oracle/csum_oracle.c)."""
        f = self.lib.orc_validate_frames
        f.restype = None
        f.argtypes = [_u8p, _u64p, _u16p, C.c_uint64, _u8p]
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint16)
        out = np.zeros(len(offsets), dtype=np.uint8)
        f(_ptr(arena, _u8p), _ptr(offsets, _u64p), _ptr(lengths, _u16p), len(offsets),
          _ptr(out, _u8p))
        return out

    def generate_frames(self, arena, offsets, lengths):
        """Checksum generation (oracle/csum_oracle.c orc_generate_frames) on a
        copy of `arena`; returns (new arena, TULIPS_FRAME_* flags)."""
        f = self.lib.orc_generate_frames
        f.restype = None
        f.argtypes = [_u8p, _u64p, _u16p, C.c_uint64, _u8p]
        arena = np.array(arena, dtype=np.uint8, copy=True)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint16)
        out = np.zeros(len(offsets), dtype=np.uint8)
        f(_ptr(arena, _u8p), _ptr(offsets, _u64p), _ptr(lengths, _u16p), len(offsets),
          _ptr(out, _u8p))
        return arena, out

    def segment_frames(self, arena, offsets, lengths, mss: int, stride: int):
        """Segmentation offload (oracle/csum_oracle.c orc_segment_frames).
        Returns (first[n+1], out bytes [total*stride], out_lengths[total])."""
        L = self.lib
        L.orc_segment_count.restype = C.c_uint32
        L.orc_segment_count.argtypes = [_u8p, _u64p, _u16p, C.c_uint32, C.c_uint32, _u32p]
        L.orc_segment_frames.restype = None
        L.orc_segment_frames.argtypes = [_u8p, _u64p, _u16p, C.c_uint32, C.c_uint32, _u8p,
                                         C.c_uint64, C.c_uint32, _u16p, _u32p]
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint16)
        n = len(offsets)
        first = np.zeros(n + 1, dtype=np.uint32)
        total = L.orc_segment_count(_ptr(arena, _u8p), _ptr(offsets, _u64p),
                                    _ptr(lengths, _u16p), n, mss, _ptr(first, _u32p))
        out = np.zeros(max(total, 1) * stride, dtype=np.uint8)
        out_lens = np.zeros(max(total, 1), dtype=np.uint16)
        L.orc_segment_frames(_ptr(arena, _u8p), _ptr(offsets, _u64p), _ptr(lengths, _u16p),
                             n, mss, _ptr(out, _u8p), stride, total, _ptr(out_lens, _u16p),
                             _ptr(first, _u32p))
        return first, out[:total * stride], out_lens[:total]

    def toeplitz(self, saddr: int, daddr: int, sport: int, dport: int, key: bytes,
                 init: int = 0) -> int:
        """src/stack/Utils.cpp:86-133 restated (oracle/csum_oracle.c)."""
        f = self.lib.orc_toeplitz
        f.restype = C.c_int
        f.argtypes = [C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint16, C.c_size_t,
                      _u8p, C.c_uint32, _u32p]
        k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
        out = np.zeros(1, dtype=np.uint32)
        if f(saddr, daddr, sport, dport, len(key), _ptr(k, _u8p), init & 0xFFFFFFFF,
             _ptr(out, _u32p)) != 0:
            raise ValueError("bad toeplitz arguments")
        return int(out[0])


class Reference(_Batchable):
    """The reference's own functions (oracle/_ref/libtulips_ref.so)."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(
                f"{path} missing: run `make -C oracle ref` where /root/reference exists")
        L = C.CDLL(path)
        self.lib = L
        L.ref_checksum.restype = C.c_uint16
        L.ref_checksum.argtypes = [C.c_uint16, _u8p, C.c_uint16]
        L.ref_ipv4_checksum.restype = C.c_uint16
        L.ref_ipv4_checksum.argtypes = [_u8p]
        L.ref_icmpv4_checksum.restype = C.c_uint16
        L.ref_icmpv4_checksum.argtypes = [_u8p]
        L.ref_tcp_checksum.restype = C.c_uint16
        L.ref_tcp_checksum.argtypes = [C.c_uint32, C.c_uint32, C.c_uint16, _u8p]
        self._batch = self._bind_batch(L.ref_batch)

    @staticmethod
    def available(path: str = REF_SO) -> bool:
        return os.path.exists(path)

    def checksum(self, seed: int, data: bytes) -> int:
        buf = np.frombuffer(bytes(data) or b"\0", dtype=np.uint8).copy()
        return self.lib.ref_checksum(seed, _ptr(buf, _u8p), len(data))

    def ipv4_checksum(self, hdr: bytes) -> int:
        buf = np.frombuffer(bytes(hdr), dtype=np.uint8).copy()
        return self.lib.ref_ipv4_checksum(_ptr(buf, _u8p))

    def icmpv4_checksum(self, hdr: bytes) -> int:
        buf = np.frombuffer(bytes(hdr), dtype=np.uint8).copy()
        return self.lib.ref_icmpv4_checksum(_ptr(buf, _u8p))

    def tcp_checksum(self, src: int, dst: int, data: bytes, length=None) -> int:
        length = len(data) if length is None else length
        buf = np.frombuffer(bytes(data) or b"\0", dtype=np.uint8).copy()
        return self.lib.ref_tcp_checksum(src, dst, length, _ptr(buf, _u8p))

    def toeplitz(self, saddr: int, daddr: int, sport: int, dport: int, key: bytes,
                 init: int = 0) -> int:
        """The reference's own tulips::stack::utils::toeplitz."""
        f = self.lib.ref_toeplitz
        f.restype = C.c_uint32
        f.argtypes = [C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint16, C.c_size_t,
                      _u8p, C.c_uint32]
        k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
        return int(f(saddr, daddr, sport, dport, len(key), _ptr(k, _u8p), init & 0xFFFFFFFF))


def ip4(a: int, b: int, c: int, d: int) -> int:
    """ipv4::Address::m_data for a.b.c.d (wire bytes as a native uint32)."""
    return int.from_bytes(bytes([a, b, c, d]), "little")


def fixed_offsets(n: int, stride: int) -> np.ndarray:
    return np.arange(n, dtype=np.uint64) * np.uint64(stride)


def packed_offsets(lengths: np.ndarray) -> np.ndarray:
    off = np.zeros(len(lengths), dtype=np.uint64)
    if len(lengths) > 1:
        np.cumsum(lengths[:-1], dtype=np.uint64, out=off[1:])
    return off
