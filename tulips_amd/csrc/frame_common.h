// frame_common.h — device helpers shared by the frame kernels (frames.hip,
// segment.hip): absolute-chunk sums, subgroup reductions, and the header
// fields of an Ethernet/IPv4/TCP frame gathered by one subgroup.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tulips_csum.h"
#include "csum_common.h"

namespace tulips_amd {
namespace frame {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4* gchunk_ptr;
typedef const __attribute__((address_space(1))) uint8_t* gbyte_ptr;

__device__ __forceinline__ uint64_t
hsum(u32x4 v)
{
  return (uint64_t(v.x) + uint64_t(v.y)) + (uint64_t(v.z) + uint64_t(v.w));
}

__device__ __forceinline__ uint32_t
byte_mask(int lo, int hi, int b)
{
  int ml = min(max(lo - b, 0), 4);
  int mh = min(max(hi - b, 0), 4);
  return uint32_t((1ull << (8 * mh)) - 1ull) & ~uint32_t((1ull << (8 * ml)) - 1ull);
}

__device__ __forceinline__ uint64_t
masked_hsum(u32x4 v, int lo, int hi)
{
  return (uint64_t(v.x & byte_mask(lo, hi, 0)) +
          uint64_t(v.y & byte_mask(lo, hi, 4))) +
         (uint64_t(v.z & byte_mask(lo, hi, 8)) +
          uint64_t(v.w & byte_mask(lo, hi, 12)));
}

// This lane's LE dword sum of [sa, sa+len) over absolute 16-byte chunks
// (G lanes, U unconditional clamped loads per lane per batch).
template<int G, int U, bool NT>
__device__ __forceinline__ uint64_t
lane_sum(uintptr_t sa, uint32_t len, int lane)
{
  if (len == 0) {
    return 0;
  }
  const uintptr_t a0 = sa & ~uintptr_t(15);
  const int nch = int((sa + len - a0 + 15) >> 4);
  const int last = nch - 1;
  const int head = int(sa - a0);
  const int tail = int(sa + len - a0) - 16 * last;
  const gchunk_ptr p = reinterpret_cast<gchunk_ptr>(a0);
  uint64_t acc = 0;
  for (int c = lane; c < nch; c += U * G) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int cc = min(c + u * G, last);
      v[u] = NT ? __builtin_nontemporal_load(p + cc) : p[cc];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int cc = c + u * G;
      acc += cc <= last ? hsum(v[u]) : 0;
      if (u == 0 && cc == 0 && head != 0) {
        acc -= masked_hsum(v[u], 0, head);
      }
      if (cc == last && tail != 16) {
        acc -= masked_hsum(v[u], tail, 16);
      }
    }
  }
  return acc;
}

template<int G>
__device__ __forceinline__ uint32_t
sub_sum(uint32_t x)
{
  if constexpr (G >= 16) {
    return subgroup_total<G>(x);
  } else {
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) {
      x += __shfl_xor(x, m, 64);
    }
    return x;
  }
}

// The fields of an Ethernet/IPv4/TCP header the frame kernels act on.
struct Header
{
  uint32_t type, vhl, total, frag0, frag1, proto, src, dst;
  bool runt, ipv4, tcp, trunc;
  uint32_t tcplen;
  uint32_t ipck0, ipck1, tcpck0, tcpck1; // checksum field bytes (W >= 40)
  uint32_t id, seq, doff, tflags;         // IP id, TCP seq/offset/flags (W >= 40)
};

// Parse from a byte accessor `byte(off)` (0 for bytes outside the frame);
// `full` also reads the send-side fields (bytes up to 51).
template<bool full, typename ByteAt>
__device__ __forceinline__ Header
parse_header(ByteAt byte, uint32_t flen)
{
  Header h;
  h.type = (byte(12) << 8) | byte(13);
  h.vhl = byte(14);
  h.total = (byte(16) << 8) | byte(17);
  h.frag0 = byte(20);
  h.frag1 = byte(21);
  h.proto = byte(23);
  h.src = byte(26) | (byte(27) << 8) | (byte(28) << 16) | (byte(29) << 24);
  h.dst = byte(30) | (byte(31) << 8) | (byte(32) << 16) | (byte(33) << 24);
  if (full) {
    h.ipck0 = byte(24);
    h.ipck1 = byte(25);
    h.tcpck0 = byte(50);
    h.tcpck1 = byte(51);
    h.id = (byte(18) << 8) | byte(19);
    h.seq = (byte(38) << 24) | (byte(39) << 16) | (byte(40) << 8) | byte(41);
    h.doff = byte(46) >> 4;
    h.tflags = byte(47);
  } else {
    h.ipck0 = h.ipck1 = h.tcpck0 = h.tcpck1 = 0;
    h.id = h.seq = h.doff = h.tflags = 0;
  }
  const bool eth_ip = flen >= 14 && h.type == 0x0800u;
  h.runt = eth_ip && flen < 34;
  h.ipv4 = eth_ip && !h.runt && h.vhl == 0x45u;
  h.tcp = h.ipv4 && (h.frag0 & 0x3fu) == 0 && h.frag1 == 0 && h.proto == 6u;
  h.tcplen = (h.total - 20u) & 0xffffu;
  h.trunc = h.tcp && (h.total < 20u || 34u + h.tcplen > flen);
  return h;
}

// One subgroup: lanes 0..W-1 each fetch one of frame bytes 12 .. 12+W-1
// (only bytes inside the frame) and share them by cross-lane shuffles.
template<int W>
__device__ __forceinline__ Header
gather_header(uintptr_t fa, uint32_t flen, int lane, int sub0)
{
  uint32_t hb = 0;
  if (lane < W && uint32_t(12 + lane) < flen) {
    hb = *reinterpret_cast<gbyte_ptr>(fa + 12 + lane);
  }
  return parse_header<(W >= 40)>(
    [&](int off) { return __shfl(hb, sub0 + off - 12, 64); }, flen);
}

// Frame-aligned dwords F[j] = frame bytes 4j .. 4j+3 for j = 3..12 from the
// 20 dwords w[] of the five aligned chunks holding frame bytes 0..79 (the
// frame starts h0 = 0..15 bytes into chunk 0). w[j + s] for s = h0 >> 2 is
// selected in two bit steps by bit blends (one v_bfi each), then funnel-
// shifted by h0 & 3. Written as a 4-way `s == 0 ? : s == 1 ? ...` chain the
// compiler formed a switch and lowered it to exec-masked branches, ~70
// instructions per header word (the subgroups of a wave differ in s); as
// `?:` on array elements it selected the element's address and went through
// scratch.
__device__ __forceinline__ void
funnel_words(const uint32_t (&w)[20], int h0, uint32_t (&F)[13])
{
  const uint32_t m1 = 0u - uint32_t((h0 >> 2) & 1), m2 = 0u - uint32_t((h0 >> 3) & 1);
  const uint32_t r = uint32_t(h0 & 3);
  uint32_t x[18], y[14];
#pragma unroll
  for (int k = 3; k < 18; ++k) {
    x[k] = (w[k + 1] & m1) | (w[k] & ~m1);
  }
#pragma unroll
  for (int k = 3; k < 14; ++k) {
    y[k] = (x[k + 2] & m2) | (x[k] & ~m2);
  }
#pragma unroll
  for (int j = 3; j < 13; ++j) {
    F[j] = __builtin_amdgcn_alignbyte(y[j + 1], y[j], r);
  }
  F[0] = F[1] = F[2] = 0;
}

// One thread reads the header itself: the five aligned chunks holding frame
// bytes 0..79 (clamped to the frame's last chunk, so nothing outside a chunk
// with frame bytes is touched), funnel-shifted to frame-aligned dwords.
// Within a subgroup that parses the same frame these are broadcast loads.
static __device__ u32x4 k_hdr_zero_chunk;

// load_header split in two so callers can issue the five loads together
// with other loads and parse once they arrive.
struct HeaderChunks
{
  u32x4 c[5];
};

__device__ __forceinline__ HeaderChunks
load_header_chunks(uintptr_t fa, uint32_t flen)
{
  const uintptr_t lo = fa & ~uintptr_t(15);
  const uintptr_t hi = flen ? (fa + flen - 1) & ~uintptr_t(15) : lo;
  HeaderChunks hc;
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    uintptr_t q = lo + 16 * c;
    q = q > hi ? hi : q;
    hc.c[c] = *reinterpret_cast<gchunk_ptr>(
      flen ? q : reinterpret_cast<uintptr_t>(&k_hdr_zero_chunk));
  }
  return hc;
}

__device__ __forceinline__ Header
parse_header_chunks(const HeaderChunks& hc, uintptr_t fa, uint32_t flen)
{
  const uintptr_t lo = fa & ~uintptr_t(15);
  uint32_t w[20];
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    w[4 * c + 0] = hc.c[c].x;
    w[4 * c + 1] = hc.c[c].y;
    w[4 * c + 2] = hc.c[c].z;
    w[4 * c + 3] = hc.c[c].w;
  }
  uint32_t D[13];
  funnel_words(w, int(fa - lo), D);
  return parse_header<true>(
    [&](int k) -> uint32_t {
      return uint32_t(k) < flen ? (D[k >> 2] >> (8 * (k & 3))) & 0xffu : 0u;
    },
    flen);
}

__device__ __forceinline__ Header
load_header(uintptr_t fa, uint32_t flen)
{
  return parse_header_chunks(load_header_chunks(fa, flen), fa, flen);
}

// The header fields a segment count needs (Ethernet type, IPv4 version/IHL,
// total length, fragment bits, protocol: frame bytes 12..23; TCP data
// offset: byte 46) from THREE chunk loads instead of five: the chunk holding
// byte 12, the next one (bytes 12..23 span at most two chunks), and the one
// holding byte 46 (never one of those two). The other fields of the returned
// Header are unspecified. One thread per frame in the segmentation prologue:
// a single workgroup issues these scattered loads for up to 1,024 frames, and
// its memory pipeline, one 64-byte line per lane, is what the prologue waits
// on.
__device__ __forceinline__ Header
load_seg_header(uintptr_t fa, uint32_t flen)
{
  const uintptr_t lo = fa & ~uintptr_t(15);
  const uintptr_t hi = flen ? (fa + flen - 1) & ~uintptr_t(15) : lo;
  const int h0 = int(fa - lo);
  const int ca = (h0 + 12) >> 4, cb = (h0 + 46) >> 4;
  auto ld = [&](int c) {
    uintptr_t q = lo + 16 * uintptr_t(c);
    q = q > hi ? hi : q;
    return *reinterpret_cast<gchunk_ptr>(
      flen ? q : reinterpret_cast<uintptr_t>(&k_hdr_zero_chunk));
  };
  const u32x4 x = ld(ca), y = ld(ca + 1), z = ld(cb);
  HeaderChunks hc;
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    hc.c[c] = c == ca ? x : (c == ca + 1 ? y : z);
  }
  return parse_header_chunks(hc, fa, flen);
}

__device__ __forceinline__ uint32_t
frame_flags(const Header& h, bool ip_ok, bool l4_ok)
{
  if (h.runt) {
    return TULIPS_FRAME_TRUNCATED;
  }
  if (!h.ipv4) {
    return 0;
  }
  return TULIPS_FRAME_IPV4 | (ip_ok ? TULIPS_FRAME_IP_CSUM_OK : 0u) |
         (h.tcp ? TULIPS_FRAME_TCP : 0u) | (h.trunc ? TULIPS_FRAME_TRUNCATED : 0u) |
         (l4_ok ? TULIPS_FRAME_L4_CSUM_OK : 0u);
}

// Contribution of the 16-bit field {b0 @ a, b1 @ a+1} to an LE dword sum
// taken at absolute addresses, modulo 65535 (2^16 == 1).
__device__ __forceinline__ uint32_t
field_contrib(uintptr_t a, uint32_t b0, uint32_t b1)
{
  return (a & 1) ? ((b0 << 8) | b1) : (b0 | (b1 << 8));
}

// Store the 16-bit field v (LE bytes) at a, which may be odd.
__device__ __forceinline__ void
store_field(uintptr_t a, uint32_t v)
{
  typedef __attribute__((address_space(1))) uint8_t* gbyte_wptr;
  typedef __attribute__((address_space(1))) uint16_t* gshort_wptr;
  if ((a & 1) == 0) {
    *reinterpret_cast<gshort_wptr>(a) = uint16_t(v);
  } else {
    reinterpret_cast<gbyte_wptr>(a)[0] = uint8_t(v & 0xff);
    reinterpret_cast<gbyte_wptr>(a)[1] = uint8_t(v >> 8);
  }
}

// ---- whole-frame loads -----------------------------------------------------
//
// A frame's aligned 16-byte chunks, loaded unconditionally as soon as its
// offset and length are known: lane l of a G-lane subgroup holds chunks
// l, l+G, ..., l+(U-1)G (clamped to the last chunk that holds frame bytes, so
// no load ever touches a chunk without one). Header fields and both checksum
// ranges are then taken from these registers: one memory round trip per
// frame instead of one per dependent step (offsets -> header -> IP -> TCP).

static __device__ u32x4 k_frame_zero_chunk; // what an empty frame "loads"

template<int G, int U>
struct FrameChunks
{
  u32x4 v[U];
  uintptr_t a0; // 16-aligned address of chunk 0
  int h0;       // frame start - a0
  int last;     // last chunk holding frame bytes (-1: empty frame)
};

template<int G, int U, bool NT>
__device__ __forceinline__ void
load_frame(uintptr_t fa, uint32_t flen, int lane, FrameChunks<G, U>& fc)
{
  fc.a0 = fa & ~uintptr_t(15);
  fc.h0 = int(fa - fc.a0);
  fc.last = flen ? int((uint32_t(fc.h0) + flen - 1) >> 4) : -1;
  const gchunk_ptr p =
    flen ? reinterpret_cast<gchunk_ptr>(fc.a0)
         : reinterpret_cast<gchunk_ptr>(reinterpret_cast<uintptr_t>(&k_frame_zero_chunk));
  const int lim = max(fc.last, 0);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int cc = min(lane + u * G, lim);
    fc.v[u] = NT ? __builtin_nontemporal_load(p + cc) : p[cc];
  }
}

// Frame-aligned header dwords F[j] = frame bytes 4j .. 4j+3 for j = 3..12
// (bytes 12..51), assembled from chunks 0..4 held by lanes 0..4 of the
// subgroup. Bytes past the frame end are unspecified (callers bound them).
// G = 16 (a subgroup is one DPP row): row_newbcast moves lane c's dwords to
// the whole row in VALU; G = 64: readlane; otherwise ds_bpermute.
template<int G>
__device__ __forceinline__ uint32_t
from_lane(uint32_t x, int c, int sub0)
{
  if constexpr (G == 16) {
    switch (c) { // (the DPP control must be an immediate)
    case 0: return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x150, 0xf, 0xf, false));
    case 1: return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x151, 0xf, 0xf, false));
    case 2: return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x152, 0xf, 0xf, false));
    case 3: return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x153, 0xf, 0xf, false));
    default: return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x154, 0xf, 0xf, false));
    }
  } else if constexpr (G == 64) {
    return __builtin_amdgcn_readlane(x, c);
  } else {
    return __shfl(x, sub0 + c, 64);
  }
}

template<int G>
__device__ __forceinline__ void
header_words(const u32x4& v0, int h0, int sub0, uint32_t (&F)[13])
{
  // Lane c (c < 4) funnel-shifts its own chunk and the next lane's (one DPP
  // row_shl:1 per dword) to the frame-aligned words 4c .. 4c+3, then those
  // ten words are broadcast: a few registers per lane instead of the whole
  // 80-byte window replicated on every lane.
  uint32_t e[8] = {v0.x, v0.y, v0.z, v0.w};
  e[4] = uint32_t(__builtin_amdgcn_update_dpp(0, int(v0.x), 0x101, 0xf, 0xf, false));
  e[5] = uint32_t(__builtin_amdgcn_update_dpp(0, int(v0.y), 0x101, 0xf, 0xf, false));
  e[6] = uint32_t(__builtin_amdgcn_update_dpp(0, int(v0.z), 0x101, 0xf, 0xf, false));
  e[7] = uint32_t(__builtin_amdgcn_update_dpp(0, int(v0.w), 0x101, 0xf, 0xf, false));
  const uint32_t m1 = 0u - uint32_t((h0 >> 2) & 1), m2 = 0u - uint32_t((h0 >> 3) & 1);
  const uint32_t r = uint32_t(h0 & 3);
  uint32_t t[7], q[5], o[4];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    t[k] = (e[k + 1] & m1) | (e[k] & ~m1);
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    q[k] = (t[k + 2] & m2) | (t[k] & ~m2);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    o[k] = __builtin_amdgcn_alignbyte(q[k + 1], q[k], r);
  }
#pragma unroll
  for (int j = 3; j < 13; ++j) {
    F[j] = from_lane<G>(o[j & 3], j >> 2, sub0);
  }
  F[0] = F[1] = F[2] = 0;
}

// Header bytes past the frame end read as 0 (parse_header's contract): the
// words are masked once, and only for frames shorter than the 52 bytes they
// hold (a test per subgroup), instead of a compare and a select per byte
// read (the frame kernels' per-frame VALU count is what bounds them).
__device__ __forceinline__ void
mask_past_end(uint32_t (&F)[13], uint32_t flen)
{
  if (flen < 52u) {
#pragma unroll
    for (int j = 3; j < 13; ++j) {
      const int n = min(max(int(flen) - 4 * j, 0), 4);
      F[j] &= n >= 4 ? 0xffffffffu : (1u << (8 * n)) - 1u;
    }
  }
}

// The frame's header fields from its first register row (header_words), and
// the IPv4 header's LE 16-bit word sum (frame bytes 14..33, from the same
// broadcast words: frame-relative, so the header starts at an even offset of
// this word grid) folded to 32 bits.
template<int G, int U>
__device__ __forceinline__ Header
frame_header_ip(const FrameChunks<G, U>& fc, uint32_t flen, int sub0, uint32_t& ipsum)
{
  uint32_t F[13];
  header_words<G>(fc.v[0], fc.h0, sub0, F);
  mask_past_end(F, flen);
  ipsum = fold64(uint64_t(F[3] >> 16) + F[4] + F[5] + F[6] + F[7] + (F[8] & 0xffffu));
  return parse_header<true>(
    [&](int k) -> uint32_t { return (F[k >> 2] >> (8 * (k & 3))) & 0xffu; }, flen);
}

// This lane's sum of the bytes at chunk-relative offsets [lo, hi) (offsets
// from a0; the range must lie inside the frame), as 32-bit accumulated
// 16-bit halves (v_dot2: congruent to the LE dword sum mod 65535, at most
// 8 * 0xffff per chunk, so no 64-bit adds), with byte masks only where a
// chunk straddles lo or hi: the whole-chunk test is a compare and a select
// per row, and the masked sum runs under a branch rows without a boundary
// skip. Only the first UM rows of registers are looked at; with UM == U,
// bytes beyond the G*U chunks held in registers are summed by a trailing
// lane_sum (jumbo). (A branch-free form with 64-bit adds took 10 % fewer
// instructions at 16 x 6 but spilled at 16 x 8 and 8 x 8/16:
// profiles/probe_frames_r03.txt.)
typedef unsigned short fr_u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t
dot2_acc(uint32_t x, uint32_t acc)
{
  const fr_u16x2 one = {1, 1};
  fr_u16x2 h;
  __builtin_memcpy(&h, &x, sizeof(h));
  return __builtin_amdgcn_udot2(h, one, acc, false);
}

// bytes [ml, mh) of a dword, 0 <= ml, mh <= 4 (32-bit shifts only)
__device__ __forceinline__ uint32_t
dword_mask(int ml, int mh)
{
  const uint32_t below_h = mh >= 4 ? 0xffffffffu : (1u << (8 * mh)) - 1u;
  const uint32_t below_l = ml >= 4 ? 0xffffffffu : (1u << (8 * ml)) - 1u;
  return below_h & ~below_l;
}

// acc plus the 16-bit halves of v (all 16 bytes, or bytes [lo, hi) only)
__device__ __forceinline__ uint32_t
chunk_dot2(u32x4 v, uint32_t acc)
{
  return dot2_acc(v.w, dot2_acc(v.z, dot2_acc(v.y, dot2_acc(v.x, acc))));
}

__device__ __forceinline__ uint32_t
masked_dot2(u32x4 v, int l, int h, uint32_t acc)
{
  acc = dot2_acc(v.x & dword_mask(min(l, 4), min(h, 4)), acc);
  acc = dot2_acc(v.y & dword_mask(min(max(l - 4, 0), 4), min(max(h - 4, 0), 4)), acc);
  acc = dot2_acc(v.z & dword_mask(min(max(l - 8, 0), 4), min(max(h - 8, 0), 4)), acc);
  return dot2_acc(v.w & dword_mask(min(max(l - 12, 0), 4), min(max(h - 12, 0), 4)), acc);
}

template<int G, int U, bool NT, int UM = U>
__device__ __forceinline__ uint32_t
range_sum32(const FrameChunks<G, U>& fc, int lane, int lo, int hi)
{
  static_assert(UM >= 1 && UM <= U, "rows");
  static_assert(G >= 4, "lo (< 64) lies in the first row");
  uint32_t acc = 0;
#pragma unroll
  for (int u = 0; u < UM; ++u) {
    const int b = 16 * (lane + u * G);
    const u32x4 v = fc.v[u];
    const bool full = b >= lo && b + 16 <= hi;
    const uint32_t with = chunk_dot2(v, acc); // (chained through acc: one live temporary)
    acc = full ? with : acc;
    if (!full && b < hi && b + 16 > lo) {
      // rows past the first start past lo (lo < 16 * G: the frame's header),
      // so only their upper bound cuts a chunk
      acc = u == 0 ? masked_dot2(v, max(lo - b, 0), min(hi - b, 16), acc)
                   : masked_dot2(v, 0, min(hi - b, 16), acc);
    }
  }
  if constexpr (UM == U) {
    constexpr int held = 16 * G * U;
    if (hi > held) {
      const int from = max(lo, held);
      acc += fold64(lane_sum<G, U, NT>(fc.a0 + uintptr_t(from), uint32_t(hi - from), lane));
    }
  }
  return acc;
}


// The same with 64-bit LE dword sums and per-row masks: kept for the
// geometries with 16 rows per lane (8 x 16), where range_sum32's extra
// temporaries cost a VGPR spill at their 128-register budget.
template<int G, int U, bool NT, int UM = U>
__device__ __forceinline__ uint64_t
range_sum64(const FrameChunks<G, U>& fc, int lane, int lo, int hi)
{
  static_assert(UM >= 1 && UM <= U, "rows");
  uint64_t acc = 0;
#pragma unroll
  for (int u = 0; u < UM; ++u) {
    const int b = 16 * (lane + u * G);
    const int l = max(lo - b, 0), h = min(hi - b, 16);
    if (l < h) {
      acc += (l == 0 && h == 16) ? hsum(fc.v[u]) : masked_hsum(fc.v[u], l, h);
    }
  }
  if constexpr (UM == U) {
    constexpr int held = 16 * G * U;
    if (hi > held) {
      const int from = max(lo, held);
      acc += lane_sum<G, U, NT>(fc.a0 + uintptr_t(from), uint32_t(hi - from), lane);
    }
  }
  return acc;
}

// A lane's share of the TCP range [lo, hi), folded to 32 bits: range_sum32,
// or range_sum64 for the 16-row geometries.
template<int G, int U, bool NT>
__device__ __forceinline__ uint32_t
tcp_range_part(const FrameChunks<G, U>& fc, int lane, int lo, int hi)
{
  if constexpr (U > 8) {
    return fold64(range_sum64<G, U, NT>(fc, lane, lo, hi));
  } else {
    return fold32(range_sum32<G, U, NT>(fc, lane, lo, hi));
  }
}

} // namespace frame
} // namespace tulips_amd
