// csum_device.h — device-side building blocks shared by the checksum kernels
// (csum_kernels.hip) and the archived measured variants
// (tools/sessions/variants/csum_variants.hip): 16-byte chunk loads at absolute
// alignment, exact boundary masking, per-chunk 16-bit-half sums (v_dot2),
// DPP wave scans, per-segment side inputs and result emission, and the
// in-order-arena (SPAN) launch arguments. Semantics: csum_common.h
// (src/stack/Utils.cpp:14-42 closed form).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "csum_common.h"
#include "csum_launch.h"

namespace tulips_amd {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Global (address space 1) pointers: global_load_* instead of flat_load_*,
// which would also tie every load to lgkmcnt.
typedef const __attribute__((address_space(1))) u32x4* gchunk_ptr;

template<bool NT>
__device__ __forceinline__ u32x4
load_chunk(gchunk_ptr p)
{
  if constexpr (NT) {
    return __builtin_nontemporal_load(p);
  } else {
    return *p;
  }
}

__device__ __forceinline__ uint64_t
hsum(u32x4 v)
{
  return (uint64_t(v.x) + uint64_t(v.y)) + (uint64_t(v.z) + uint64_t(v.w));
}

// Mask of the bytes [lo, hi) of a dword whose first byte is byte `b` of its
// chunk (lo/hi are chunk-relative, 0..16).
__device__ __forceinline__ uint32_t
byte_mask(int lo, int hi, int b)
{
  int ml = min(max(lo - b, 0), 4);
  int mh = min(max(hi - b, 0), 4);
  uint32_t keep_hi = uint32_t((1ull << (8 * mh)) - 1ull);
  uint32_t drop_lo = uint32_t((1ull << (8 * ml)) - 1ull);
  return keep_hi & ~drop_lo;
}

// Dword sum of the bytes [lo, hi) of chunk v.
__device__ __forceinline__ uint64_t
masked_hsum(u32x4 v, int lo, int hi)
{
  return (uint64_t(v.x & byte_mask(lo, hi, 0)) +
          uint64_t(v.y & byte_mask(lo, hi, 4))) +
         (uint64_t(v.z & byte_mask(lo, hi, 8)) +
          uint64_t(v.w & byte_mask(lo, hi, 12)));
}

// Sum of the bytes of segment [sa, sa+len) held by this lane, as a 64-bit
// little-endian dword sum over absolute 16-byte-aligned chunks. The hot loop
// adds whole chunks with no masking or predication; the bytes of the first
// and last chunk that lie outside the segment are then subtracted exactly by
// the (at most two) lanes that own those chunks.
template<int G, int U, bool NT>
__device__ __forceinline__ uint64_t
lane_partial(uintptr_t sa, uint32_t len, int lane)
{
  if (len == 0) {
    return 0;
  }
  const uintptr_t a0 = sa & ~uintptr_t(15);
  const uintptr_t ea = sa + len;
  const int nch = int((ea - a0 + 15) >> 4);
  const gchunk_ptr p = reinterpret_cast<gchunk_ptr>(a0);
  const int head = int(sa - a0);                   // bytes [0, head) of chunk 0
  const int last = nch - 1;
  const int tail = int(ea - a0) - 16 * last;       // bytes [tail, 16) of the last
  uint64_t acc = 0;
  // Add chunk `cc` (already in registers) and take out, exactly, the bytes of
  // the two boundary chunks that lie outside the segment. The corrections run
  // under exec masks that are empty for all but <= 2 lanes per segment, so
  // the common path costs one compare + skip per chunk and no extra load.
  auto consume = [&](const u32x4& v, int cc, bool may_be_first) {
    const uint64_t s = hsum(v);
    acc += cc <= last ? s : 0;  // slots past the end re-read chunk `last`
    if (may_be_first && cc == 0 && head != 0) {
      acc -= masked_hsum(v, 0, head);
    }
    if (cc == last && tail != 16) {
      acc -= masked_hsum(v, tail, 16);
    }
  };
  // Every load is unconditional: slots past the segment's last chunk load
  // that chunk again (same line, merged by the TA, L1-resident) and are
  // discarded by a select. Loads under exec-mask branches would make hipcc
  // drain vmcnt after each one, i.e. one memory round trip per chunk.
  for (int c = lane; c < nch; c += U * G) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u] = load_chunk<NT>(p + min(c + u * G, last));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      consume(v[u], c + u * G, u == 0);
    }
  }
  return acc;
}

template<int G>
__device__ __forceinline__ uint32_t
subgroup_sum(uint32_t x)
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

struct FixedSegs
{
  const uint8_t* base;
  uint64_t stride;
  uint32_t len;
  __device__ __forceinline__ uint64_t off(uint32_t i) const
  {
    return uint64_t(i) * stride;
  }
  __device__ __forceinline__ uint32_t length(uint32_t) const { return len; }
};

struct VarSegs
{
  const uint8_t* base;
  const uint64_t* offs;
  const uint16_t* lens;
  __device__ __forceinline__ uint64_t off(uint32_t i) const { return offs[i]; }
  __device__ __forceinline__ uint32_t length(uint32_t i) const
  {
    return lens[i];
  }
};

// Per-segment side inputs (seed or TCP pseudo-header addresses).
struct SideIn
{
  uint32_t seed, src, dst;
};

__device__ uint32_t k_zero_word[1] = { 0 }; // global memory, never written

typedef const __attribute__((address_space(1))) uint16_t* gu16_ptr;
typedef const __attribute__((address_space(1))) uint32_t* gu32_ptr;

// Issue the side-input loads of segment `seg` UNCONDITIONALLY, before its
// chunk loads so that they travel together: an unused input reads a zero
// word instead (pointer select, no branch). A load under a branch would make
// hipcc drain vmcnt(0) at the join; a load issued after the reduction would
// cost the segment one more memory round trip.
__device__ __forceinline__ SideIn
load_side(uint32_t seg, const uint16_t* __restrict__ seeds,
          const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
          uint32_t mode)
{
  const uint32_t m = mode & MODE_MASK;
  const bool tcp = m == MODE_TCP;
  const bool seeded = !tcp && seeds != nullptr;
  const uintptr_t zero = reinterpret_cast<uintptr_t>(k_zero_word);
  // explicit global-address-space pointers: a generic (flat) load would make
  // hipcc wait for vmcnt(0) and lgkmcnt(0) before any use
  const gu16_ptr ps = reinterpret_cast<gu16_ptr>(
    seeded ? reinterpret_cast<uintptr_t>(seeds + seg) : zero);
  const gu32_ptr pa = reinterpret_cast<gu32_ptr>(
    tcp ? reinterpret_cast<uintptr_t>(src + seg) : zero);
  const gu32_ptr pb = reinterpret_cast<gu32_ptr>(
    tcp ? reinterpret_cast<uintptr_t>(dst + seg) : zero);
  return SideIn{ *ps, *pa, *pb };
}

// Finish and write one segment's result (lane 0 of its subgroup); no loads.
__device__ __forceinline__ void
emit_with(uint32_t seg, uint32_t part, uintptr_t sa, uint32_t len, SideIn in,
          uint16_t* __restrict__ out, uint32_t* __restrict__ bad,
          uint32_t mode, bool nt_store)
{
  const uint32_t r =
    finish(part, (sa & 1) != 0, mode, in.seed, in.src, in.dst, len);
  if (out) {
    if (nt_store) {
      __builtin_nontemporal_store(uint16_t(r), out + seg);
    } else {
      out[seg] = uint16_t(r);
    }
  }
  if (bad && (r ^ ((mode & FLAG_COMPLEMENT) ? 0u : 0xffffu)) != 0) {
    // this block's counter shard (csum_launch.h): a verify of an all-bad
    // burst otherwise serialises one same-address atomic per wave
    atomicAdd(bad + CNT_LINE * (blockIdx.x % CNT_SHARDS), 1u);
  }
}

__device__ uint32_t k_zero_chunk[4] __attribute__((aligned(16))) = { 0, 0, 0, 0 };

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// Sum of the eight little-endian 16-bit halves of a chunk.
__device__ __forceinline__ uint32_t
half_sum(uint32_t x, uint32_t acc)
{
  const u16x2 one = {1, 1};
  // (through a scalar + memcpy: __builtin_bit_cast applied directly to an
  // ext_vector element compiled to element .x for every element here)
  u16x2 h;
  __builtin_memcpy(&h, &x, sizeof(h));
  return __builtin_amdgcn_udot2(h, one, acc, false);
}

__device__ __forceinline__ uint32_t
chunk_value_acc(u32x4 v, uint32_t acc)
{
  const uint32_t x = v.x, y = v.y, z = v.z, w = v.w;
  return half_sum(w, half_sum(z, half_sum(y, half_sum(x, acc))));
}

__device__ __forceinline__ uint32_t
chunk_value(u32x4 v)
{
  return chunk_value_acc(v, 0u);
}

// The same for the bytes [lo, hi) of a chunk only.
__device__ __forceinline__ uint32_t
masked_value(u32x4 v, int lo, int hi)
{
  u32x4 m;
  m.x = v.x & byte_mask(lo, hi, 0);
  m.y = v.y & byte_mask(lo, hi, 4);
  m.z = v.z & byte_mask(lo, hi, 8);
  m.w = v.w & byte_mask(lo, hi, 12);
  return chunk_value(m);
}

// Inclusive u32 add-scan over the 64 lanes of a wave (csum_common.h).
__device__ __forceinline__ uint32_t
wave_incl_scan(uint32_t x)
{
  return wave_inclusive_sum(x);
}

__device__ __forceinline__ uint64_t
readlane64(uint64_t v, uint32_t k)
{
  const uint32_t lo = __builtin_amdgcn_readlane(uint32_t(v), k);
  const uint32_t hi = __builtin_amdgcn_readlane(uint32_t(v >> 32), k);
  return (uint64_t(hi) << 32) | lo;
}

// Workgroup barrier for LDS hand-offs only: the wave's LDS operations are
// complete (lgkmcnt(0)), its vector-memory loads may still be in flight.
// __syncthreads() would also wait for every outstanding global load
// (vmcnt(0)), i.e. for the slowest of them, at each barrier.
__device__ __forceinline__ void
lds_barrier()
{
  __builtin_amdgcn_s_waitcnt(0xc07f); // vmcnt(63) expcnt(7) lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
}

struct SpanArgs
{
  const uint8_t* base;
  uint64_t arena;
  const uint64_t* offs;
  const uint16_t* lens;
  const uint16_t* seeds;
  const uint32_t* src;
  const uint32_t* dst;
  uint16_t* out;
  uint32_t* bad;
  uint32_t n;
  uint32_t mode;
  uint32_t nt_store;
  uint64_t* slots; // split form: one 64-bit word per range (stream_state.h)
  uint64_t nslots; // words in `slots`
  uint32_t salt;   // xor-ed into the split words' tag (per word array)
  uint64_t bias;   // segment i starts at base + offs[i] - bias
  uint64_t k1;     // tail-shaped form: ranges k >= k1 are the short tail ranges
};

typedef const __attribute__((address_space(1))) uint64_t* gu64_ptr;

// Ranges of W bytes covering [A, A + K W), A = base rounded down to 16 B:
// position base + arena (where an empty last segment may start) included.
inline uint64_t
span_ranges(const uint8_t* base, uint64_t arena, uint64_t W)
{
  return ((arena + (reinterpret_cast<uintptr_t>(base) & 15u)) / W) + 1;
}

// Search interval update after one round of 256 samples L + q*st (q < 256):
// c of them (a prefix, offsets being sorted) lie below the target.
__device__ __forceinline__ void
span_narrow(uint32_t& L, uint32_t& R, uint32_t st, uint32_t c)
{
  if (c == 0) {
    R = L;
  } else {
    const uint32_t nl = L + (c - 1) * st + 1;
    R = min(L + c * st, R);
    L = nl;
  }
}

} // namespace
} // namespace tulips_amd
