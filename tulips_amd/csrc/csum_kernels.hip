// csum_kernels.hip — gfx950 (MI355X, CDNA4) kernels for batched TULIPS
// checksums. Reference semantics: src/stack/Utils.cpp:14-42 (a1),
// src/stack/tcpv4/Processor.cpp:337-357 (a2), src/stack/IPv4.cpp:75-82 (a5),
// src/stack/ICMPv4.cpp:10-15 (a6); closed form in csum_common.h.
//
// Design: the op is an HBM-read-bound integer reduction
// (~0.5 VALU op per byte), so the kernels are built for bytes in flight, not
// arithmetic. Three shipped families, one per batch shape:
//   * csum_kernel — fixed stride and length (F1500, F9000): a SUBGROUP of G
//     lanes (G = 16/32/64) owns one segment; lane l reads the 16-byte-aligned
//     chunks l, l+G, ... with global_load_dwordx4, U per lane in flight,
//     boundary bytes taken out exactly in registers;
//   * csum_packed_kernel — variable lengths at any offsets: one wave per 8
//     segments, their chunk lists laid end to end in one packed chunk space,
//     double-buffered 64-chunk windows;
//   * csum_span_kernel — in-order arenas (tulips_csum_batch_arena): the work
//     is cut by arena BYTES; segments crossing a range boundary are summed in
//     parts that meet in a per-range word.
// The measured losers of rounds 1-2 (hybrid, lane-parallel cursors,
// workgroup-balanced, halo / boundary-slot / staged span forms, metadata
// prefetch) live in tools/sessions/variants/, outside the product library.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tulips_csum.h"
#include "csum_common.h"
#include "csum_device.h"
#include "csum_launch.h"
#include "span_kernel.h"
#include "stream_state.h"

#include <memory>
#include <mutex>

namespace tulips_amd {

namespace {

template<int G, int U, bool NT, class Segs>
__global__ __launch_bounds__(1024) void
csum_kernel(Segs segs, const uint16_t* __restrict__ seeds,
            const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
            uint16_t* __restrict__ out, uint32_t* __restrict__ bad,
            uint32_t n, uint32_t mode, bool nt_store)
{
  const int lane = threadIdx.x & (G - 1);
  const uint32_t groups_per_block = blockDim.x / G;
  const uint32_t nsub = gridDim.x * groups_per_block;
  uint32_t seg = xcd_block(blockIdx.x, gridDim.x) * groups_per_block + threadIdx.x / G;
  for (; seg < n; seg += nsub) {
    const uint64_t off = segs.off(seg);
    const uint32_t len = segs.length(seg);
    const uintptr_t sa = reinterpret_cast<uintptr_t>(segs.base) + off;
    const SideIn side = load_side(seg, seeds, src, dst, mode);
    const uint64_t acc = lane_partial<G, U, NT>(sa, len, lane);
    const uint32_t part = subgroup_sum<G>(fold64(acc));
    if (lane == 0) {
      emit_with(seg, part, sa, len, side, out, bad, mode, nt_store);
    }
  }
}

// ---------------------------------------------------------------------------
// PACKED variable-length kernel: one wave per S consecutive segments, whose
// chunk lists are laid end to end in one "packed chunk space" of T chunks
// (segment k owns packed chunks [P_k, P_k + nch_k), P = exclusive prefix of
// nch over the wave's lanes). The wave walks that space in 64-chunk windows:
// lane j of window b reads packed chunk b + j, so every lane of every load
// instruction carries a useful chunk whatever the length mix (a 64 B and a
// 9 KB segment cost 5 and 563 lane-loads), U windows are in flight per lane,
// and no segment ever waits on another's round trip.
//
//   * window -> address: a scalar cursor walks the wave's non-empty segments
//     (s_ff1 over a ballot). The window starts with the segment holding its
//     first chunk; each segment starting inside it hands its lanes
//     D_k = chunkbase_k - 16*P_k with one compare + 2 selects, and a lane's
//     address is D + 16*(b + j). Uniform across lanes except at segment
//     starts (about 1.5 per window for Zipf lengths).
//   * per-chunk value: sum of the 8 little-endian 16-bit halves (4 x
//     v_dot2_u32_u16 against (1,1)) — congruent to the LE dword sum mod
//     65535, linear in the bytes, zero iff the bytes are zero, <= 0x7fff8.
//   * per-segment sum without a segmented reduction: an inclusive wave scan
//     of the values (u32, wrapping) gives a running prefix R over the packed
//     space; a segment's sum is R(its last chunk) - R(previous segment's last
//     chunk), exact because one segment's true sum is < 2^31 (4097 chunks).
//     A second scalar cursor picks those R values out with v_readlane and
//     parks each sum in its segment's lane with a lane-select.
//   * boundary bytes: the bulk adds whole chunks; the bytes of the first and
//     last chunk outside the segment are subtracted at the end from two
//     chunk loads the segment's own lane issued with its metadata.
// The result matches the other kernels' partial (finish(), csum_common.h).
// ---------------------------------------------------------------------------
// Metadata of one segment (lane k < S of a wave owns segment g0 + k).
struct SegMeta
{
  uint32_t len;
  uint64_t off;
  SideIn side;
};

template<int S, int U, bool NT>
__global__ __launch_bounds__(1024) void
csum_packed_kernel(VarSegs segs, const uint16_t* __restrict__ seeds,
                   const uint32_t* __restrict__ src,
                   const uint32_t* __restrict__ dst, uint16_t* __restrict__ out,
                   uint32_t* __restrict__ bad, uint32_t n, uint32_t mode,
                   bool nt_store)
{
  static_assert(S >= 1 && S <= 64, "one segment per lane at most");
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = (xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  const uintptr_t base = reinterpret_cast<uintptr_t>(segs.base);
  const uintptr_t zero_chunk = reinterpret_cast<uintptr_t>(k_zero_chunk);
  // metadata: lane k < S owns segment g + k (coalesced loads; lanes past n
  // re-read segment n - 1 and drop it)
  auto load_meta = [&](uint32_t g) {
    const uint32_t sg = g + lane;
    const bool own = lane < uint32_t(S) && sg < n;
    const uint32_t sk = own ? sg : n - 1;
    SegMeta m;
    m.len = own ? segs.length(sk) : 0u;
    m.off = segs.off(sk);
    m.side = load_side(sk, seeds, src, dst, mode);
    return m;
  };
  const uint32_t gstride = nwaves * S;
  for (uint32_t g0 = wave * S; g0 < n; g0 += gstride) {
    const SegMeta meta = load_meta(g0);
    const uint32_t seg = g0 + lane;
    const bool mine = lane < uint32_t(S) && seg < n;
    const uint32_t len = meta.len;
    const uintptr_t sa = base + meta.off;
    const SideIn side = meta.side;
    const uintptr_t a0 = sa & ~uintptr_t(15);
    const uint32_t nch = len ? uint32_t((sa + len - a0 + 15) >> 4) : 0u;
    const int head = int(sa - a0);
    const int tail = nch ? int(sa + len - a0) - 16 * int(nch - 1) : 16;
    // boundary chunks, only where bytes must be taken out (else a zero chunk)
    const gchunk_ptr pf = reinterpret_cast<gchunk_ptr>(
      (nch && head != 0) ? a0 : zero_chunk);
    const gchunk_ptr pl = reinterpret_cast<gchunk_ptr>(
      (nch && tail != 16) ? a0 + 16 * uintptr_t(nch - 1) : zero_chunk);
    const u32x4 cfirst = load_chunk<NT>(pf);
    const u32x4 clast = load_chunk<NT>(pl);
    // ---- packed chunk space ------------------------------------------------
    const uint32_t incl = wave_incl_scan(nch);
    const uint32_t P = incl - nch;                  // first packed chunk
    const uint32_t T = __builtin_amdgcn_readlane(incl, 63);
    const uint32_t Lst = incl - 1;                  // last packed chunk
    const uint64_t D = uint64_t(a0) - 16ull * P;    // address = D + 16*c
    const uint64_t nonempty = __ballot(nch != 0);
    uint64_t pend_start = nonempty, pend_end = nonempty;
    uint64_t dcur = uint64_t(zero_chunk);           // D of the open segment
    uint32_t run = 0;                               // R carried across windows
    uint32_t eprev = 0;                             // R at the previous end
    uint32_t sum = 0;                               // segment sum (lane k)
    // U windows starting at chunk w0: all U addresses first, then the U loads
    // back to back (a load followed by control flow gets a vmcnt drain from
    // hipcc)
    auto issue = [&](uint32_t w0, u32x4 (&v)[U]) {
      uint64_t addr[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t b = w0 + 64u * u;
        // the segment holding chunk b owns the window; segments starting in
        // [b, b + 64) take over their lanes
        uint64_t dl = dcur;
        while (pend_start) {
          const uint32_t k = uint32_t(__builtin_ctzll(pend_start));
          const uint32_t pk = __builtin_amdgcn_readlane(P, k);
          if (pk >= b + 64u) {
            break;
          }
          pend_start &= pend_start - 1;
          const uint64_t dk = readlane64(D, k);
          dl = lane + b >= pk ? dk : dl;
          dcur = dk;
        }
        const uint32_t c = min(b + lane, T - 1u);   // past T: re-read, dropped
        addr[u] = dl + 16ull * c;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v[u] = load_chunk<NT>(reinterpret_cast<gchunk_ptr>(addr[u]));
      }
    };
    auto consume = [&](uint32_t w0, const u32x4 (&v)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t b = w0 + 64u * u;
        const uint32_t val = b + lane < T ? chunk_value(v[u]) : 0u;
        const uint32_t r = wave_incl_scan(val) + run;
        // segments whose last chunk is in [b, b + 64): sum = R(end) - R(prev)
        while (pend_end) {
          const uint32_t k = uint32_t(__builtin_ctzll(pend_end));
          const uint32_t lk = __builtin_amdgcn_readlane(Lst, k);
          if (lk >= b + 64u) {
            break;
          }
          pend_end &= pend_end - 1;
          const uint32_t e = __builtin_amdgcn_readlane(r, lk - b);
          sum = lane == k ? e - eprev : sum;
          eprev = e;
        }
        run = __builtin_amdgcn_readlane(r, 63);
      }
    };
    if (T != 0) {
      // double-buffered: the next U windows are in flight while this batch is
      // scanned, so a wave with a long chunk list (a 9 KB segment among its
      // S) pays about half the round trips. The loop condition is
      // wave-uniform and both edges into its header carry exactly the U loads
      // of `cur`, so hipcc's vmcnt bookkeeping stays exact (vmcnt(U) before
      // scanning `cur`, no drain); the last batch is scanned after the loop
      // with nothing newer in flight.
      u32x4 cur[U];
      issue(0, cur);
      uint32_t w0 = 0;
      for (; w0 + 64u * U < T; w0 += 64u * U) {
        u32x4 nxt[U];
        issue(w0 + 64u * U, nxt);
        consume(w0, cur);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cur[u] = nxt[u];
        }
      }
      consume(w0, cur);
    }
    // ---- boundary bytes out, finish --------------------------------------
    const uint32_t outside =
      masked_value(cfirst, 0, head) + masked_value(clast, tail, 16);
    if (mine) {
      emit_with(seg, sum - outside, sa, len, side, out, bad, mode, nt_store);
    }
  }
}

template<int S, int U, bool NT>
hipError_t
launch_packed(const VarSegs& segs, const LaunchArgs& a, hipStream_t stream)
{
  const int block = a.block ? a.block : 256;
  const uint64_t per_block = uint64_t(block / 64) * S;
  uint64_t blocks = (uint64_t(a.n) + per_block - 1) / per_block;
  if (a.max_blocks && blocks > a.max_blocks) {
    blocks = a.max_blocks;
  }
  if (blocks == 0) {
    return hipSuccess;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL((csum_packed_kernel<S, U, NT>), dim3(uint32_t(blocks)),
                     dim3(block), 0, stream, segs, a.seeds, a.src, a.dst, a.out,
                     a.bad, a.n, a.mode, a.nt_store);
  return hipGetLastError();
}

template<int U, bool PRIO = false>
hipError_t
launch_span_u(const SpanArgs& sp, hipStream_t stream)
{
  constexpr uint64_t W = 4096ull * U;
  const uint64_t ranges = span_ranges(sp.base, sp.arena, W);
  if (ranges > 0x7fffffffull || ranges > sp.nslots) {
    return hipErrorInvalidValue;
  }
  (void)hipGetLastError();
  if constexpr (PRIO) {
    hipLaunchKernelGGL((csum_span_kernel<U, NoProbe, 8, 1024, U / 3, true, 256, 0, true>),
                       dim3(uint32_t(ranges)), dim3(256), 0, stream, sp, NoProbe{});
  } else {
    hipLaunchKernelGGL((csum_span_kernel<U>), dim3(uint32_t(ranges)), dim3(256), 0, stream,
                       sp, NoProbe{});
  }
  return hipGetLastError();
}

// The tail-shaped cut (group 9): ranges of U rows over the first
// (100 - tail_pct) % of the arena, then ranges of TR = U / 2 rows.
template<int U>
hipError_t
launch_span_tail(SpanArgs sp, uint32_t tail_pct, hipStream_t stream)
{
  constexpr int TR = U / 2;
  constexpr uint64_t W = 4096ull * U, WT = 4096ull * TR;
  const uint64_t hull = sp.arena + (reinterpret_cast<uintptr_t>(sp.base) & 15u);
  const uint64_t k1 = hull / 100 * (100 - tail_pct) / W;
  const uint64_t ranges = k1 + (hull - k1 * W) / WT + 1;
  if (ranges > 0x7fffffffull || ranges > sp.nslots) {
    return hipErrorInvalidValue;
  }
  sp.k1 = k1;
  (void)hipGetLastError();
  hipLaunchKernelGGL((csum_span_kernel<U, NoProbe, 8, 1024, U / 3, true, 256, TR>),
                     dim3(uint32_t(ranges)), dim3(256), 0, stream, sp, NoProbe{});
  return hipGetLastError();
}

template<int G, int U, bool NT, class Segs>
hipError_t
launch_one(const Segs& segs, const LaunchArgs& a, hipStream_t stream)
{
  const int block = a.block ? a.block : 256;
  const uint32_t per_block = uint32_t(block / G);
  uint64_t blocks = (uint64_t(a.n) + per_block - 1) / per_block;
  if (a.max_blocks && blocks > a.max_blocks) {
    blocks = a.max_blocks;
  }
  if (blocks == 0) {
    return hipSuccess;
  }
  (void)hipGetLastError(); // drop a stale error another runtime user left
  hipLaunchKernelGGL((csum_kernel<G, U, NT, Segs>), dim3(uint32_t(blocks)),
                     dim3(block), 0, stream, segs, a.seeds, a.src, a.dst,
                     a.out, a.bad, a.n, a.mode, a.nt_store);
  return hipGetLastError();
}

template<class Segs>
hipError_t
dispatch(const Segs& segs, const LaunchArgs& a, hipStream_t stream)
{
#define TCS_CASE(G_, U_)                                                       \
  if (a.group == G_ && a.unroll == U_) {                                       \
    return a.nontemporal ? launch_one<G_, U_, true>(segs, a, stream)           \
                         : launch_one<G_, U_, false>(segs, a, stream);         \
  }
  TCS_CASE(16, 2)
  TCS_CASE(16, 4)
  TCS_CASE(16, 8)
  TCS_CASE(32, 2)
  TCS_CASE(32, 3)
  TCS_CASE(32, 4)
  TCS_CASE(32, 8)
  TCS_CASE(64, 4)
  TCS_CASE(64, 8)
  TCS_CASE(64, 9)
  TCS_CASE(64, 10)
  TCS_CASE(64, 12)
#undef TCS_CASE
  return hipErrorInvalidValue;
}
} // namespace

hipError_t
launch_fixed(const uint8_t* base, uint64_t stride, uint32_t len,
             const LaunchArgs& a, hipStream_t stream)
{
  const FixedSegs segs{base, stride, len};
  return dispatch(segs, a, stream);
}

hipError_t
launch_var(const uint8_t* base, const uint64_t* offs, const uint16_t* lens,
           const LaunchArgs& a, hipStream_t stream)
{
  const VarSegs segs{base, offs, lens};
  if (a.kind == TULIPS_CSUM_KIND_PACKED) {
    // group = segments per wave, unroll = 64-chunk windows per batch
#define TCS_PCASE(S_, U_)                                                      \
  if (a.group == S_ && a.unroll == U_) {                                       \
    return a.nontemporal ? launch_packed<S_, U_, true>(segs, a, stream)        \
                         : launch_packed<S_, U_, false>(segs, a, stream);      \
  }
    TCS_PCASE(8, 2)
    TCS_PCASE(8, 4)
    TCS_PCASE(16, 2)
    TCS_PCASE(16, 4)
#undef TCS_PCASE
    return hipErrorInvalidValue;
  }
  return dispatch(segs, a, stream);
}

bool
span_geometry_ok(int u, int group)
{
  return ((group == 0 || group == 7) && u >= 4 && u <= 8) ||
         ((group == 9 || group == 10) && u >= 6 && u <= 8);
}

hipError_t
launch_span(const uint8_t* base, uint64_t arena, const uint64_t* offs,
            const uint16_t* lens, const LaunchArgs& a, hipStream_t stream)
{
  if (a.n == 0) {
    return hipSuccess;
  }
  SpanArgs sp{base, arena, offs, lens, a.seeds, a.src, a.dst, a.out, a.bad,
              a.n, a.mode, a.nt_store ? 1u : 0u, nullptr, 0, 0, a.offs_bias, 0};
  // the stream's per-range words, held for the launch
  std::shared_ptr<StreamState> ss;
  hipError_t e = stream_state(stream, &ss);
  if (e != hipSuccess) {
    return e;
  }
  std::lock_guard<std::recursive_mutex> g(ss->call);
  // (the tail-shaped cut has at most twice the ranges of the uniform one)
  const uint64_t ranges =
    span_ranges(base, arena, 4096ull * a.unroll) * (a.group == 9 ? 2 : 1);
  e = span_slots(*ss, stream_capturing(stream), ranges, &sp.slots, &sp.nslots, &sp.salt);
  if (e != hipSuccess) {
    return e == hipErrorStreamCaptureUnsupported ? hipErrorInvalidValue : e;
  }
  if (a.group == 9) {
    const uint32_t pct = a.spw > 0 && a.spw < 100 ? uint32_t(a.spw) : 12u;
    switch (a.unroll) {
      case 6: return launch_span_tail<6>(sp, pct, stream);
      case 7: return launch_span_tail<7>(sp, pct, stream);
      case 8: return launch_span_tail<8>(sp, pct, stream);
      default: return hipErrorInvalidValue;
    }
  }
  if (a.group == 10) { // measurement option: ranges prioritised by quarter
    switch (a.unroll) {
      case 6: return launch_span_u<6, true>(sp, stream);
      case 7: return launch_span_u<7, true>(sp, stream);
      case 8: return launch_span_u<8, true>(sp, stream);
      default: return hipErrorInvalidValue;
    }
  }
#define TCS_SCASE(U_)                                                          \
  if (a.unroll == U_) {                                                        \
    return launch_span_u<U_>(sp, stream);                                      \
  }
  TCS_SCASE(4)
  TCS_SCASE(5)
  TCS_SCASE(6)
  TCS_SCASE(7)
  TCS_SCASE(8)
#undef TCS_SCASE
  return hipErrorInvalidValue;
}

} // namespace tulips_amd
