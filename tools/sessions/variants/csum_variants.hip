// csum_variants.hip — the measured variants of rounds 1-2, kept OUTSIDE the
// product library (VERDICT r02 "kernel-variant sprawl"): hybrid short/long
// subgroups, the packed kernel's single-buffered and metadata-prefetch
// forms, lane-parallel cursors (vpacked), workgroup-balanced, and the span
// forms with halo rows (v1), boundary slots (v2) and staged chunks (v3),
// with the per-wave realtime stamps and the span diagnostic builds
// (TULIPS_SPAN_DIAG) they were measured with. DESIGN.md §4 records each
// one's numbers against the shipped kernels. Built by `make -C tools/variants`
// into tools/variants/libcsum_variants.so; the product never loads it.
//
// Entry points (same argument order as the library's *_tuned calls):
//   tulips_variant_batch_tuned        kinds HYBRID (2), PACKED (3, sps 1/3/4),
//                                     BALANCED (4)
//   tulips_variant_batch_arena_tuned  KIND_SPAN groups 1-6
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "../../include/tulips_csum.h"
#include "../../include/tulips_csum_util.h"
#include "../../tulips_amd/csrc/csum_common.h"
#include "../../tulips_amd/csrc/csum_device.h"
#include "../../tulips_amd/csrc/csum_launch.h"

#define TULIPS_CSUM_KIND_HYBRID 2
#define TULIPS_CSUM_KIND_BALANCED 4

namespace tulips_amd {
namespace {

#ifdef TULIPS_CSUM_STAMPS
// Diagnostic build only (tools/libcsum_stamps.so, tools/probe_stamps.py):
// every wave records {start, end, hw_id} of its life in 100 MHz realtime
// ticks. No product build defines TULIPS_CSUM_STAMPS.
__device__ uint64_t* g_stamps;
__device__ uint32_t g_stamp_count;

__device__ __forceinline__ void
stamp_wave(uint64_t t0)
{
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0 && g_stamps) {
    // wave index from the launch geometry: no atomic (it would serialise)
    const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (i == 0) {
      g_stamp_count = (gridDim.x * blockDim.x) >> 6;
    }
    // HW_REG_XCC_ID (20) bits [3:0]; HW_REG_HW_ID (4) all 32 bits
    const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11));
    const uint32_t hwid = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
    g_stamps[4 * i + 0] = t0;
    g_stamps[4 * i + 1] = t1;
    g_stamps[4 * i + 2] = xcc;
    g_stamps[4 * i + 3] = hwid;
  }
}

// The same with a mid-life stamp in place of the XCC id.
__device__ __forceinline__ void
stamp_wave_mid(uint64_t t0, uint64_t tm)
{
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0 && g_stamps) {
    const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (i == 0) {
      g_stamp_count = (gridDim.x * blockDim.x) >> 6;
    }
    g_stamps[4 * i + 0] = t0;
    g_stamps[4 * i + 1] = t1;
    g_stamps[4 * i + 2] = tm;
    g_stamps[4 * i + 3] = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
  }
}
#endif

// Variable-length batches with a long tail (Zipf, mean 668 B, 64 B..9 KB).
// One subgroup size cannot serve both a 64 B and a 9 KB segment, and a wave
// that owns one short segment per subgroup spends its life on two dependent
// round trips (metadata, then data) for a few hundred bytes — with 65,536
// segments the kernel is then bound by generations of short waves, not by
// bytes (tools/probe_zipf.py: ~7 us floor for 65,536 x 64 B). Here each wave
// owns SPW*SPS consecutive segments, SPW = 64/GS subgroups x SPS each:
//   phase 1: every segment of at most GS*US chunks is summed by its GS-lane
//            subgroup; the metadata of all SPS segments, then the US chunk
//            loads of all SPS segments, are issued before anything is
//            consumed (SPS*US loads in flight per lane, all unconditional);
//   phase 2: the wave's longer segments (found by a ballot) are summed one at
//            a time by all 64 lanes, UL loads per lane per batch.
template<int GS, int US, int UL, int SPS, bool NT>
__global__ __launch_bounds__(256) void
csum_hybrid_kernel(VarSegs segs, const uint16_t* __restrict__ seeds,
                   const uint32_t* __restrict__ src,
                   const uint32_t* __restrict__ dst, uint16_t* __restrict__ out,
                   uint32_t* __restrict__ bad, uint32_t n, uint32_t mode,
                   bool nt_store)
{
  constexpr int SPW = 64 / GS;
  constexpr int SEGS = SPW * SPS;
  const int lane64 = threadIdx.x & 63;
  const int lane = lane64 & (GS - 1);
  const int sub = lane64 / GS;
  const uint32_t wave = (xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  const uintptr_t base = reinterpret_cast<uintptr_t>(segs.base);
  const uintptr_t zero_chunk = reinterpret_cast<uintptr_t>(k_zero_chunk);
  for (uint32_t w0 = wave * SEGS; w0 < n; w0 += nwaves * SEGS) {
    uint32_t seg[SPS], len[SPS];
    uintptr_t sa[SPS];
    bool valid[SPS], is_long[SPS];
    SideIn side[SPS];
    u32x4 v[SPS][US];
#pragma unroll
    for (int k = 0; k < SPS; ++k) {
      seg[k] = w0 + uint32_t(k * SPW + sub);
      valid[k] = seg[k] < n;
      const uint32_t sk = valid[k] ? seg[k] : n - 1;
      len[k] = valid[k] ? segs.length(sk) : 0u;
      sa[k] = base + segs.off(sk);
      side[k] = load_side(sk, seeds, src, dst, mode);
    }
#pragma unroll
    for (int k = 0; k < SPS; ++k) {
      const uintptr_t a0 = sa[k] & ~uintptr_t(15);
      const int nch = len[k] ? int((sa[k] + len[k] - a0 + 15) >> 4) : 0;
      is_long[k] = nch > GS * US;
      // short and non-empty: its chunks; otherwise a harmless zero chunk
      const bool use = nch > 0 && !is_long[k];
      const uintptr_t p0 = use ? a0 : zero_chunk;
      const int last = use ? nch - 1 : 0;
#pragma unroll
      for (int u = 0; u < US; ++u) {
        v[k][u] = load_chunk<NT>(reinterpret_cast<gchunk_ptr>(p0) +
                                 min(lane + u * GS, last));
      }
    }
    uint32_t part[SPS];
#pragma unroll
    for (int k = 0; k < SPS; ++k) {
      const uintptr_t a0 = sa[k] & ~uintptr_t(15);
      const int nch = len[k] ? int((sa[k] + len[k] - a0 + 15) >> 4) : 0;
      const int last = nch - 1;
      const int head = int(sa[k] - a0);
      const int tail = int(sa[k] + len[k] - a0) - 16 * last;
      const bool use = nch > 0 && !is_long[k];
      uint64_t acc = 0;
#pragma unroll
      for (int u = 0; u < US; ++u) {
        const int cc = lane + u * GS;
        const uint64_t h = hsum(v[k][u]);
        acc += (use && cc <= last) ? h : 0;
        if (use && u == 0 && cc == 0 && head != 0) {
          acc -= masked_hsum(v[k][u], 0, head);
        }
        if (use && cc == last && tail != 16) {
          acc -= masked_hsum(v[k][u], tail, 16);
        }
      }
      part[k] = subgroup_sum<GS>(fold64(acc));
    }
    // phase 2: long segments, whole wave, one at a time
#pragma unroll
    for (int k = 0; k < SPS; ++k) {
      uint64_t longs = __ballot(is_long[k] && lane == 0);
      while (longs) {
        const int j = __ffsll(static_cast<unsigned long long>(longs)) - 1;
        longs &= longs - 1;
        const uint32_t lo = __builtin_amdgcn_readlane(uint32_t(sa[k]), j);
        const uint32_t hi = __builtin_amdgcn_readlane(uint32_t(sa[k] >> 32), j);
        const uint32_t llen = __builtin_amdgcn_readlane(len[k], j);
        const uintptr_t lsa = (uintptr_t(hi) << 32) | lo;
        const uint64_t lacc = lane_partial<64, UL, NT>(lsa, llen, lane64);
        const uint32_t lpart = subgroup_sum<64>(fold64(lacc));
        if (lane64 == j) {
          part[k] = lpart;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < SPS; ++k) {
      if (valid[k] && lane == 0) {
        emit_with(seg[k], part[k], sa[k], len[k], side[k], out, bad, mode,
                  nt_store);
      }
    }
  }
}

// Metadata of one segment (lane k < S of a wave owns segment g0 + k).
struct SegMeta
{
  uint32_t len;
  uint64_t off;
  SideIn side;
};

// PF: 0 = one batch of U windows at a time, 1 = double-buffered windows,
// 2 = double-buffered + the NEXT group's metadata loaded while this group's
// first windows are in flight (grid-stride waves; pays once a wave owns more
// than one group, i.e. with a capped grid).
template<int S, int U, bool NT, int PF>
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
#ifdef TULIPS_CSUM_STAMPS
  const uint64_t stamp0 = __builtin_amdgcn_s_memrealtime();
#endif
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
  SegMeta meta;
  if constexpr (PF == 2) {
    meta = load_meta(wave * S);
  }
  for (uint32_t g0 = wave * S; g0 < n; g0 += gstride) {
    if constexpr (PF != 2) {
      meta = load_meta(g0);
    }
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
    SegMeta next;
    if constexpr (PF == 0) {
      for (uint32_t w0 = 0; w0 < T; w0 += 64u * U) {
        u32x4 v[U];
        issue(w0, v);
        consume(w0, v);
      }
    } else if (T != 0) {
      // double-buffered: the next U windows are in flight while this batch is
      // scanned, so a wave with a long chunk list (a 9 KB segment among its
      // S) pays about half the round trips. The loop condition is
      // wave-uniform and both edges into its header carry exactly the U loads
      // of `cur`, so hipcc's vmcnt bookkeeping stays exact (vmcnt(U) before
      // scanning `cur`, no drain); the last batch is scanned after the loop
      // with nothing newer in flight.
      u32x4 cur[U];
      issue(0, cur);
      if constexpr (PF == 2) {
        // behind the first windows: arrives while they are scanned
        next = load_meta(g0 + gstride);
      }
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
    } else if constexpr (PF == 2) {
      next = load_meta(g0 + gstride);
    }
    // ---- boundary bytes out, finish --------------------------------------
    const uint32_t outside =
      masked_value(cfirst, 0, head) + masked_value(clast, tail, 16);
    if (mine) {
      emit_with(seg, sum - outside, sa, len, side, out, bad, mode, nt_store);
    }
    if constexpr (PF == 2) {
      meta = next;
    }
  }
#ifdef TULIPS_CSUM_STAMPS
  stamp_wave(stamp0);
#endif
}

template<int S, int U, bool NT, int PF>
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
  hipLaunchKernelGGL((csum_packed_kernel<S, U, NT, PF>), dim3(uint32_t(blocks)),
                     dim3(block), 0, stream, segs, a.seeds, a.src, a.dst, a.out,
                     a.bad, a.n, a.mode, a.nt_store);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// VPACKED: the packed kernel's chunk space with lane-parallel cursors.
//
// rocprofv3 counters of csum_packed_kernel on the §8c ZIPF batch
// (tools/pmc_var.sh): 462 VALU + 360 SALU instructions per wave for 5.3 KB,
// waves stalled on instruction issue 41 % of their life (SQ_WAIT_INST_ANY)
// vs 36 % on memory — with 8 waves per SIMD the launch is bound by issuing
// the two scalar cursors' per-segment loops, not by HBM. Here both cursors
// become a few vector instructions per 64-chunk window, whatever the number
// of segments in it:
//   * window -> address: lane j (chunk c = b + j) owns segment
//     s(c) = #{k : P_k <= c} - 1 (the starts P_k sit in SGPRs; an empty
//     segment shares its start with the next one and never wins), and takes
//     D_s with two ds_bpermutes: address = D_s + 16c;
//   * sums: the wave's running prefix R (inclusive scan, as before); lane k
//     captures e_k = R(its last chunk) with one ds_bpermute in the window
//     holding that chunk; after the last window sum_k = e_k - e_{k-1} (a DPP
//     shift; e_{-1} = 0, and an empty segment repeats its predecessor's e).
// Batches of U windows ping-pong between two register sets with every load
// unconditional (a batch past T re-reads chunk T - 1 and is dropped), so at
// each scan only the other set's U loads are newer (vmcnt(U)).
// ---------------------------------------------------------------------------
template<int S, int U, bool NT>
__global__ __launch_bounds__(256, 8) void
csum_vpacked_kernel(VarSegs segs, const uint16_t* __restrict__ seeds,
                    const uint32_t* __restrict__ src,
                    const uint32_t* __restrict__ dst, uint16_t* __restrict__ out,
                    uint32_t* __restrict__ bad, uint32_t n, uint32_t mode,
                    bool nt_store)
{
  static_assert(S >= 1 && S <= 32, "segment starts are held in SGPRs");
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(
    (xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x) >> 6);
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  const uintptr_t base = reinterpret_cast<uintptr_t>(segs.base);
  const uintptr_t zero_chunk = reinterpret_cast<uintptr_t>(k_zero_chunk);
#ifdef TULIPS_CSUM_STAMPS
  const uint64_t stamp0 = __builtin_amdgcn_s_memrealtime();
#endif
  for (uint32_t g0 = wave * S; g0 < n; g0 += nwaves * S) {
    const uint32_t seg = g0 + lane;
    const bool mine = lane < uint32_t(S) && seg < n;
    const uint32_t sk = mine ? seg : n - 1;
    const uint32_t len = mine ? segs.length(sk) : 0u;
    const uintptr_t sa = base + segs.off(sk);
    const SideIn side = load_side(sk, seeds, src, dst, mode);
    const uintptr_t a0 = sa & ~uintptr_t(15);
    const uint32_t nch = len ? uint32_t((sa + len - a0 + 15) >> 4) : 0u;
    const int head = int(sa - a0);
    const int tail = nch ? int(sa + len - a0) - 16 * int(nch - 1) : 16;
    const gchunk_ptr pf = reinterpret_cast<gchunk_ptr>(
      (nch && head != 0) ? a0 : zero_chunk);
    const gchunk_ptr pl = reinterpret_cast<gchunk_ptr>(
      (nch && tail != 16) ? a0 + 16 * uintptr_t(nch - 1) : zero_chunk);
    const u32x4 cfirst = load_chunk<NT>(pf);
    const u32x4 clast = load_chunk<NT>(pl);
    // ---- packed chunk space ------------------------------------------------
    const uint32_t incl = wave_incl_scan(nch);
    const uint32_t P = incl - nch;
    const uint32_t T = __builtin_amdgcn_readlane(incl, 63);
    const uint32_t Lst = incl - 1;
    const uint64_t D = uint64_t(a0) - 16ull * P;
    const int dlo = int(uint32_t(D)), dhi = int(uint32_t(D >> 32));
    uint32_t ps[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
      ps[k] = __builtin_amdgcn_readlane(P, k);
    }
    uint32_t run = 0;
    uint32_t e = 0; // R at this lane's segment's last chunk
    auto issue = [&](uint32_t w0, u32x4 (&v)[U]) {
      uint64_t addr[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t c = min(w0 + 64u * u + lane, T - 1u); // past T: re-read
        uint32_t sidx = 0;
#pragma unroll
        for (int k = 1; k < S; ++k) {
          sidx += c >= ps[k] ? 1u : 0u;
        }
        const uint32_t lo = uint32_t(__builtin_amdgcn_ds_bpermute(int(sidx << 2), dlo));
        const uint32_t hi = uint32_t(__builtin_amdgcn_ds_bpermute(int(sidx << 2), dhi));
        addr[u] = ((uint64_t(hi) << 32) | lo) + 16ull * c;
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
        const uint32_t at = Lst - b;                 // wraps when outside
        const uint32_t rv = uint32_t(__builtin_amdgcn_ds_bpermute(int(at << 2), int(r)));
        e = at < 64u ? rv : e;
        run = __builtin_amdgcn_readlane(r, 63);
      }
    };
    if (T != 0) {
      // pairs of batches, nothing in flight across a loop edge or a join
      // (see csum_balanced_kernel)
      u32x4 A[U];
      issue(0, A);
      if (64u * U < T) {
        u32x4 Bf[U];
        issue(64u * U, Bf);
        consume(0, A);
        consume(64u * U, Bf);
        for (uint32_t w0 = 128u * U; w0 < T; w0 += 128u * U) {
          issue(w0, A);
          issue(w0 + 64u * U, Bf);
          consume(w0, A);
          if (w0 + 64u * U < T) {
            consume(w0 + 64u * U, Bf);
          }
        }
      } else {
        consume(0, A);
      }
    }
    // sum_k = e_k - e_{k-1}: lane k - 1's value one lane up (row_shr:1 within
    // each row of 16, then the row boundary lanes from readlane)
    uint32_t eprev = uint32_t(__builtin_amdgcn_update_dpp(0, int(e), 0x111, 0xf, 0xf, false));
    if constexpr (S > 16) {
      const uint32_t e15 = __builtin_amdgcn_readlane(e, 15);
      eprev = lane == 16 ? e15 : eprev;
    }
    const uint32_t sum = e - eprev;
    const uint32_t outside =
      masked_value(cfirst, 0, head) + masked_value(clast, tail, 16);
    if (mine) {
      emit_with(seg, sum - outside, sa, len, side, out, bad, mode, nt_store);
    }
  }
#ifdef TULIPS_CSUM_STAMPS
  stamp_wave(stamp0);
#endif
}

template<int S, int U, bool NT>
hipError_t
launch_vpacked(const VarSegs& segs, const LaunchArgs& a, hipStream_t stream)
{
  const uint64_t per_block = uint64_t(256 / 64) * S;
  uint64_t blocks = (uint64_t(a.n) + per_block - 1) / per_block;
  if (a.max_blocks && blocks > a.max_blocks) {
    blocks = a.max_blocks;
  }
  if (blocks == 0) {
    return hipSuccess;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL((csum_vpacked_kernel<S, U, NT>), dim3(uint32_t(blocks)), dim3(256), 0,
                     stream, segs, a.seeds, a.src, a.dst, a.out, a.bad, a.n, a.mode,
                     a.nt_store);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// BALANCED variable-length kernel: the packed chunk space of a whole
// WORKGROUP, split evenly over its waves.
//
// With one wave per 8 Zipf segments the launch lasts as long as its heaviest
// wave: the sum of 8 draws reaches 28.8 KB against a 5.3 KB mean, and such a
// wave needs 4-5 dependent batches after the bulk of the chip's requests has
// drained (the latency-bound tail of csum_packed_kernel). Here a workgroup of
// NW waves owns 8*NW consecutive segments; their chunk lists are laid end to
// end in one workgroup packed space of TB chunks, and wave w reads chunks
// [w*TB/NW, (w+1)*TB/NW) with the packed kernel's window machinery. The
// heaviest wave drops to 16.0 KB (NW = 4) / 10.6 KB (NW = 8) for the §8c Zipf
// batch. A segment cut by a range boundary gets its partial sums from two or
// more waves; they meet in LDS (one ds_add per touched segment per wave).
//
//   1. lane k < 8 of wave w: metadata of segment 8w + k, its boundary chunks
//      (as the packed kernel), nch / chunk base into LDS, its LDS sum zeroed;
//   2. barrier; every wave reads the workgroup's table (lane j = segment j,
//      8*NW <= 64) and scans it (P_j, D_j = chunkbase_j - 16*P_j, last chunk);
//   3. wave w walks its range in 64-chunk windows, U windows per batch,
//      double-buffered; per-segment prefix differences as in the packed
//      kernel; the open segment at the range end takes run - eprev;
//   4. each lane adds its segment's partial to LDS; barrier; lane k < 8 of
//      wave w takes out the boundary bytes and emits segment 8w + k.
// ---------------------------------------------------------------------------
// 8 waves per SIMD (= 32 per CU, the whole grid of a 65,536-segment batch
// resident at once): the register budget is 64 VGPRs
template<int NW, int U, bool NT, int PF>
__global__ __launch_bounds__(64 * NW, 8) void
csum_balanced_kernel(VarSegs segs, const uint16_t* __restrict__ seeds,
                     const uint32_t* __restrict__ src,
                     const uint32_t* __restrict__ dst, uint16_t* __restrict__ out,
                     uint32_t* __restrict__ bad, uint32_t n, uint32_t mode,
                     bool nt_store)
{
  constexpr uint32_t S = 8, B = S * NW;
  static_assert(B <= 64, "the workgroup table lives in one wave's lanes");
  // the table, and what the owners need back at the end (held in LDS, not in
  // VGPRs, across the window loop: 8 waves per SIMD leave 64 VGPRs)
  __shared__ uint32_t s_nch[B];
  __shared__ uint64_t s_a0[B];
  __shared__ uint32_t s_sum[B];
  __shared__ uint32_t s_len[B];   // length | start-odd << 16
  __shared__ uint32_t s_out[B];   // boundary bytes outside the segment
  __shared__ SideIn s_side[B];
  const uint32_t lane = threadIdx.x & 63;
  // wave index as a scalar: the range [r0, r1) and the window loop derived
  // from it must be wave-uniform (SGPRs), or hipcc builds an exec-masked loop
  // whose buffer rotation waits for every load (vmcnt(0)) each iteration
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uintptr_t base = reinterpret_cast<uintptr_t>(segs.base);
  const uintptr_t zero_chunk = reinterpret_cast<uintptr_t>(k_zero_chunk);
#ifdef TULIPS_CSUM_STAMPS
  const uint64_t stamp0 = __builtin_amdgcn_s_memrealtime();
#endif
  for (uint32_t blk = xcd_block(blockIdx.x, gridDim.x); blk * B < n; blk += gridDim.x) {
    // ---- 1. own segments' metadata ----------------------------------------
    // (lds_barrier() waits for every outstanding load of the wave, so
    // nothing but the metadata may be in flight at the barrier: the boundary
    // chunks are loaded after it, in front of the first windows)
    gchunk_ptr pf, pl;
    int head, tail;
    {
      const uint32_t seg = blk * B + w * S + lane;
      const bool mine = lane < S && seg < n;
      const uint32_t sk = mine ? seg : n - 1;
      const uint32_t len = mine ? segs.length(sk) : 0u;
      const uintptr_t sa = base + segs.off(sk);
      const SideIn side = load_side(sk, seeds, src, dst, mode);
      const uintptr_t a0 = sa & ~uintptr_t(15);
      const uint32_t nch = len ? uint32_t((sa + len - a0 + 15) >> 4) : 0u;
      head = int(sa - a0);
      tail = nch ? int(sa + len - a0) - 16 * int(nch - 1) : 16;
      pf = reinterpret_cast<gchunk_ptr>((nch && head != 0) ? a0 : zero_chunk);
      pl = reinterpret_cast<gchunk_ptr>(
        (nch && tail != 16) ? a0 + 16 * uintptr_t(nch - 1) : zero_chunk);
      if (lane < S) {
        const uint32_t j = w * S + lane;
        s_nch[j] = nch;
        s_a0[j] = uint64_t(a0);
        s_sum[j] = 0u;
        s_len[j] = len | (uint32_t(sa & 1) << 16);
        s_side[j] = side;
      }
    }
    lds_barrier();
    // ---- 2. the workgroup's packed space ----------------------------------
    const uint32_t tn = lane < B ? s_nch[lane] : 0u;
    const uint32_t incl = wave_incl_scan(tn);
    const uint32_t P = incl - tn;
    const uint32_t TB = __builtin_amdgcn_readlane(incl, 63);
    const uint32_t Lst = incl - 1;
    const uint64_t D = (lane < B ? s_a0[lane] : 0ull) - 16ull * P;
    const uint32_t r0 = uint32_t((uint64_t(TB) * w) / NW);
    const uint32_t r1 = uint32_t((uint64_t(TB) * (w + 1)) / NW);
    // segments that end inside or after this range, in packed order
    const uint64_t live = __ballot(tn != 0 && incl > r0);
    uint64_t pend_start = live, pend_end = live;
    uint64_t dcur = uint64_t(zero_chunk);
    uint32_t run = 0, eprev = 0;
    uint32_t part = 0;                               // this wave's share, lane j
    auto issue = [&](uint32_t w0, u32x4 (&v)[U]) {
      uint64_t addr[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t b = w0 + 64u * u;
        uint64_t dl = dcur;
        while (pend_start) {
          const uint32_t k = uint32_t(__builtin_ctzll(pend_start));
          const uint32_t pk = __builtin_amdgcn_readlane(P, k);
          // segments starting at r1 or later belong to the next wave: their
          // D must not reach the lanes clamped to chunk r1 - 1
          if (pk >= b + 64u || pk >= r1) {
            break;
          }
          pend_start &= pend_start - 1;
          const uint64_t dk = readlane64(D, k);
          dl = lane + b >= pk ? dk : dl;
          dcur = dk;
        }
        const uint32_t c = min(b + lane, r1 - 1u);  // past r1: re-read, dropped
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
        const uint32_t val = b + lane < r1 ? chunk_value(v[u]) : 0u;
        const uint32_t r = wave_incl_scan(val) + run;
        while (pend_end) {
          const uint32_t k = uint32_t(__builtin_ctzll(pend_end));
          const uint32_t lk = __builtin_amdgcn_readlane(Lst, k);
          if (lk >= b + 64u || lk >= r1) {
            break;
          }
          pend_end &= pend_end - 1;
          const uint32_t e = __builtin_amdgcn_readlane(r, lk - b);
          part = lane == k ? e - eprev : part;
          eprev = e;
        }
        run = __builtin_amdgcn_readlane(r, 63);
      }
    };
    // the boundary chunks are older than the windows: their outside bytes
    // are taken right after the first batch is issued (vmcnt(U)), so they do
    // not occupy 8 VGPRs through the loop
    const u32x4 cfirst = load_chunk<NT>(pf);
    const u32x4 clast = load_chunk<NT>(pl);
    auto retire_boundary = [&]() {
      if (lane < S) {
        s_out[w * S + lane] =
          masked_value(cfirst, 0, head) + masked_value(clast, tail, 16);
      }
    };
    if (r1 > r0) {
      // Pairs of batches: A and B (U windows each) are issued back to back
      // and scanned in order, so A's scan waits vmcnt(U) while B is still in
      // flight; no load is in flight across a loop edge or a branch join (a
      // loop-carried buffer made hipcc wait for every load at the loop
      // header). A wave's range of up to 2U windows costs one round trip.
      u32x4 A[U];
      issue(r0, A);
      retire_boundary();
      if (r0 + 64u * U < r1) {
        u32x4 Bf[U];
        issue(r0 + 64u * U, Bf);
        consume(r0, A);
        consume(r0 + 64u * U, Bf);
        for (uint32_t w0 = r0 + 128u * U; w0 < r1; w0 += 128u * U) {
          issue(w0, A);
          issue(w0 + 64u * U, Bf);   // past r1: re-reads chunk r1 - 1, dropped
          consume(w0, A);
          if (w0 + 64u * U < r1) {
            consume(w0 + 64u * U, Bf);
          }
        }
      } else {
        consume(r0, A);
      }
    } else {
      retire_boundary();
    }
    // the segment still open at the range end continues in the next wave
    if (r1 > r0 && pend_end) {
      const uint32_t k = uint32_t(__builtin_ctzll(pend_end));
      if (uint32_t(__builtin_amdgcn_readlane(P, k)) < r1) {
        part = lane == k ? run - eprev : part;
      }
    }
    // ---- 4. partials meet in LDS; owners finish -----------------------------
    if (lane < B && part != 0u) {
      atomicAdd(&s_sum[lane], part);
    }
    lds_barrier();
    {
      const uint32_t j = w * S + lane;
      const uint32_t seg = blk * B + j;
      if (lane < S && seg < n) {
        const uint32_t lw = s_len[j];
        // emit_with reads only the start's parity from the address
        emit_with(seg, s_sum[j] - s_out[j], uintptr_t(lw >> 16), lw & 0xffffu, s_side[j],
                  out, bad, mode, nt_store);
      }
    }
    if (blk + gridDim.x < (n + B - 1) / B) {
      lds_barrier(); // the table is rewritten by the next iteration
    }
  }
#ifdef TULIPS_CSUM_STAMPS
  stamp_wave(stamp0);
#endif
}

template<int NW, int U, bool NT, int PF>
hipError_t
launch_balanced(const VarSegs& segs, const LaunchArgs& a, hipStream_t stream)
{
  constexpr uint64_t B = 8 * NW;
  uint64_t blocks = (uint64_t(a.n) + B - 1) / B;
  if (a.max_blocks && blocks > a.max_blocks) {
    blocks = a.max_blocks;
  }
  if (blocks == 0) {
    return hipSuccess;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL((csum_balanced_kernel<NW, U, NT, PF>), dim3(uint32_t(blocks)),
                     dim3(64 * NW), 0, stream, segs, a.seeds, a.src, a.dst, a.out, a.bad,
                     a.n, a.mode, a.nt_store);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// SPAN: in-order arenas (tulips_csum_batch_arena), work cut by BYTES.
//
// Every kernel above hands each wave (or workgroup) a fixed number of
// segments, so its life is a chain of dependent round trips whose length
// follows the bytes it drew: on the Zipf batch the heaviest waves (28.8 KB
// for 8 segments) end ~8 us after the median one whatever the grid does
// (tools/probe_stamps_small.py; floor of ~8 us even at n = 1024). When the
// segments lie in order in one arena, the byte range of the arena itself can
// be cut instead: workgroup k owns the 16-byte-aligned range
// [A + kW, A + (k+1)W), W = 4 KiB * U, and
//   * its 4 waves load the range plus a 4 KiB halo past its end at once
//     (U + 1 chunks per lane, one round trip), stage the range's chunks in
//     LDS and scan their 16-bit-half sums into an LDS prefix P;
//   * the segments STARTING in the range,
//     [lo, hi) = [first s: off_s >= kW - d, first s: off_s >= (k+1)W - d),
//     come from a 1024-entry window of offsets/lengths loaded in the same
//     round trip, BEFORE the chunks (vmcnt retires in order), where an evenly
//     filled arena puts them (n * range middle / arena bytes); on the Zipf
//     batch it brackets [lo, hi) for all but 0.1 % of the ranges. Otherwise
//     wave 0 finds lo and hi by a 256-ary search (a few more round trips);
//   * segment s in [lo, hi) (one per thread) is a prefix difference plus its
//     two masked boundary chunks, all from LDS. Only hi - 1 can run past the
//     range: the workgroup sums its bytes in the halo (still in registers)
//     and past the halo (a tail > 4 KiB: one more round trip, taken only
//     when such a tail exists).
// Segment s is finished by the one workgroup its first byte falls in, so no
// partial crosses workgroups and no workspace or atomic is needed. A
// workgroup's life is one round trip + LDS work; its bytes are fixed by
// construction.
// Contract (include/tulips_csum.h): offsets[i] + lengths[i] <= offsets[i+1]
// and offsets[n-1] + lengths[n-1] <= arena_bytes. Every access is clamped
// into the arena, so a batch breaking the contract gets wrong results but no
// access outside [base & ~15, (base + arena_bytes + 15) & ~15).
// ---------------------------------------------------------------------------
template<int U, int HR, bool NT>
__global__ __launch_bounds__(256) void
csum_span_kernel(SpanArgs p)
{
  constexpr uint32_t R = U + HR;         // rows of 256 chunks: range + halo
  constexpr uint32_t NC = 256u * U;      // chunks per range
  constexpr uint64_t W = 16ull * NC;     // bytes per range
  constexpr uint32_t NWIN = 1024;        // speculative window entries
  constexpr int UE = 4;                  // tail chunks per thread per batch
  constexpr int UH = 6;                  // HR = 0: crossing tail chunks per lane
  __shared__ u32x4 s_raw[256 * R];       // the range's and the halo's chunks
  __shared__ uint32_t s_sc[256 * R];     // row-wise wave scans of chunk values
  __shared__ uint32_t s_tot[4 * R];      // per (row, wave) scan totals
  __shared__ uint32_t s_woff[4][4 * R];  // each wave's copy of their exclusive prefix
  __shared__ uint32_t s_cnt[12];         // per wave: window counts, tail flag
  __shared__ uint64_t s_meta[4];         // end of a segment past the halo; search
  __shared__ uint32_t s_ext[4];

  const uint32_t t = threadIdx.x, lane = t & 63u;
  const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6);
  const uint32_t k = xcd_block(blockIdx.x, gridDim.x);
  const uintptr_t b = reinterpret_cast<uintptr_t>(p.base);
  const uint64_t d = b & 15u;
  const uintptr_t x0 = (b & ~uintptr_t(15)) + uint64_t(k) * W, x1 = x0 + W;
  const uintptr_t xe = x1 + 16u * 256u * HR; // end of the halo
  const uintptr_t aend = b + p.arena;
  const uintptr_t zero = reinterpret_cast<uintptr_t>(k_zero_chunk);
  const uintptr_t last = p.arena ? ((aend - 1) & ~uintptr_t(15)) : zero;
  const uint32_t n = p.n;
  const gu64_ptr offs = reinterpret_cast<gu64_ptr>(reinterpret_cast<uintptr_t>(p.offs));
  const gu16_ptr lens = reinterpret_cast<gu16_ptr>(reinterpret_cast<uintptr_t>(p.lens));
  // lo = first s with off_s >= tg0, hi = first s with off_s >= tg1
  const uint64_t tg0 = k ? uint64_t(k) * W - d : 0, tg1 = uint64_t(k + 1) * W - d;
#ifdef TULIPS_CSUM_STAMPS
  const uint64_t stamp0 = __builtin_amdgcn_s_memrealtime();
#endif

  // 1. one round trip: the offsets/lengths window where an evenly filled
  //    arena would put this range's segments, then the range + halo chunks
  //    (window first: vmcnt retires in order, so its wait never waits for
  //    the chunks)
  const uint64_t mid = (tg0 + tg1) / 2;
  const uint64_t guess = uint64_t(double(n) * double(mid) / double(p.arena ? p.arena : 1));
  const uint32_t gmax = n > NWIN ? n - NWIN : 0u;
  const uint32_t G = uint32_t(min(guess > NWIN / 2 ? guess - NWIN / 2 : 0ull, uint64_t(gmax)));
  uint64_t wo[4];
  uint32_t wl[4];
#if TULIPS_SPAN_DIAG == 1
  // diagnostic build (tools/libcsum_spandiag1.so): no offsets window
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    wo[r] = G + t + 256u * r;
    wl[r] = 0;
  }
#else
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t i = min(G + t + 256u * r, n - 1);
    wo[r] = offs[i];
    wl[r] = lens[i];
  }
#endif
  // Rows read twice (this range's first HR rows are the previous range's
  // halo, the last HR rows are this range's) are loaded temporal so that the
  // second read, by the neighbouring workgroup, hits L2; the rest streams.
  u32x4 v[R];
#pragma unroll
  for (uint32_t j = 0; j < R; ++j) {
    const uintptr_t a = x0 + 16u * (j * 256u + t);
    const gchunk_ptr q = reinterpret_cast<gchunk_ptr>(p.arena ? min(a, last) : zero);
    v[j] = (j < HR || j >= U) ? load_chunk<false>(q) : load_chunk<NT>(q);
  }
  // every load is out before the first wait: without this fence the
  // scheduler pulls the window's first uses between the chunk loads, and the
  // vmcnt waits they bring hold the remaining chunk loads back for a whole
  // round trip
  __builtin_amdgcn_sched_barrier(0);
  // HR = 0: the segment crossing the range end (at most one, in order) is
  // found in the window by the wave holding its entry, which loads and sums
  // its bytes past the range itself, as soon as the window is in: no halo
  // rows, no re-read bytes, no extra barrier.
  int hold = -1;          // this thread's entry of the crossing segment
  uint32_t xsum = 0;      // HR = 0: the crossing wave's sum past the range
  uintptr_t hte = 0;      // HR = 0: the crossing segment's end
  u32x4 hv[HR == 0 ? UH : 1];
  {
    // window counts below each target, and whether an entry starting in
    // the range runs past the halo (at most one can, in order)
    uint32_t c0 = 0, c1 = 0;
    bool far = false;
    uintptr_t myte = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool in = G + t + 256u * r < n;
      c0 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in && wo[r] < tg0));
      c1 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in && wo[r] < tg1));
      const uintptr_t sa = b + wo[r], se = min(b + wo[r] + wl[r], aend);
      if (in && sa >= x0 && sa < x1 && se > xe) {
        far = true;
        hold = r;
        myte = se;
        if (HR > 0) {
          s_meta[3] = se;
        }
      }
    }
    const uint64_t fb = __builtin_amdgcn_ballot_w64(far);
    if (lane == 0) {
      s_cnt[w] = c0;
      s_cnt[4 + w] = c1;
      s_cnt[8 + w] = HR > 0 && fb != 0;
    }
    if constexpr (HR == 0) {
      if (fb != 0) {
        const uint32_t lc = uint32_t(__builtin_ctzll(fb));
        hte = uintptr_t(readlane64(uint64_t(myte), lc));
        hold = lane == lc ? hold : -1;
        const uint32_t nh = uint32_t((hte - x1 + 15) >> 4);
        const uintptr_t hl = x1 + 16u * (nh - 1);
#pragma unroll
        for (int q = 0; q < UH; ++q) {
          const uint32_t c = lane + 64u * q;
          hv[q] = load_chunk<NT>(reinterpret_cast<gchunk_ptr>(c < nh ? x1 + 16u * c : hl));
        }
      } else {
        hold = -1;
      }
    }
  }
  // 2. chunks to LDS with the row-wise wave scans of their values
#pragma unroll
  for (uint32_t j = 0; j < R; ++j) {
    s_raw[j * 256u + t] = v[j];
    const uint32_t sc = wave_incl_scan(chunk_value(v[j]));
    s_sc[j * 256u + t] = sc;
    if (lane == 63) {
      s_tot[4 * j + w] = sc;
    }
  }
  if constexpr (HR == 0) {
    // the crossing wave sums its tail past the range (first UH * 64 chunks
    // already in flight, any rest in further batches)
    if (hte > x1) {
      const uint32_t nh = uint32_t((hte - x1 + 15) >> 4);
      const uintptr_t hl = x1 + 16u * (nh - 1);
      const int tb = int(hte - x1) - 16 * int(nh - 1);
      uint32_t ts = 0;
#pragma unroll
      for (int q = 0; q < UH; ++q) {
        const uint32_t c = lane + 64u * q;
        ts += c + 1 < nh ? chunk_value(hv[q]) : (c + 1 == nh ? masked_value(hv[q], 0, tb) : 0u);
      }
      for (uint32_t c0 = 64u * UH; c0 < nh; c0 += 64u * UH) {
#pragma unroll
        for (int q = 0; q < UH; ++q) {
          const uint32_t c = c0 + lane + 64u * q;
          hv[q] = load_chunk<NT>(reinterpret_cast<gchunk_ptr>(c < nh ? x1 + 16u * c : hl));
        }
#pragma unroll
        for (int q = 0; q < UH; ++q) {
          const uint32_t c = c0 + lane + 64u * q;
          ts += c + 1 < nh ? chunk_value(hv[q])
                           : (c + 1 == nh ? masked_value(hv[q], 0, tb) : 0u);
        }
      }
      xsum = __builtin_amdgcn_readlane(wave_incl_scan(ts), 63);
    }
  }
  lds_barrier();
#ifdef TULIPS_CSUM_STAMPS
  const uint64_t stamp_mid = __builtin_amdgcn_s_memrealtime();
#endif
#if defined(TULIPS_SPAN_DIAG) && TULIPS_SPAN_DIAG > 0 && TULIPS_SPAN_DIAG < 4
  // diagnostic builds: stop after the chunks are staged and scanned
  if (t == 0 && p.out && k < n) {
    p.out[k] = uint16_t(s_tot[0] + s_cnt[0] + s_sc[5]);
  }
  return;
#endif

  // 3. this wave's copy of the (row, wave) offsets: inclusive prefix of
  //    chunk c = s_woff[c >> 6] + s_sc[c]
  {
    const uint32_t x = lane < 4 * R ? s_tot[lane] : 0u;
    const uint32_t inc = wave_incl_scan(x);
    if (lane < 4 * R) {
      s_woff[w][lane] = inc - x;
    }
  }
#if TULIPS_SPAN_DIAG == 4
  // diagnostic build: stop before the segment pass
  if (t == 0 && p.out && k < n) {
    p.out[k] = uint16_t(s_woff[w][1] + s_cnt[0] + s_sc[5]);
  }
  return;
#endif
  auto P = [&](uint32_t c) { return s_woff[w][c >> 6] + s_sc[c]; };
  const uint32_t c0 = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
  const uint32_t c1 = s_cnt[4] + s_cnt[5] + s_cnt[6] + s_cnt[7];
  const bool tail = (s_cnt[8] | s_cnt[9] | s_cnt[10] | s_cnt[11]) != 0;
  const uint32_t nw = min(NWIN, n - G);
  const bool tail_ok = G + NWIN >= n;
  const bool ok = (c0 > 0 || G == 0) && (c0 < nw || tail_ok) && (c1 > 0 || G == 0) &&
                  (c1 < nw || tail_ok);

  // 4. rare: a segment runs past the halo (> 4 KiB * HR beyond the range):
  //    the workgroup sums its bytes past the halo in one more round trip
  auto tail_sum = [&](uintptr_t te) {
    const uint32_t tch = uint32_t((te - xe + 15) >> 4);
    const uintptr_t tlast = xe + 16u * (tch - 1);
    const int tbytes = int(te - xe) - 16 * int(tch - 1);
    uint32_t tsum = 0;
    for (uint32_t q0 = 0; q0 < tch; q0 += 256u * UE) {
      u32x4 e[UE];
#pragma unroll
      for (int j = 0; j < UE; ++j) {
        const uint32_t c = q0 + t + 256u * j;
        e[j] = load_chunk<NT>(reinterpret_cast<gchunk_ptr>(c < tch ? xe + 16u * c : tlast));
      }
#pragma unroll
      for (int j = 0; j < UE; ++j) {
        const uint32_t c = q0 + t + 256u * j;
        tsum += c + 1 < tch ? chunk_value(e[j])
                            : (c + 1 == tch ? masked_value(e[j], 0, tbytes) : 0u);
      }
    }
    tsum = wave_incl_scan(tsum);
    if (lane == 63) {
      s_ext[w] = tsum;
    }
    lds_barrier();
    return s_ext[0] + s_ext[1] + s_ext[2] + s_ext[3];
  };
  uint32_t ext = 0;

  // 5. one segment: prefix differences over [x0, xe) plus the tail
  const uint32_t want = (p.mode & FLAG_COMPLEMENT) ? 0u : 0xffffu;
  const bool side_in = (p.mode & MODE_MASK) == MODE_TCP || p.seeds != nullptr;
  auto emit = [&](uint32_t s, bool mine, uint64_t so, uint32_t sl, uint32_t ext) {
    SideIn side{0, 0, 0};
    if (side_in) {
      side = load_side(mine ? s : 0u, p.seeds, p.src, p.dst, p.mode);
    }
    const uintptr_t sa = min(max(b + so, x0), x1 - 1);
    const uintptr_t se = min(b + so + sl, aend);
    const uintptr_t ie = min(se, xe);
    uint32_t sum = 0;
    if (ie > sa) {
      const uint32_t ca = uint32_t((sa - x0) >> 4);
      const uint32_t ce = uint32_t((ie - 1 - x0) >> 4);
      const int ha = int(sa & 15u), tb = int(((ie - 1) & 15u) + 1u);
      sum = ca == ce ? masked_value(s_raw[ca], ha, tb)
                     : masked_value(s_raw[ca], ha, 16) + (P(ce - 1) - P(ca)) +
                         masked_value(s_raw[ce], 0, tb);
    }
    sum += se > xe ? ext : 0u;
    const uint32_t r =
      finish(sum, (sa & 1u) != 0, p.mode, side.seed, side.src, side.dst, sl);
#if TULIPS_SPAN_DIAG == 5
    if (mine && p.out && r == 0x1234567u) {
#else
    if (mine && p.out) {
#endif
#if TULIPS_SPAN_DIAG == 6
      // diagnostic build: each workgroup's results to its own 256-byte block
      // (wrong layout; only the store pattern differs)
      p.out[(k * 128u + (s & 127u)) % n] = uint16_t(r);
#else
      if (p.nt_store) {
        __builtin_nontemporal_store(uint16_t(r), p.out + s);
      } else {
        p.out[s] = uint16_t(r);
      }
#endif
    }
    if (p.bad) {
      const uint32_t nb =
        __builtin_popcountll(__builtin_amdgcn_ballot_w64(mine && r != want));
      if (lane == 0 && nb) {
        atomicAdd(p.bad + CNT_LINE * (blockIdx.x % CNT_SHARDS), nb);
      }
    }
  };

  if (ok) {
    // the window brackets [lo, hi): each thread finishes the segments whose
    // metadata it loaded
    const uint32_t lo = G + c0, hi = G + c1;
    if (tail) {
      ext = tail_sum(s_meta[3]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t i = G + t + 256u * r;
      const bool mine = i >= lo && i < hi;
      if (__builtin_amdgcn_ballot_w64(mine) != 0) {
        emit(i, mine, mine ? wo[r] : 0, mine ? wl[r] : 0u, HR == 0 ? (hold == r ? xsum : 0u)
                                                                     : ext);
      }
    }
  } else {
    // rare: wave 0 searches [lo, hi); segments' metadata from memory
    if (w == 0) {
      uint32_t L0 = 0, R0 = n, L1 = 0, R1 = n;
      while (R0 > L0 || R1 > L1) {
        const uint32_t st0 = (R0 - L0 + 255u) >> 8, st1 = (R1 - L1 + 255u) >> 8;
        uint64_t o0[4], o1[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t q = lane + 64u * r;
          o0[r] = offs[min(uint64_t(L0) + uint64_t(q) * st0, uint64_t(n - 1))];
          o1[r] = offs[min(uint64_t(L1) + uint64_t(q) * st1, uint64_t(n - 1))];
        }
        uint32_t d0 = 0, d1 = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t q = lane + 64u * r;
          const bool in0 = uint64_t(L0) + uint64_t(q) * st0 < R0;
          const bool in1 = uint64_t(L1) + uint64_t(q) * st1 < R1;
          d0 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in0 && o0[r] < tg0));
          d1 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in1 && o1[r] < tg1));
        }
        if (R0 > L0) {
          span_narrow(L0, R0, st0, __builtin_amdgcn_readfirstlane(d0));
        }
        if (R1 > L1) {
          span_narrow(L1, R1, st1, __builtin_amdgcn_readfirstlane(d1));
        }
      }
      if (lane == 0) {
        s_meta[0] = L0;
        s_meta[1] = L1;
      }
    }
    lds_barrier();
    const uint32_t lo = uint32_t(s_meta[0]), hi = uint32_t(s_meta[1]);
    if (hi > lo) {
      const uintptr_t te = min(b + p.offs[hi - 1] + p.lens[hi - 1], aend);
      if (te > xe) {
        ext = tail_sum(te);
      }
    }
    for (uint32_t s0 = lo; s0 < hi; s0 += 256u) {
      const uint32_t s = s0 + t;
      const bool mine = s < hi;
      emit(s, mine, mine ? p.offs[s] : 0, mine ? p.lens[s] : 0u, ext);
    }
  }
#ifdef TULIPS_CSUM_STAMPS
  stamp_wave_mid(stamp0, stamp_mid);
#endif
}

// SPAN, boundary-slot form (`group` 4/5 = halo rows 2/1): the same work
// cut, but only the chunks a segment boundary falls in are staged in LDS.
// The holder of a segment's window entry knows its first and last chunk as
// soon as the window is in (before the range's data): it marks them in a
// per-chunk word (head slot in the low half, tail slot in the high half,
// slot = window index mod 128); after one barrier the chunk's owner copies
// the chunk into that slot; after a second the holder sums its segment from
// the slots and the prefix. LDS per workgroup is ~1.25 KiB per 1 KiB of range
// smaller than the staged form, so twice as many workgroups are resident.
// Segments shorter than 32 B (two heads or tails could share a chunk) or
// more than 128 starting in one range take their boundary chunks from
// memory instead (uniform per workgroup).
template<int U, int HR, bool NT>
__global__ __launch_bounds__(256) void
csum_span2_kernel(SpanArgs p)
{
  constexpr uint32_t R = U + HR;         // rows of 256 chunks: range + halo
  constexpr uint32_t NC = 256u * U;      // chunks per range
  constexpr uint64_t W = 16ull * NC;     // bytes per range
  constexpr uint32_t NWIN = 1024;        // speculative window entries
  constexpr uint32_t NSLOT = 128;        // boundary slots (window index mod 128)
  constexpr int UE = 4;                  // tail chunks per thread per batch
  __shared__ uint32_t s_mk[256 * R];     // per chunk: head slot + 1 | tail slot + 1 << 16
  __shared__ uint32_t s_sc[256 * R];     // row-wise wave scans of chunk values
  __shared__ u32x4 s_head[NSLOT];        // a segment's first chunk
  __shared__ u32x4 s_tail[NSLOT];        // a segment's last chunk
  __shared__ uint32_t s_tot[4 * R];      // per (row, wave) scan totals
  __shared__ uint32_t s_woff[4][4 * R];  // each wave's copy of their exclusive prefix
  __shared__ uint32_t s_cnt[16];         // per wave: window counts, tail flag, tiny flag
  __shared__ uint64_t s_meta[4];         // end of a segment past the halo; search
  __shared__ uint32_t s_ext[4];

  const uint32_t t = threadIdx.x, lane = t & 63u;
  const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6);
  const uint32_t k = xcd_block(blockIdx.x, gridDim.x);
  const uintptr_t b = reinterpret_cast<uintptr_t>(p.base);
  const uint64_t d = b & 15u;
  const uintptr_t x0 = (b & ~uintptr_t(15)) + uint64_t(k) * W, x1 = x0 + W;
  const uintptr_t xe = x1 + 16u * 256u * HR; // end of the halo
  const uintptr_t aend = b + p.arena;
  const uintptr_t zero = reinterpret_cast<uintptr_t>(k_zero_chunk);
  const uintptr_t last = p.arena ? ((aend - 1) & ~uintptr_t(15)) : zero;
  const uint32_t n = p.n;
  const gu64_ptr offs = reinterpret_cast<gu64_ptr>(reinterpret_cast<uintptr_t>(p.offs));
  const gu16_ptr lens = reinterpret_cast<gu16_ptr>(reinterpret_cast<uintptr_t>(p.lens));
  const uint64_t tg0 = k ? uint64_t(k) * W - d : 0, tg1 = uint64_t(k + 1) * W - d;
  auto chunk_at = [&](uintptr_t a) {
    return load_chunk<false>(reinterpret_cast<gchunk_ptr>(p.arena ? min(a, last) : zero));
  };
#ifdef TULIPS_CSUM_STAMPS
  const uint64_t stamp0 = __builtin_amdgcn_s_memrealtime();
#endif

  // 0. clear the marks (the barrier costs little before any load is out)
#pragma unroll
  for (uint32_t j = 0; j < R; ++j) {
    s_mk[j * 256u + t] = 0;
  }
  lds_barrier();
  // 1. one round trip: the offsets window, then the range + halo
  const uint64_t mid = (tg0 + tg1) / 2;
  const uint64_t guess = uint64_t(double(n) * double(mid) / double(p.arena ? p.arena : 1));
  const uint32_t gmax = n > NWIN ? n - NWIN : 0u;
  const uint32_t G = uint32_t(min(guess > NWIN / 2 ? guess - NWIN / 2 : 0ull, uint64_t(gmax)));
  uint64_t wo[4];
  uint32_t wl[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t i = min(G + t + 256u * r, n - 1);
    wo[r] = offs[i];
    wl[r] = lens[i];
  }
  u32x4 v[R];
#pragma unroll
  for (uint32_t j = 0; j < R; ++j) {
    const uintptr_t a = x0 + 16u * (j * 256u + t);
    const gchunk_ptr q = reinterpret_cast<gchunk_ptr>(p.arena ? min(a, last) : zero);
    v[j] = (j < HR || j >= U) ? load_chunk<false>(q) : load_chunk<NT>(q);
  }
  // every load is out before the first wait: without this fence the
  // scheduler pulls the window's first uses between the chunk loads, and the
  // vmcnt waits they bring hold the remaining chunk loads back for a whole
  // round trip
  __builtin_amdgcn_sched_barrier(0);
  {
    // window counts, the segment past the halo, and the boundary marks of
    // every entry starting in the range
    uint32_t c0 = 0, c1 = 0;
    bool far = false, tiny = false;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t e = G + t + 256u * r;
      const bool in = e < n;
      c0 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in && wo[r] < tg0));
      c1 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in && wo[r] < tg1));
      const uintptr_t sa = b + wo[r], se = min(b + wo[r] + wl[r], aend);
      const bool starts = in && sa >= x0 && sa < x1;
      if (starts && se > xe) {
        far = true;
        s_meta[3] = se;
      }
      if (starts && se > sa) {
        tiny = tiny || wl[r] < 32u;
        const uintptr_t ie = min(se, xe);
        const uint32_t ca = uint32_t((sa - x0) >> 4), ce = uint32_t((ie - 1 - x0) >> 4);
        const uint32_t slot = (e & (NSLOT - 1)) + 1;
        atomicOr(&s_mk[ca], slot);
        atomicOr(&s_mk[ce], slot << 16);
      }
    }
    const bool anyfar = __builtin_amdgcn_ballot_w64(far) != 0;
    const bool anytiny = __builtin_amdgcn_ballot_w64(tiny) != 0;
    if (lane == 0) {
      s_cnt[w] = c0;
      s_cnt[4 + w] = c1;
      s_cnt[8 + w] = anyfar;
      s_cnt[12 + w] = anytiny;
    }
  }
  // 2. row-wise wave scans of the chunk values
#pragma unroll
  for (uint32_t j = 0; j < R; ++j) {
    const uint32_t sc = wave_incl_scan(chunk_value(v[j]));
    s_sc[j * 256u + t] = sc;
    if (lane == 63) {
      s_tot[4 * j + w] = sc;
    }
  }
  lds_barrier();
#if TULIPS_SPAN_DIAG == 2 || TULIPS_SPAN_DIAG == 3
  // diagnostic builds: stop once the range is in and scanned
  if (t == 0 && p.out && k < n) {
    p.out[k] = uint16_t(s_tot[0] + s_cnt[0] + s_mk[5]);
  }
  return;
#endif
  // 3. requested chunks to their slots (all marks read first: a read after a
  //    slot store would wait for it)
  uint32_t mks[R];
#pragma unroll
  for (uint32_t j = 0; j < R; ++j) {
    mks[j] = s_mk[j * 256u + t];
  }
#pragma unroll
  for (uint32_t j = 0; j < R; ++j) {
    // (marks OR-ed together by colliding entries are never read back, but
    // must not index past the slots)
    const uint32_t mk = mks[j];
    const uint32_t mh = (mk & 0xffffu) - 1, mt = (mk >> 16) - 1;
    if (mh < NSLOT) {
      s_head[mh] = v[j];
    }
    if (mt < NSLOT) {
      s_tail[mt] = v[j];
    }
  }
  {
    const uint32_t x = lane < 4 * R ? s_tot[lane] : 0u;
    const uint32_t inc = wave_incl_scan(x);
    if (lane < 4 * R) {
      s_woff[w][lane] = inc - x;
    }
  }
  lds_barrier();
#ifdef TULIPS_CSUM_STAMPS
  const uint64_t stamp_mid = __builtin_amdgcn_s_memrealtime();
#endif
#if TULIPS_SPAN_DIAG == 4
  // diagnostic build: stop once the slots are filled
  if (t == 0 && p.out && k < n) {
    p.out[k] = uint16_t(s_woff[w][1] + s_cnt[0] + s_head[5][0]);
  }
  return;
#endif
  auto P = [&](uint32_t c) { return s_woff[w][c >> 6] + s_sc[c]; };
  const uint32_t c0 = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
  const uint32_t c1 = s_cnt[4] + s_cnt[5] + s_cnt[6] + s_cnt[7];
  const bool tail = (s_cnt[8] | s_cnt[9] | s_cnt[10] | s_cnt[11]) != 0;
  const bool tiny = (s_cnt[12] | s_cnt[13] | s_cnt[14] | s_cnt[15]) != 0;
  const uint32_t nw = min(NWIN, n - G);
  const bool tail_ok = G + NWIN >= n;
  const bool ok = (c0 > 0 || G == 0) && (c0 < nw || tail_ok) && (c1 > 0 || G == 0) &&
                  (c1 < nw || tail_ok);

  auto tail_sum = [&](uintptr_t te) {
    const uint32_t tch = uint32_t((te - xe + 15) >> 4);
    const uintptr_t tlast = xe + 16u * (tch - 1);
    const int tbytes = int(te - xe) - 16 * int(tch - 1);
    uint32_t tsum = 0;
    for (uint32_t q0 = 0; q0 < tch; q0 += 256u * UE) {
      u32x4 e[UE];
#pragma unroll
      for (int j = 0; j < UE; ++j) {
        const uint32_t c = q0 + t + 256u * j;
        e[j] = load_chunk<NT>(reinterpret_cast<gchunk_ptr>(c < tch ? xe + 16u * c : tlast));
      }
#pragma unroll
      for (int j = 0; j < UE; ++j) {
        const uint32_t c = q0 + t + 256u * j;
        tsum += c + 1 < tch ? chunk_value(e[j])
                            : (c + 1 == tch ? masked_value(e[j], 0, tbytes) : 0u);
      }
    }
    tsum = wave_incl_scan(tsum);
    if (lane == 63) {
      s_ext[w] = tsum;
    }
    lds_barrier();
    return s_ext[0] + s_ext[1] + s_ext[2] + s_ext[3];
  };
  uint32_t ext = 0;

  const uint32_t want = (p.mode & FLAG_COMPLEMENT) ? 0u : 0xffffu;
  const bool side_in = (p.mode & MODE_MASK) == MODE_TCP || p.seeds != nullptr;
  // slots: boundary chunks from the LDS slots (slot >= 0) or from memory
  auto emit = [&](uint32_t s, bool mine, uint64_t so, uint32_t sl, int slot) {
    SideIn side{0, 0, 0};
    if (side_in) {
      side = load_side(mine ? s : 0u, p.seeds, p.src, p.dst, p.mode);
    }
    const uintptr_t sa = min(max(b + so, x0), x1 - 1);
    const uintptr_t se = min(b + so + sl, aend);
    const uintptr_t ie = min(se, xe);
    uint32_t sum = 0;
    if (ie > sa) {
      const uint32_t ca = uint32_t((sa - x0) >> 4);
      const uint32_t ce = uint32_t((ie - 1 - x0) >> 4);
      const int ha = int(sa & 15u), tb = int(((ie - 1) & 15u) + 1u);
      u32x4 hv, tv;
      if (slot >= 0) {
        hv = s_head[slot];
        tv = s_tail[slot];
      } else {
        hv = chunk_at(x0 + 16u * ca);
        tv = chunk_at(x0 + 16u * ce);
      }
      sum = ca == ce ? masked_value(hv, ha, tb)
                     : masked_value(hv, ha, 16) + (P(ce - 1) - P(ca)) + masked_value(tv, 0, tb);
    }
    sum += se > xe ? ext : 0u;
    const uint32_t r =
      finish(sum, (sa & 1u) != 0, p.mode, side.seed, side.src, side.dst, sl);
#if TULIPS_SPAN_DIAG == 5
    if (mine && p.out && r == 0x1234567u) {
#else
    if (mine && p.out) {
#endif
#if TULIPS_SPAN_DIAG == 6
      // diagnostic build: each workgroup's results to its own 256-byte block
      // (wrong layout; only the store pattern differs)
      p.out[(k * 128u + (s & 127u)) % n] = uint16_t(r);
#else
      if (p.nt_store) {
        __builtin_nontemporal_store(uint16_t(r), p.out + s);
      } else {
        p.out[s] = uint16_t(r);
      }
#endif
    }
    if (p.bad) {
      const uint32_t nb =
        __builtin_popcountll(__builtin_amdgcn_ballot_w64(mine && r != want));
      if (lane == 0 && nb) {
        atomicAdd(p.bad + CNT_LINE * (blockIdx.x % CNT_SHARDS), nb);
      }
    }
  };

  if (ok) {
    const uint32_t lo = G + c0, hi = G + c1;
    if (tail) {
      ext = tail_sum(s_meta[3]);
    }
    // slots are unambiguous unless > 128 segments start here or some are short
    const bool slots = !tiny && hi - lo <= NSLOT;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t i = G + t + 256u * r;
      const bool mine = i >= lo && i < hi;
      if (__builtin_amdgcn_ballot_w64(mine) != 0) {
        emit(i, mine, mine ? wo[r] : 0, mine ? wl[r] : 0u,
             slots ? int(i & (NSLOT - 1)) : -1);
      }
    }
  } else {
    if (w == 0) {
      uint32_t L0 = 0, R0 = n, L1 = 0, R1 = n;
      while (R0 > L0 || R1 > L1) {
        const uint32_t st0 = (R0 - L0 + 255u) >> 8, st1 = (R1 - L1 + 255u) >> 8;
        uint64_t o0[4], o1[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t q = lane + 64u * r;
          o0[r] = offs[min(uint64_t(L0) + uint64_t(q) * st0, uint64_t(n - 1))];
          o1[r] = offs[min(uint64_t(L1) + uint64_t(q) * st1, uint64_t(n - 1))];
        }
        uint32_t d0 = 0, d1 = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t q = lane + 64u * r;
          const bool in0 = uint64_t(L0) + uint64_t(q) * st0 < R0;
          const bool in1 = uint64_t(L1) + uint64_t(q) * st1 < R1;
          d0 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in0 && o0[r] < tg0));
          d1 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in1 && o1[r] < tg1));
        }
        if (R0 > L0) {
          span_narrow(L0, R0, st0, __builtin_amdgcn_readfirstlane(d0));
        }
        if (R1 > L1) {
          span_narrow(L1, R1, st1, __builtin_amdgcn_readfirstlane(d1));
        }
      }
      if (lane == 0) {
        s_meta[0] = L0;
        s_meta[1] = L1;
      }
    }
    lds_barrier();
    const uint32_t lo = uint32_t(s_meta[0]), hi = uint32_t(s_meta[1]);
    if (hi > lo) {
      const uintptr_t te = min(b + p.offs[hi - 1] + p.lens[hi - 1], aend);
      if (te > xe) {
        ext = tail_sum(te);
      }
    }
    for (uint32_t s0 = lo; s0 < hi; s0 += 256u) {
      const uint32_t s = s0 + t;
      const bool mine = s < hi;
      emit(s, mine, mine ? p.offs[s] : 0, mine ? p.lens[s] : 0u, -1);
    }
  }
#ifdef TULIPS_CSUM_STAMPS
  stamp_wave_mid(stamp0, stamp_mid);
#endif
}

// SPAN, split form (`group` 6): the same byte cut with NO halo. A segment
// that crosses range boundaries is split there: every range it touches sums
// its own part from LDS and adds it, with an arrival count, to the word of
// the segment's first range (one returning agent-scope atomicAdd, executed at
// the memory side, so no cross-XCD fence is needed). The range whose add
// completes the count finishes the segment and zeroes the word, so the words
// are all zero again when the launch ends. Each range reads exactly its own
// bytes, and no workgroup ever waits for another.
// Parts are folded with end-around carry (zero iff every byte is zero), so
// their sum keeps the closed form's 0 / 0xffff distinction (csum_common.h).
#ifndef TULIPS_SPAN3_STRIDE
#define TULIPS_SPAN3_STRIDE 1
#endif
constexpr uint64_t SPAN3_STRIDE = TULIPS_SPAN3_STRIDE; // words per range
#ifndef TULIPS_SPAN3_CLUSTER
#define TULIPS_SPAN3_CLUSTER 8
#endif
#ifndef TULIPS_SPAN3_NWIN
#define TULIPS_SPAN3_NWIN 1024
#endif
#ifndef TULIPS_SPAN4_NWIN
#define TULIPS_SPAN4_NWIN 1024
#endif

template<int U, bool NT>
__global__ __launch_bounds__(256) void
csum_span3_kernel(SpanArgs p)
{
  constexpr uint32_t NC = 256u * U;      // chunks per range
  constexpr uint64_t W = 16ull * NC;     // bytes per range
  constexpr uint32_t NWIN = TULIPS_SPAN3_NWIN; // speculative window entries
  constexpr int RW = NWIN / 256;         // window entries per thread
  __shared__ u32x4 s_raw[NC];            // the range's chunks
  __shared__ uint32_t s_sc[NC];          // row-wise wave scans of chunk values
  __shared__ uint32_t s_tot[4 * U];      // per (row, wave) scan totals
  __shared__ uint32_t s_woff[4][4 * U];  // each wave's copy of their exclusive prefix
  __shared__ uint32_t s_cnt[8];          // per wave: window counts
  __shared__ uint32_t s_meta[2];         // search results

  const uint32_t t = threadIdx.x, lane = t & 63u;
  const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6);
  const uint32_t k = xcd_block_c<TULIPS_SPAN3_CLUSTER>(blockIdx.x, gridDim.x);
  const uintptr_t b = reinterpret_cast<uintptr_t>(p.base);
  const uint64_t d = b & 15u;
  const uintptr_t A = b & ~uintptr_t(15);
  const uintptr_t x0 = A + uint64_t(k) * W, x1 = x0 + W;
  const uintptr_t aend = b + p.arena;
  const uintptr_t zero = reinterpret_cast<uintptr_t>(k_zero_chunk);
  const uintptr_t last = p.arena ? ((aend - 1) & ~uintptr_t(15)) : zero;
  const uint32_t n = p.n;
  const gu64_ptr offs = reinterpret_cast<gu64_ptr>(reinterpret_cast<uintptr_t>(p.offs));
  const gu16_ptr lens = reinterpret_cast<gu16_ptr>(reinterpret_cast<uintptr_t>(p.lens));
  // lo = first s with off_s >= tg0, hi = first s with off_s >= tg1
  const uint64_t tg0 = k ? uint64_t(k) * W - d : 0, tg1 = uint64_t(k + 1) * W - d;

  // 1. one round trip: the offsets window, then the range's chunks
  const uint64_t mid = (tg0 + tg1) / 2;
  const uint64_t guess = uint64_t(double(n) * double(mid) / double(p.arena ? p.arena : 1));
  const uint32_t gmax = n > NWIN ? n - NWIN : 0u;
  const uint32_t G = uint32_t(min(guess > NWIN / 2 ? guess - NWIN / 2 : 0ull, uint64_t(gmax)));
  uint64_t wo[RW];
  uint32_t wl[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const uint32_t i = min(G + t + 256u * r, n - 1);
    wo[r] = offs[i];
    wl[r] = lens[i];
  }
  u32x4 v[U];
#pragma unroll
  for (uint32_t j = 0; j < U; ++j) {
    const uintptr_t a = x0 + 16u * (j * 256u + t);
    v[j] = load_chunk<NT>(reinterpret_cast<gchunk_ptr>(p.arena ? min(a, last) : zero));
  }
  __builtin_amdgcn_sched_barrier(0);
  {
    uint32_t c0 = 0, c1 = 0;
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const bool in = G + t + 256u * r < n;
      c0 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in && wo[r] < tg0));
      c1 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in && wo[r] < tg1));
    }
    if (lane == 0) {
      s_cnt[w] = c0;
      s_cnt[4 + w] = c1;
    }
  }
  // 2. chunks to LDS with the row-wise wave scans of their values
#pragma unroll
  for (uint32_t j = 0; j < U; ++j) {
    s_raw[j * 256u + t] = v[j];
    const uint32_t sc = wave_incl_scan(chunk_value(v[j]));
    s_sc[j * 256u + t] = sc;
    if (lane == 63) {
      s_tot[4 * j + w] = sc;
    }
  }
  lds_barrier();
  // 3. this wave's copy of the (row, wave) offsets
  {
    const uint32_t x = lane < 4 * U ? s_tot[lane] : 0u;
    const uint32_t inc = wave_incl_scan(x);
    if (lane < 4 * U) {
      s_woff[w][lane] = inc - x;
    }
  }
  auto P = [&](uint32_t c) { return s_woff[w][c >> 6] + s_sc[c]; };
  const uint32_t c0 = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
  const uint32_t c1 = s_cnt[4] + s_cnt[5] + s_cnt[6] + s_cnt[7];
  const uint32_t nw = min(NWIN, n - G);
  const bool tail_ok = G + NWIN >= n;
  const bool ok = (c0 > 0 || G == 0) && (c0 < nw || tail_ok) && (c1 > 0 || G == 0) &&
                  (c1 < nw || tail_ok);

  // 4. one segment: its part in [x0, x1) from LDS; a split segment's part
  //    goes to its first range's word and the last arrival finishes it
  const uint32_t want = (p.mode & FLAG_COMPLEMENT) ? 0u : 0xffffu;
  const bool side_in = (p.mode & MODE_MASK) == MODE_TCP || p.seeds != nullptr;
  auto emit = [&](uint32_t s, bool act, uint64_t so, uint32_t sl) {
    SideIn side{0, 0, 0};
    if (side_in) {
      side = load_side(act ? s : 0u, p.seeds, p.src, p.dst, p.mode);
    }
    const uintptr_t sa = b + so;
    const uintptr_t se = min(b + so + sl, aend);
    const uintptr_t u0 = max(sa, x0), u1 = min(se, x1);
    uint32_t sum = 0;
    if (act && u1 > u0) {
      const uint32_t ca = uint32_t((u0 - x0) >> 4);
      const uint32_t ce = uint32_t((u1 - 1 - x0) >> 4);
      const int ha = int(u0 & 15u), tb = int(((u1 - 1) & 15u) + 1u);
      sum = ca == ce ? masked_value(s_raw[ca], ha, tb)
                     : masked_value(s_raw[ca], ha, 16) + (P(ce - 1) - P(ca)) +
                         masked_value(s_raw[ce], 0, tb);
    }
    bool done = act;
    if (act && (sa < x0 || se > x1)) {
      // word = epoch << 40 | arrivals << 32 | sum of the parts so far; a
      // word tagged with another epoch is residue of an earlier call (only
      // a batch breaking the arena contract leaves one) and is taken over
      const uint64_t ra = (sa - A) / W;
      const uint32_t need = uint32_t((se - 1 - A) / W - ra);  // arrivals before the last
      const uint32_t part = fold32(sum);
      const uint64_t ep = uint64_t(p.salt) << 40;
      const uint64_t mine = ep | (1ull << 32) | part;
      unsigned long long* wp =
        reinterpret_cast<unsigned long long*>(p.slots + ra * SPAN3_STRIDE);
      unsigned long long seen = atomicCAS(wp, 0ull, mine);
      done = false;
      // every failed exchange means another arrival changed the word: the
      // loop ends after at most as many rounds as the segment has parts
      for (int round = 0; seen != 0 && round < 64; ++round) {
        unsigned long long next;
        if ((seen >> 40) != p.salt) {
          next = mine;
        } else if (uint32_t((seen >> 32) & 0xffu) == need) {
          done = true;
          sum = uint32_t(seen) + part;
          __hip_atomic_store(wp, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        } else {
          next = seen + (1ull << 32) + part;
        }
        const unsigned long long prev = atomicCAS(wp, seen, next);
        if (prev == seen) {
          break;
        }
        seen = prev;
      }
    }
    const uint32_t r =
      finish(sum, (sa & 1u) != 0, p.mode, side.seed, side.src, side.dst, sl);
    if (done && p.out) {
      if (p.nt_store) {
        __builtin_nontemporal_store(uint16_t(r), p.out + s);
      } else {
        p.out[s] = uint16_t(r);
      }
    }
    if (p.bad) {
      const uint32_t nb =
        __builtin_popcountll(__builtin_amdgcn_ballot_w64(done && r != want));
      if (lane == 0 && nb) {
        atomicAdd(p.bad + CNT_LINE * (blockIdx.x % CNT_SHARDS), nb);
      }
    }
  };

  uint32_t lo, hi;
  if (ok) {
    lo = G + c0;
    hi = G + c1;
  } else {
    // rare: wave 0 searches [lo, hi) (offsets sorted)
    if (w == 0) {
      uint32_t L0 = 0, R0 = n, L1 = 0, R1 = n;
      while (R0 > L0 || R1 > L1) {
        const uint32_t st0 = (R0 - L0 + 255u) >> 8, st1 = (R1 - L1 + 255u) >> 8;
        uint64_t o0[4], o1[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t q = lane + 64u * r;
          o0[r] = offs[min(uint64_t(L0) + uint64_t(q) * st0, uint64_t(n - 1))];
          o1[r] = offs[min(uint64_t(L1) + uint64_t(q) * st1, uint64_t(n - 1))];
        }
        uint32_t d0 = 0, d1 = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t q = lane + 64u * r;
          const bool in0 = uint64_t(L0) + uint64_t(q) * st0 < R0;
          const bool in1 = uint64_t(L1) + uint64_t(q) * st1 < R1;
          d0 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in0 && o0[r] < tg0));
          d1 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in1 && o1[r] < tg1));
        }
        if (R0 > L0) {
          span_narrow(L0, R0, st0, __builtin_amdgcn_readfirstlane(d0));
        }
        if (R1 > L1) {
          span_narrow(L1, R1, st1, __builtin_amdgcn_readfirstlane(d1));
        }
      }
      if (lane == 0) {
        s_meta[0] = L0;
        s_meta[1] = L1;
      }
    }
    lds_barrier();
    lo = s_meta[0];
    hi = s_meta[1];
  }
  // the segments starting in the range, [lo, hi), and the one before them
  // if it runs into the range (its start lies in an earlier range)
  const uint32_t first = lo > 0 ? lo - 1 : 0;
  if (ok) {
    // each thread finishes the segments whose window entries it loaded
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const uint32_t i = G + t + 256u * r;
      bool act = i >= lo && i < hi;
      if (lo > 0 && i == lo - 1) {
        act = min(b + wo[r] + wl[r], aend) > x0;
      }
      if (__builtin_amdgcn_ballot_w64(act) != 0) {
        emit(i, act, act ? wo[r] : 0, act ? wl[r] : 0u);
      }
    }
  } else {
    for (uint32_t s0 = first; s0 < hi; s0 += 256u) {
      const uint32_t s = s0 + t;
      bool act = s < hi;
      const uint64_t so = act ? p.offs[s] : 0;
      const uint32_t sl = act ? p.lens[s] : 0u;
      if (s < lo) {
        act = act && min(b + so + sl, aend) > x0;
      }
      emit(s, act, act ? so : 0, act ? sl : 0u);
    }
  }
}

template<int U, bool NT>
hipError_t
launch_span3_u(const SpanArgs& sp, hipStream_t stream)
{
  constexpr uint64_t W = 4096ull * U;
  const uint64_t ranges = span_ranges(sp.base, sp.arena, W);
  if (ranges > 0x7fffffffull) {
    return hipErrorInvalidValue;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL((csum_span3_kernel<U, NT>), dim3(uint32_t(ranges)), dim3(256), 0, stream,
                     sp);
  return hipGetLastError();
}

template<int U, int HR, bool NT>
hipError_t
launch_span2_u(const SpanArgs& sp, hipStream_t stream)
{
  constexpr uint64_t W = 4096ull * U;
  const uint64_t ranges = ((sp.arena + (reinterpret_cast<uintptr_t>(sp.base) & 15u)) / W) + 1;
  if (ranges > 0x7fffffffull) {
    return hipErrorInvalidValue;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL((csum_span2_kernel<U, HR, NT>), dim3(uint32_t(ranges)), dim3(256), 0,
                     stream, sp);
  return hipGetLastError();
}

template<int U, int HR, bool NT>
hipError_t
launch_span_u(const SpanArgs& sp, hipStream_t stream)
{
  constexpr uint64_t W = 4096ull * U;
  // ranges cover [A, A + K W) with A <= base: position base + arena (where
  // an empty last segment may start) included
  const uint64_t ranges = ((sp.arena + (reinterpret_cast<uintptr_t>(sp.base) & 15u)) / W) + 1;
  if (ranges > 0x7fffffffull) {
    return hipErrorInvalidValue;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL((csum_span_kernel<U, HR, NT>), dim3(uint32_t(ranges)), dim3(256), 0, stream,
                     sp);
  return hipGetLastError();
}

template<int GS, int US, int UL, int SPS, bool NT>
hipError_t
launch_hybrid(const VarSegs& segs, const LaunchArgs& a, hipStream_t stream)
{
  const uint64_t per_block = uint64_t(256 / 64) * uint64_t(64 / GS) * SPS;
  uint64_t blocks = (uint64_t(a.n) + per_block - 1) / per_block;
  if (a.max_blocks && blocks > a.max_blocks) {
    blocks = a.max_blocks;
  }
  if (blocks == 0) {
    return hipSuccess;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL((csum_hybrid_kernel<GS, US, UL, SPS, NT>),
                     dim3(uint32_t(blocks)), dim3(256), 0, stream, segs,
                     a.seeds, a.src, a.dst, a.out, a.bad, a.n, a.mode,
                     a.nt_store);
  return hipGetLastError();
}

#ifdef TULIPS_CSUM_STAMPS
extern "C" int
tulips_csum_stamps_arm(uint64_t* buf)
{
  const uint32_t zero = 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &buf, sizeof(buf)) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_count), &zero, sizeof(zero)) !=
        hipSuccess) {
    return 2;
  }
  return 0;
}

extern "C" uint32_t
tulips_csum_stamps_count()
{
  uint32_t c = 0;
  (void)hipMemcpyFromSymbol(&c, HIP_SYMBOL(g_stamp_count), sizeof(c));
  return c;
}
#endif

// PACKED sps = 4: the lane-parallel-cursor form (csum_vpacked_kernel)
template<int S, int U>
hipError_t
vpacked(const VarSegs& segs, const LaunchArgs& a, hipStream_t stream)
{
  if constexpr (S > 32 || U > 4) {
    return hipErrorInvalidValue;
  } else {
    return a.nontemporal ? launch_vpacked<S, U, true>(segs, a, stream)
                         : launch_vpacked<S, U, false>(segs, a, stream);
  }
}
// Process-wide split words for the staged split form (group 6), tagged with
// a 24-bit epoch per call.
std::mutex g_words_mu;
uint64_t* g_words = nullptr;
uint64_t g_nwords = 0;
uint32_t g_epoch = 0;

hipError_t
variant_words(uint64_t need, uint64_t** out, uint32_t* epoch)
{
  std::lock_guard<std::mutex> g(g_words_mu);
  if (need > g_nwords) {
    if (g_words) {
      (void)hipDeviceSynchronize();
      (void)hipFree(g_words);
      g_words = nullptr;
    }
    hipError_t e = hipMalloc(&g_words, need * sizeof(uint64_t));
    if (e == hipSuccess) {
      e = hipMemset(g_words, 0, need * sizeof(uint64_t));
    }
    if (e != hipSuccess) {
      g_nwords = 0;
      return e;
    }
    g_nwords = need;
  }
  g_epoch = (g_epoch + 1) & 0xffffffu;
  g_epoch += g_epoch == 0;
  *out = g_words;
  *epoch = g_epoch;
  return hipSuccess;
}

hipError_t
variant_var(const uint8_t* base, const uint64_t* offs, const uint16_t* lens,
           const LaunchArgs& a, hipStream_t stream)
{
  const VarSegs segs{base, offs, lens};
  if (a.kind == TULIPS_CSUM_KIND_PACKED) {
    // group = segments per wave, unroll = 64-chunk windows in flight,
    // spw = 2: double-buffered (next windows in flight while scanning)
#define TCS_PCASE(S_, U_)                                                      \
  if (a.group == S_ && a.unroll == U_) {                                       \
    if (a.spw == 4) {                                                          \
      return vpacked<S_, U_>(segs, a, stream);                                 \
    }                                                                          \
    if (a.spw == 3) {                                                          \
      return a.nontemporal ? launch_packed<S_, U_, true, 2>(segs, a, stream)   \
                           : launch_packed<S_, U_, false, 2>(segs, a, stream); \
    }                                                                          \
    if (a.spw == 2) {                                                          \
      return a.nontemporal ? launch_packed<S_, U_, true, 1>(segs, a, stream)   \
                           : launch_packed<S_, U_, false, 1>(segs, a, stream); \
    }                                                                          \
    return a.nontemporal ? launch_packed<S_, U_, true, 0>(segs, a, stream)     \
                         : launch_packed<S_, U_, false, 0>(segs, a, stream);   \
  }
    TCS_PCASE(4, 4)
    TCS_PCASE(6, 4)
    TCS_PCASE(8, 2)
    TCS_PCASE(8, 4)
    TCS_PCASE(12, 4)
    TCS_PCASE(16, 2)
    TCS_PCASE(16, 4)
    TCS_PCASE(16, 8)
    TCS_PCASE(32, 4)
    TCS_PCASE(32, 8)
    TCS_PCASE(64, 4)
    TCS_PCASE(64, 8)
#undef TCS_PCASE
    return hipErrorInvalidValue;
  }
  if (a.kind == TULIPS_CSUM_KIND_BALANCED) {
    // block = 64 * waves per workgroup, unroll = windows per batch
    const int nw = a.block / 64;
#define TCS_BCASE(NW_, U_)                                                     \
  if (nw == NW_ && a.unroll == U_) {                                           \
    if (a.spw == 2) {                                                          \
      return a.nontemporal ? launch_balanced<NW_, U_, true, 1>(segs, a, stream)  \
                           : launch_balanced<NW_, U_, false, 1>(segs, a, stream); \
    }                                                                          \
    return a.nontemporal ? launch_balanced<NW_, U_, true, 0>(segs, a, stream)  \
                         : launch_balanced<NW_, U_, false, 0>(segs, a, stream); \
  }
    TCS_BCASE(4, 2)
    TCS_BCASE(4, 4)
    TCS_BCASE(4, 6)
    TCS_BCASE(8, 2)
    TCS_BCASE(8, 4)
    TCS_BCASE(8, 6)
#undef TCS_BCASE
    return hipErrorInvalidValue;
  }
  if (a.kind == TULIPS_CSUM_KIND_HYBRID) {
    // group = short subgroup lanes, unroll = short loads per lane,
    // spw = segments per short subgroup in flight; 8 loads/lane when long
#define TCS_HCASE(GS_, US_, SPS_)                                              \
  if (a.group == GS_ && a.unroll == US_ && a.spw == SPS_) {                    \
    return a.nontemporal                                                       \
             ? launch_hybrid<GS_, US_, 8, SPS_, true>(segs, a, stream)         \
             : launch_hybrid<GS_, US_, 8, SPS_, false>(segs, a, stream);       \
  }
    TCS_HCASE(8, 4, 1)
    TCS_HCASE(8, 4, 2)
    TCS_HCASE(8, 4, 4)
    TCS_HCASE(8, 8, 1)
    TCS_HCASE(16, 2, 1)
    TCS_HCASE(16, 2, 2)
    TCS_HCASE(16, 2, 4)
    TCS_HCASE(16, 4, 1)
    TCS_HCASE(16, 4, 2)
    TCS_HCASE(16, 8, 1)
    TCS_HCASE(32, 4, 1)
#undef TCS_HCASE
    return hipErrorInvalidValue;
  }
  return hipErrorInvalidValue;
}

hipError_t
variant_span(const uint8_t* base, uint64_t arena, const uint64_t* offs,
            const uint16_t* lens, const LaunchArgs& a, hipStream_t stream)
{
  const SpanArgs sp{base, arena, offs, lens, a.seeds, a.src, a.dst, a.out, a.bad,
                    a.n, a.mode, a.nt_store ? 1u : 0u, nullptr, 0, 0};
  if (a.n == 0) {
    return hipSuccess;
  }
  if (a.group == 6) {
    // staged split form: process-wide words (one call at a time; tools only)
    SpanArgs sp3 = sp;
    hipError_t e = variant_words(span_ranges(base, arena, 4096ull * a.unroll) * SPAN3_STRIDE,
                                 &sp3.slots, &sp3.salt);
    if (e != hipSuccess) {
      return e;
    }
#define TCS_S3CASE(U_)                                                         \
  if (a.unroll == U_) {                                                        \
    return a.nontemporal ? launch_span3_u<U_, true>(sp3, stream)               \
                         : launch_span3_u<U_, false>(sp3, stream);             \
  }
    TCS_S3CASE(2)
    TCS_S3CASE(4)
    TCS_S3CASE(5)
    TCS_S3CASE(6)
    TCS_S3CASE(7)
    TCS_S3CASE(8)
    TCS_S3CASE(10)
    TCS_S3CASE(12)
#undef TCS_S3CASE
    return hipErrorInvalidValue;
  }
  // group = halo rows of 4 KiB read past the range (1 or 2), or 3 = none:
  // the crossing segment's wave reads exactly its tail (0 = default);
  // 4 / 5 = the boundary-slot form with 2 / 1 halo rows
  if (a.group == 4 || a.group == 5) {
#define TCS_S2CASE(U_, H_)                                                     \
  if (a.unroll == U_ && (a.group == 4 ? 2 : 1) == H_) {                        \
    return a.nontemporal ? launch_span2_u<U_, H_, true>(sp, stream)            \
                         : launch_span2_u<U_, H_, false>(sp, stream);          \
  }
    TCS_S2CASE(4, 2)
    TCS_S2CASE(6, 2)
    TCS_S2CASE(8, 2)
    TCS_S2CASE(8, 1)
    TCS_S2CASE(10, 2)
    TCS_S2CASE(12, 2)
#undef TCS_S2CASE
    return hipErrorInvalidValue;
  }
  const int hr = a.group == 3 ? 0 : a.group;
#define TCS_SCASE(U_, H_)                                                      \
  if (a.unroll == U_ && hr == H_) {                                            \
    return a.nontemporal ? launch_span_u<U_, H_, true>(sp, stream)             \
                         : launch_span_u<U_, H_, false>(sp, stream);           \
  }
  TCS_SCASE(6, 0)
  TCS_SCASE(7, 0)
  TCS_SCASE(8, 0)
  TCS_SCASE(2, 1)
  TCS_SCASE(2, 2)
  TCS_SCASE(4, 1)
  TCS_SCASE(4, 2)
  TCS_SCASE(6, 1)
  TCS_SCASE(6, 2)
  TCS_SCASE(8, 1)
  TCS_SCASE(8, 2)
  TCS_SCASE(10, 2)
  TCS_SCASE(12, 2)
#undef TCS_SCASE
  return hipErrorInvalidValue;
}
} // namespace
} // namespace tulips_amd

using namespace tulips_amd;

namespace {

int
status_of(hipError_t e)
{
  return e == hipSuccess ? TULIPS_STATUS_OK
         : e == hipErrorInvalidValue ? TULIPS_STATUS_INVALID_ARGUMENT
                                     : TULIPS_STATUS_HARDWARE_ERROR;
}

LaunchArgs
args_of(const tulips_csum_tuning* t, const uint16_t* seeds, const uint32_t* src,
        const uint32_t* dst, uint16_t* out, uint32_t n, uint32_t mode)
{
  LaunchArgs a{};
  a.seeds = seeds;
  a.src = src;
  a.dst = dst;
  a.out = out;
  a.n = n;
  a.mode = mode;
  a.kind = t->kind;
  a.group = t->group;
  a.unroll = t->unroll;
  a.nontemporal = t->nontemporal < 0 || (t->nontemporal & 1) != 0;
  a.nt_store = t->nontemporal > 0 && (t->nontemporal & 2) != 0;
  a.max_blocks = t->max_blocks;
  a.block = t->block ? t->block : 256;
  a.spw = t->sps ? t->sps : 1;
  return a;
}

} // namespace

extern "C" int
tulips_variant_batch_tuned(const uint8_t* base, const uint64_t* offsets,
                           const uint16_t* lengths, const uint16_t* seeds,
                           const uint32_t* src, const uint32_t* dst, uint16_t* out,
                           uint32_t n, uint32_t mode, const tulips_csum_tuning* tuning,
                           void* stream)
{
  if (!tuning || (n && (!base || !offsets || !lengths || !out))) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (n == 0) {
    return TULIPS_STATUS_OK;
  }
  const LaunchArgs a = args_of(tuning, seeds, src, dst, out, n, mode);
  return status_of(variant_var(base, offsets, lengths, a, static_cast<hipStream_t>(stream)));
}

extern "C" int
tulips_variant_batch_arena_tuned(const uint8_t* base, uint64_t arena_bytes,
                                 const uint64_t* offsets, const uint16_t* lengths,
                                 const uint16_t* seeds, const uint32_t* src,
                                 const uint32_t* dst, uint16_t* out, uint32_t n, uint32_t mode,
                                 const tulips_csum_tuning* tuning, void* stream)
{
  if (!tuning || tuning->kind != TULIPS_CSUM_KIND_SPAN ||
      (n && (!offsets || !lengths || !out))) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  const LaunchArgs a = args_of(tuning, seeds, src, dst, out, n, mode);
  return status_of(
    variant_span(base, arena_bytes, offsets, lengths, a, static_cast<hipStream_t>(stream)));
}
