// span_kernel.h — the in-order-arena (SPAN) checksum kernel, split form with
// the chunk prefixes in LDS (its history profiles/HISTORY.md §4). The kernel is a template over a
// probe so that tools/sessions/probes/span_stamps.hip can time the product code path
// itself; the product launches csum_span_kernel<U> (NoProbe, which compiles
// to nothing) from csum_kernels.hip. Semantics: src/stack/Utils.cpp:14-42
// (closed form in csum_common.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "csum_common.h"
#include "csum_device.h"

namespace tulips_amd {
namespace {

// ---------------------------------------------------------------------------
// SPAN: in-order arenas (tulips_csum_batch_arena), work cut by arena BYTES.
//
// Any decomposition by segment count gives a wave a chain of dependent round
// trips whose length follows the bytes it drew (on ZIPF the heaviest
// 8-segment waves end ~8 us after the median one). When the segments lie in
// order in one arena the arena itself is cut instead: workgroup k (256
// threads) owns the 16-byte-aligned range [A + kW, A + (k+1)W), W = 4 KiB * U,
// and every workgroup reads the same bytes whatever the length mix.
//   * one round trip brings a 1024-entry window of offsets/lengths (where an
//     evenly filled arena would put the range's segments; issued first, since
//     vmcnt retires in order) and the range's own chunks, U per lane; ballot
//     counts over the window give the segments starting in the range
//     [lo, hi) (a 256-ary search by wave 0 when the window misses);
//   * only the row-wise wave scans of the chunks' 16-bit-half sums (v_dot2)
//     live in LDS (4 B per chunk), so at least seven workgroups share a CU
//     (registers bounded to 7 waves per SIMD) and a ZIPF launch (1,527
//     ranges of 28 KiB) is one generation. A segment's two boundary chunks
//     are loaded by the thread holding its window entry as soon as the
//     window is in, between the range's first U / 3 rows and the rest
//     (temporal: the lines are in L2 or in flight), so they arrive before
//     the range's last rows and cost no round trip after the data;
//   * a segment crossing range boundaries is summed in parts: every range it
//     touches adds its part (folded with end-around carry, so zero iff its
//     bytes are) and an arrival to ONE 64-bit word, its first range's, by a
//     returning agent-scope atomic (executed at the memory side, so no
//     cross-XCD fence); the arrival that completes the count finishes the
//     segment. A two-part segment (every segment shorter than a range) uses
//     one exchange per part and leaves its word as it is; longer ones
//     compare-and-swap and zero the word at the end. No workgroup ever waits
//     for another.
// Words (stream_state.h span_slots) are tagged with the launch's AQL dispatch
// id (per-queue packet index, 40 bits kept: distinct for every launch and
// every graph replay on a queue until 2^40 dispatches) offset by a hash of the
// queue (launch_tag: ids of different queues overlap), so a word left by an
// earlier launch is never taken for a part of this one: it is overwritten,
// never added to. A split part is only sent to a word
// when the segment starts inside the arena and its range has a word;
// otherwise (contract broken) it is finished locally with an undefined
// result. Contract (include/tulips_csum.h): offsets[i] + lengths[i] <=
// offsets[i+1] and offsets[n-1] + lengths[n-1] <= arena_bytes; every access
// is clamped into [base & ~15, (base + arena_bytes + 15) & ~15).
// ---------------------------------------------------------------------------
extern "C" __device__ uint64_t llvm_amdgcn_dispatch_id() __asm("llvm.amdgcn.dispatch.id");

// Split word: tag (40) | arrivals before the last (4) | sum of parts (20;
// at most 15 parts of at most 0xffff each before the last).
constexpr uint32_t WORD_ARR_SHIFT = 20, WORD_TAG_SHIFT = 24;
constexpr uint64_t WORD_SUM_MASK = (1ull << WORD_ARR_SHIFT) - 1;
constexpr uint64_t WORD_TAG_MASK = (1ull << 40) - 1;

// This launch's tag: its dispatch id (the packet's index on its queue) offset
// by a hash of the queue's address, xor the word array's salt. Every hardware
// queue counts from 0, and one word array can see launches from several
// queues (a graph replayed on another stream, a stream handle reused after
// hipStreamDestroy), so two queues in step would give two launches the same
// bare dispatch id and the later one would take the earlier one's residue for
// its own part. With the offset two queues' tags meet only when their
// counters differ by the difference of their offsets, a pseudo-random 40-bit
// number.
__device__ __forceinline__ uint64_t
launch_tag(uint32_t salt)
{
  const uint64_t q = uint64_t(reinterpret_cast<uintptr_t>(__builtin_amdgcn_queue_ptr()));
  const uint64_t h = (q * 0x9E3779B97F4A7C15ull) >> 24;
  return ((llvm_amdgcn_dispatch_id() + h) ^ salt) & WORD_TAG_MASK;
}

// The product's probe: no marks. tools/sessions/probes/span_stamps.hip instantiates
// the same kernel with a probe that records per-wave realtime stamps at
// marks 0-5 (and 7 on the rare path), and with other XC / NWIN values.
struct NoProbe
{
  static constexpr int stop = 0; // diagnostic builds stop after phase 1/2/3
  static constexpr bool data_mark = false; // stamp when the wave's loads are in
  __device__ __forceinline__ void mark(uint32_t, uint32_t, uint32_t, int) const {}
  __device__ __forceinline__ void keep(uint32_t) const {}
};

// XC: consecutive ranges kept on one XCD (xcd_block_c); NWIN: entries of the
// speculative offsets window; MH: range chunks per lane issued before the
// window is counted (the rest after the boundary chunks, which then arrive
// before the range's last rows). The product uses NoProbe, 8, 1024 and U / 3
// (tools/sessions/probes/span_stamps.py, profiles/probe_span_geometry_r03.txt).
// XCHG: a segment in two parts (always, when its length is below the range
// size) meets its other part by one exchange per part, and the word is not
// re-zeroed: the next launch's tag differs (profiles/probe_span_early_r03.txt:
// 0.2-0.4 us per ZIPF launch against compare-and-swap + re-zero).
// TR > 0: the tail-shaped cut (measured against the uniform
// one by tools/sessions/probes/probe_span_tail.py): ranges k < p.k1 hold U rows, the last
// ones (dispatched last) TR rows, so the final workgroups on each CU finish
// their data sooner and their tails overlap. TR = 0: every range U rows.
// PRIO (the one ZIPF experiment, tools/sessions/probes/probe_span_prio.py):
// a launch is one generation of workgroups whose post-data phases bunch in
// its last ~2 us; the waves of ranges in the first quarter of the arena run
// at instruction priority 3, the next quarters 2, 1, 0, so on a CU the
// earlier ranges issue (and get) their loads first and finish while later
// ones still stream.
template<int U, class Probe = NoProbe, uint32_t XC = 8, uint32_t NWIN = 1024, int MH = U / 3,
         bool XCHG = true, uint32_t TB = 256, int TR = 0, bool PRIO = false>
__global__ __launch_bounds__(TB, 7) void
csum_span_kernel(SpanArgs p, Probe pr)
{
  constexpr uint32_t NWV = TB / 64; // waves per workgroup
  static_assert(TB % 64 == 0 && NWV * U <= 64, "row totals fit one wave scan");
  static_assert(TR >= 0 && TR <= U, "tail rows");
  constexpr uint32_t NC = TB * U;
  constexpr uint64_t W = 16ull * NC;
  constexpr uint64_t WT = 16ull * TB * uint64_t(TR ? TR : U);
  constexpr int RW = NWIN / TB;
  __shared__ uint32_t s_sc[NC];
  __shared__ uint32_t s_tot[NWV * U];
  __shared__ uint32_t s_woff[NWV][NWV * U];
  __shared__ uint32_t s_cnt[2 * NWV];
  __shared__ uint32_t s_meta[2];

  const uint32_t t = threadIdx.x, lane = t & 63u;
  const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6);
  const uint32_t k = xcd_block_c<XC>(blockIdx.x, gridDim.x);
  if constexpr (PRIO) {
    const uint32_t q = uint32_t(uint64_t(k) * 4u / gridDim.x); // (wave-uniform)
    if (q == 0) {
      __builtin_amdgcn_s_setprio(3);
    } else if (q == 1) {
      __builtin_amdgcn_s_setprio(2);
    } else if (q == 2) {
      __builtin_amdgcn_s_setprio(1);
    }
  }
  pr.mark(k, w, lane, 0);

  const uintptr_t b = reinterpret_cast<uintptr_t>(p.base);
  const uint64_t d = b & 15u;
  const uintptr_t A = b & ~uintptr_t(15);
  // range k = [A + rstart(k), A + rstart(k + 1)); rix(o) = the range of
  // arena offset o (from A)
  const uint64_t K1 = TR ? p.k1 : ~0ull;
  auto rstart = [&](uint64_t kk) -> uint64_t {
    return (TR && kk > K1) ? K1 * W + (kk - K1) * WT : kk * W;
  };
  auto rix = [&](uint64_t o) -> uint64_t {
    return (TR && o >= K1 * W) ? K1 + (o - K1 * W) / WT : o / W;
  };
  const uint32_t rows = (TR && uint64_t(k) >= K1) ? uint32_t(TR) : uint32_t(U);
  const uintptr_t x0 = A + rstart(k), x1 = A + rstart(uint64_t(k) + 1);
  const uintptr_t aend = b + p.arena;
  const uintptr_t zero = reinterpret_cast<uintptr_t>(k_zero_chunk);
  const uintptr_t last = p.arena ? ((aend - 1) & ~uintptr_t(15)) : zero;
  const uint32_t n = p.n;
  const gu64_ptr offs = reinterpret_cast<gu64_ptr>(reinterpret_cast<uintptr_t>(p.offs));
  const gu16_ptr lens = reinterpret_cast<gu16_ptr>(reinterpret_cast<uintptr_t>(p.lens));
  const uint64_t tg0 = k ? (x0 - A) - d : 0, tg1 = (x1 - A) - d;
  // a chunk of the range (or zeros), clamped into the arena
  auto chunk_at = [&](uintptr_t a) {
    return reinterpret_cast<gchunk_ptr>(p.arena ? min(a, last) : zero);
  };
  // row j of the range (rows past a short tail range's read zeros)
  auto row_at = [&](uint32_t j, uintptr_t a) {
    return (TR && j >= rows) ? reinterpret_cast<gchunk_ptr>(zero) : chunk_at(a);
  };

  // 1. the offsets window, then the range's chunks (temporal whatever the
  //    tuning asks: the boundary chunks are loaded again below, and nt loads
  //    measured 0.3-0.5 us slower per launch on 4 branches, equal serially,
  //    profiles/probe_split_r02.txt)
  const uint64_t mid = (tg0 + tg1) / 2;
  const uint64_t guess = uint64_t(double(n) * double(mid) / double(p.arena ? p.arena : 1));
  const uint32_t gmax = n > NWIN ? n - NWIN : 0u;
  const uint32_t G = uint32_t(min(guess > NWIN / 2 ? guess - NWIN / 2 : 0ull, uint64_t(gmax)));
  uint64_t wo[RW];
  uint32_t wl[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const uint32_t i = min(G + t + TB * r, n - 1);
    wo[r] = offs[i] - p.bias;
    wl[r] = lens[i];
  }
  u32x4 v[U];
#pragma unroll
  for (uint32_t j = 0; j < uint32_t(MH); ++j) {
    v[j] = load_chunk<false>(row_at(j, x0 + 16u * (j * TB + t)));
  }
  __builtin_amdgcn_sched_barrier(0);
  pr.mark(k, w, lane, 1);
  {
    uint32_t c0 = 0, c1 = 0;
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const bool in = G + t + TB * r < n;
      c0 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in && wo[r] < tg0));
      c1 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(in && wo[r] < tg1));
    }
    if (lane == 0) {
      s_cnt[w] = c0;
      s_cnt[NWV + w] = c1;
    }
  }
  lds_barrier(); // (the range's loads stay in flight)
  pr.mark(k, w, lane, 2);
  uint32_t c0 = 0, c1 = 0;
#pragma unroll
  for (uint32_t q = 0; q < NWV; ++q) {
    c0 += s_cnt[q];
    c1 += s_cnt[NWV + q];
  }
  const uint32_t nw = min(NWIN, n - G);
  const bool tail_ok = G + NWIN >= n;
  const bool ok = (c0 > 0 || G == 0) && (c0 < nw || tail_ok) && (c1 > 0 || G == 0) &&
                  (c1 < nw || tail_ok);
  const uint32_t lo = G + c0, hi = G + c1;
  const uint32_t first = lo > 0 ? lo - 1 : 0;
  // fast path: at most TB entries to finish, so each thread holds at most
  // one of them
  const bool fast = ok && hi - first <= TB;

  // 2. this thread's entry and its two boundary chunks, issued now
  bool act = false;
  uint32_t s = 0, sl = 0;
  uint64_t so = 0;
  if (fast) {
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const uint32_t i = G + t + TB * r;
      bool a = i >= lo && i < hi;
      if (lo > 0 && i == lo - 1) {
        const uintptr_t ie = min(b + wo[r] + wl[r], aend);
        a = ie > x0;
      }
      if (a) {
        act = true;
        s = i;
        so = wo[r];
        sl = wl[r];
      }
    }
  }
  const uintptr_t sa = b + so, se = min(b + so + sl, aend);
  const uintptr_t u0 = max(sa, x0), u1 = min(se, x1);
  const bool has = act && u1 > u0;
  const uint32_t ca = has ? uint32_t((u0 - x0) >> 4) : 0u;
  const uint32_t ce = has ? uint32_t((u1 - 1 - x0) >> 4) : 0u;
  const u32x4 bh = load_chunk<false>(chunk_at(x0 + 16u * ca));
  const u32x4 bt = load_chunk<false>(chunk_at(x0 + 16u * ce));
  if constexpr (MH < U) {
#pragma unroll
    for (uint32_t j = MH; j < uint32_t(U); ++j) {
      v[j] = load_chunk<false>(row_at(j, x0 + 16u * (j * TB + t)));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // MH < U: the boundary chunks arrive before the range's last rows, so
  // their masked sums are taken now and the chunks do not stay live through
  // the scans
  uint32_t bsum = 0;
  if constexpr (MH < U) {
    const int ha = int(u0 & 15u), tb = int(((u1 - 1) & 15u) + 1u);
    bsum = ca == ce ? masked_value(bh, ha, tb) : masked_value(bh, ha, 16) + masked_value(bt, 0, tb);
  }
  if constexpr (Probe::stop == 1) { // loads and window only
    uint32_t x = bh.x ^ bt.y;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      x ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
    pr.keep(x);
    return;
  }

  if constexpr (Probe::data_mark) { // stamps only: when all of the wave's loads are in
    __builtin_amdgcn_s_waitcnt(0x0f70); // vmcnt(0)
    pr.mark(k, w, lane, 6);
  }
  // 3. row-wise wave scans of the range's chunk values
#pragma unroll
  for (uint32_t j = 0; j < U; ++j) {
    const uint32_t sc = wave_incl_scan(chunk_value(v[j]));
    s_sc[j * TB + t] = sc;
    if (lane == 63) {
      s_tot[NWV * j + w] = sc;
    }
  }
  lds_barrier();
  {
    const uint32_t x = lane < NWV * U ? s_tot[lane] : 0u;
    const uint32_t inc = wave_incl_scan(x);
    if (lane < NWV * U) {
      s_woff[w][lane] = inc - x;
    }
  }
  pr.mark(k, w, lane, 3);
  auto P = [&](uint32_t c) { return s_woff[w][c >> 6] + s_sc[c]; };

  if constexpr (Probe::stop == 2) { // + scans
    pr.keep(P(t) ^ bh.x ^ bt.y);
    return;
  }

  // 4. a segment's part in the range. Results of segments inside the range
  //    are stored first; parts of segments crossing its bounds then meet in
  //    their first range's word (the stores are already on their way while
  //    the compare-and-swap makes its round trip)
  const uint32_t want = (p.mode & FLAG_COMPLEMENT) ? 0u : 0xffffu;
  const bool side_in = (p.mode & MODE_MASK) == MODE_TCP || p.seeds != nullptr;
  const uint64_t tag = launch_tag(p.salt);
  auto store = [&](uint32_t s, uint32_t r) {
    if (p.out) {
      if (p.nt_store) {
        __builtin_nontemporal_store(uint16_t(r), p.out + s);
      } else {
        p.out[s] = uint16_t(r);
      }
    }
  };
  auto emit = [&](uint32_t s, bool act, uintptr_t sa, uintptr_t se, uint32_t sl, uint32_t sum) {
    SideIn side{0, 0, 0};
    if (side_in) {
      side = load_side(act ? s : 0u, p.seeds, p.src, p.dst, p.mode);
    }
    // a part goes to a word only for a segment starting inside the arena
    // whose first range has one (always, under the arena contract)
    const uint64_t ra = rix(sa - A);
    const bool split = act && (sa < x0 || se > x1) && sa >= A && sa < se && ra < p.nslots;
    bool done = act && !split;
    uint32_t r = finish(sum, (sa & 1u) != 0, p.mode, side.seed, side.src, side.dst, sl);
    if constexpr (Probe::stop == 3) { // + every part stored as a result, no atomics
      if (act) {
        store(s, r);
      }
      return;
    }
    if (done) {
      store(s, r);
    }
    pr.mark(k, w, lane, 4);
    if (__builtin_amdgcn_ballot_w64(split) != 0) {
      if (split) {
        const uint32_t need = uint32_t(rix(se - 1 - A) - ra); // arrivals before the last
        const uint32_t part = fold32(sum);
        const uint64_t mine = (tag << WORD_TAG_SHIFT) | (1ull << WORD_ARR_SHIFT) | part;
        unsigned long long* wp = reinterpret_cast<unsigned long long*>(p.slots + ra);
        unsigned long long seen = 0;
        if (XCHG && need == 1) {
          // two parts: the one that finds the other's part (this launch's
          // tag, an arrival counted) is last; the word keeps residue
          seen = atomicExch(wp, mine);
          if ((seen >> WORD_TAG_SHIFT) == tag && ((seen >> WORD_ARR_SHIFT) & 0xfu) != 0) {
            done = true;
            sum = uint32_t(seen & WORD_SUM_MASK) + part;
          }
          seen = 0;
        } else {
          seen = atomicCAS(wp, 0ull, mine);
        }
        // every failed exchange means another arrival changed the word: the
        // loop ends after at most as many rounds as the segment has parts
        for (int round = 0; seen != 0 && round < 64; ++round) {
          unsigned long long next;
          if ((seen >> WORD_TAG_SHIFT) != tag) {
            next = mine; // residue of an earlier launch: taken over
          } else if (uint32_t((seen >> WORD_ARR_SHIFT) & 0xfu) == need) {
            done = true;
            sum = uint32_t(seen & WORD_SUM_MASK) + part;
            __hip_atomic_store(wp, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          } else {
            next = seen + (1ull << WORD_ARR_SHIFT) + part;
          }
          const unsigned long long prev = atomicCAS(wp, seen, next);
          if (prev == seen) {
            break;
          }
          seen = prev;
        }
        if (done) {
          r = finish(sum, (sa & 1u) != 0, p.mode, side.seed, side.src, side.dst, sl);
          store(s, r);
        }
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
  // sum of [u0, u1) from the prefix and the two boundary chunks
  auto part_of = [&](uintptr_t u0, uintptr_t u1, uint32_t ca, uint32_t ce, const u32x4& bh,
                     const u32x4& bt) {
    const int ha = int(u0 & 15u), tb = int(((u1 - 1) & 15u) + 1u);
    return ca == ce ? masked_value(bh, ha, tb)
                    : masked_value(bh, ha, 16) + (P(ce - 1) - P(ca)) + masked_value(bt, 0, tb);
  };

  if (fast) {
    if (__builtin_amdgcn_ballot_w64(act) != 0) {
      if constexpr (MH < U) {
        emit(s, act, sa, se, sl, has ? bsum + (ca == ce ? 0u : P(ce - 1) - P(ca)) : 0u);
      } else {
        emit(s, act, sa, se, sl, has ? part_of(u0, u1, ca, ce, bh, bt) : 0u);
      }
    }
    pr.mark(k, w, lane, 5);
    return;
  }
  // rare: [lo, hi) from a search when the window missed; metadata and
  // boundary chunks from memory, TB entries per round
  pr.mark(k, w, lane, 7);
  uint32_t L = lo, H = hi;
  if (!ok) {
    if (w == 0) {
      uint32_t L0 = 0, R0 = n, L1 = 0, R1 = n;
      while (R0 > L0 || R1 > L1) {
        const uint32_t st0 = (R0 - L0 + 255u) >> 8, st1 = (R1 - L1 + 255u) >> 8;
        uint64_t o0[4], o1[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t q = lane + 64u * r;
          o0[r] = offs[min(uint64_t(L0) + uint64_t(q) * st0, uint64_t(n - 1))] - p.bias;
          o1[r] = offs[min(uint64_t(L1) + uint64_t(q) * st1, uint64_t(n - 1))] - p.bias;
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
    L = s_meta[0];
    H = s_meta[1];
  }
  for (uint32_t s0 = L > 0 ? L - 1 : 0; s0 < H; s0 += TB) {
    const uint32_t i = s0 + t;
    bool a = i < H;
    const uint64_t o = a ? p.offs[i] - p.bias : 0;
    const uint32_t l = a ? p.lens[i] : 0u;
    const uintptr_t ia = b + o, ie = min(b + o + l, aend);
    if (i < L) {
      a = a && ie > x0;
    }
    const uintptr_t v0 = max(ia, x0), v1 = min(ie, x1);
    const bool h = a && v1 > v0;
    const uint32_t qa = h ? uint32_t((v0 - x0) >> 4) : 0u;
    const uint32_t qe = h ? uint32_t((v1 - 1 - x0) >> 4) : 0u;
    const u32x4 ch = load_chunk<false>(chunk_at(x0 + 16u * qa));
    const u32x4 ct = load_chunk<false>(chunk_at(x0 + 16u * qe));
    emit(i, a, a ? ia : b, a ? ie : b, a ? l : 0u, h ? part_of(v0, v1, qa, qe, ch, ct) : 0u);
  }
  pr.mark(k, w, lane, 5);
}



} // namespace
} // namespace tulips_amd
