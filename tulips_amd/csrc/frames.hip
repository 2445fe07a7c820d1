// frames.hip — batched receive-side validation of Ethernet/IPv4/TCP frames
// (SURVEY.md §8f #1/#2): the checks the reference stack applies to a frame
// before its segment reaches TCP, done for a whole poll burst in one launch,
// producing per-frame flags in the manner of a NIC's checksum offload result
// (what transport::Device::VALIDATE_IP_CSUM / VALIDATE_L4_CSUM act on,
// include/tulips/transport/Device.h:29-30; src/transport/ena/Device.cpp:
// 318-340, src/transport/ofed/Device.cpp:530-545).
//
//   ethernet/Processor.cpp:69,91    ethertype 0x0800 -> IPv4
//   ipv4/Processor.cpp:67-73        vhl == 0x45 (no options)
//   ipv4/Processor.cpp:77-82        no fragments
//   ipv4/Processor.cpp:94-103       ipv4::checksum(header) == 0xffff
//   ipv4/Processor.cpp:108,116-122  proto 6 -> TCP over ntohs(len) - 20 bytes
//   tcpv4/Processor.cpp:121-131     tcpv4 checksum == 0xffff
//
// One 32-lane subgroup per frame: lanes 0..23 fetch header bytes 12..35 and
// the subgroup shares them by cross-lane shuffles, then the IPv4 header and
// the TCP segment are summed with the same absolute-chunk machinery as the
// checksum kernels (csum_kernels.hip) and finished per csum_common.h.
//
// The send side is here too: in-place generation of both
// checksum fields for a burst of frames, as ipv4/Producer.cpp:79-82 and
// tcpv4/Send.cpp:441-449 write them (the job of the NIC's IBV_SEND_IP_CSUM /
// checksum offload in src/transport/ofed/Device.cpp:756).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <mutex>

#include "../../include/tulips_csum.h"
#include "csum_common.h"
#include "csum_launch.h"
#include "frame_common.h"
#include "stream_state.h"
#include "zc_mailbox.h"

namespace tulips_amd {
namespace {

using namespace frame;


// One G-lane subgroup per frame (two frames per wave), frames taken in
// grid-stride order. The whole frame is loaded (load_frame) as soon as its
// offset/length arrive, and the next frame's offset/length are fetched
// behind those loads, so a frame costs one memory round trip. Header fields
// and the IPv4 header's sum come from the same registers (frame_header_ip),
// and the TCP range is summed from them (range_sum32).
//
// GENERATE = false: receive-side validation -> flags / counters.
// GENERATE = true:  send-side generation (ipv4/Producer.cpp:79-82
//   `ipchksum = ~checksum(header)`, tcpv4/Send.cpp:441-449 `chksum = ~csum`);
//   each field's current bytes are taken out of the sum arithmetically
//   (field_contrib), so the frame is read once and 4 bytes are written.
// Geometry: FG lanes x FU chunks in flight per frame. The default, 16 x 6
// (4 frames per wave, 96 chunks = a 1514 B frame in one batch, nt loads), is
// the best of tools/sessions/probes/probe_frames.py's sweep on 1514 B frames
// (profiles/probe_frames_r01.json).
// Minimum waves per SIMD the register allocator must leave room for
// (0 = no bound). Generation: 94 -> 80 VGPRs, 5 -> 6 waves/SIMD, no spill;
// 3 alternations on one box (profiles/ab_r01.txt): 21.2-22.0 -> 20.8-21.4 us
// serial, 19.4-19.7 -> 18.7-19.0 us on 4 branches. Validation at 7 waves
// spills 12 B and is slower. The generation bound applies to the default
// geometry and smaller (U <= 6): at 16 x 8 and 8 x 8/16 it spilled 12-364 B
// per lane, so those keep their natural register counts.
constexpr int FRAME_VAL_WAVES = 0, FRAME_GEN_WAVES = 6, FRAME_FPS2_WAVES = 0;

// OP: 0 = validate (flags, counters), 1 = generate in place (the two
// checksum fields patched into the frame; `fields` optionally gets a copy),
// 2 = generate compact fields only (frames untouched, one u32 per frame).
enum { OP_VALIDATE = 0, OP_GENERATE = 1, OP_FIELDS = 2 };

// FPS: frames per subgroup in flight. With FPS = 2 a subgroup issues the
// loads of two frames (f and f + nsub) before summing either, so a wave keeps
// twice the bytes in flight at the same instruction count per byte, and the
// grid is half as many workgroups.
template<int OP, int FG, int FU, bool NT, int FPS = 1>
__global__ __launch_bounds__(FPS == 3 ? 256 : 1024, FPS >= 2 ? FRAME_FPS2_WAVES : OP != OP_VALIDATE && FU <= 6 ? FRAME_GEN_WAVES : FRAME_VAL_WAVES) void
frame_kernel(uint8_t* base, const uint64_t* __restrict__ offs,
             const uint16_t* __restrict__ lens, uint32_t n,
             uint8_t* __restrict__ flags, uint32_t* __restrict__ shards,
             uint32_t* __restrict__ fields)
{
  constexpr bool GENERATE = OP != OP_VALIDATE;
  const int lane64 = threadIdx.x & 63;
  const int lane = lane64 & (FG - 1);
  const int sub0 = lane64 - lane; // first lane of this subgroup
  const uint32_t per_block = blockDim.x / FG;
  const uint32_t nsub = gridDim.x * per_block;
  uint32_t f = xcd_block(blockIdx.x, gridDim.x) * per_block + threadIdx.x / FG;
  // counters: per-block totals in LDS, then one atomic per non-zero counter
  // per block into one of CNT_SHARDS line-sized shards (finalised by
  // frame_counters_finalize). Adding every frame to the caller's 4 words
  // directly serialised ~33k same-address atomics: 378 us per 65,536-frame
  // launch instead of 18 (tools/sessions/probes/probe_counters.py).
  __shared__ uint32_t s_cnt[4];
  const bool count = !GENERATE && shards != nullptr;   // grid-uniform
  if (count) {
    if (threadIdx.x < 4) {
      s_cnt[threadIdx.x] = 0;
    }
    __syncthreads();
  }
  // frame `g` at address fa (length flen) from its loaded chunks
  auto one = [&](const FrameChunks<FG, FU>& fc, uint32_t g, uintptr_t fa, uint32_t flen) {
    // The IPv4 header's sum comes from the header words every lane already
    // holds (frame-relative, so the header starts at an even offset of that
    // word grid and its checksum field at 24): no range sum and no subgroup
    // reduction for it. Against the range sum over the chunk registers:
    // validation 0.68 -> 0.71 serial, 0.85 -> 0.87 on 4 branches; fields and
    // in-place generation +1 % (profiles/ab_frame_ip_header_r06.txt).
    uint32_t ipsum = 0;
    const Header h = frame_header_ip(fc, flen, sub0, ipsum);
    const uint32_t ip_part = h.ipv4 ? ipsum : 0u;
    constexpr bool ip_odd = false;
    constexpr uintptr_t ip_field = 24;
    const int h0 = fc.h0;
    const bool do_l4 = h.tcp && !h.trunc && (!GENERATE || h.tcplen >= 18u);
    // (32-bit v_dot2 accumulation, masks on the boundary chunks only: 4
    // branches +1.5 % against 64-bit adds, profiles/ab_frame_ip_header_r06.txt)
    const uint32_t l4_part = sub_sum<FG>(
      do_l4 ? tcp_range_part<FG, FU, NT>(fc, lane, h0 + 34, h0 + 34 + int(h.tcplen)) : 0u);
    // generation: both field values, on every lane (the sums and the header
    // are subgroup-uniform)
    uint32_t ipv = 0, l4v = 0;
    if constexpr (GENERATE) {
      if (h.ipv4) {
        const uint32_t p =
          fold32(ip_part) + (0xffffu - field_contrib(ip_field, h.ipck0, h.ipck1));
        ipv = ~finish(p, ip_odd, MODE_INET, 0, 0, 0, 20) & 0xffffu;
      }
      if (do_l4) {
        const uint32_t p =
          fold32(l4_part) + (0xffffu - field_contrib(fa + 50, h.tcpck0, h.tcpck1));
        l4v = ~finish(p, ((fa + 34) & 1) != 0, MODE_TCP, 0, h.src, h.dst, h.tcplen) & 0xffffu;
      }
    }
    if (lane == 0) {
      if (GENERATE) {
        uint32_t written = 0;
        if (h.ipv4) {
          if constexpr (OP == OP_GENERATE) {
            store_field(fa + 24, ipv);
          }
          written = ipv;
        }
        if (do_l4) {
          if constexpr (OP == OP_GENERATE) {
            store_field(fa + 50, l4v);
          }
          written |= l4v << 16;
        }
        if (fields) {
          // the two field values as stored (the u16s a little-endian load of
          // the header words gives): what tulips_csum_generate_frames_host
          // patches into the host copy, and tulips_csum_generate_fields'
          // whole output
          fields[g] = written;
        }
        if (flags) {
          flags[g] = uint8_t(frame_flags(h, h.ipv4, do_l4));
        }
      } else {
        const bool ip_ok = h.ipv4 && finish(ip_part, ip_odd, MODE_INET, 0, 0, 0, 20) == 0xffffu;
        const bool l4_ok = do_l4 && finish(l4_part, ((fa + 34) & 1) != 0, MODE_TCP, 0,
                                           h.src, h.dst, h.tcplen) == 0xffffu;
        if (flags) {
          flags[g] = uint8_t(frame_flags(h, ip_ok, l4_ok));
        }
        if (count) {
          if (h.ipv4) {
            atomicAdd(&s_cnt[0], 1u);
            if (!ip_ok) {
              atomicAdd(&s_cnt[1], 1u);
            }
          }
          if (h.tcp) {
            atomicAdd(&s_cnt[2], 1u);
            if (!l4_ok) {
              atomicAdd(&s_cnt[3], 1u);
            }
          }
        }
      }
    }
  };
  if (f < n) {
    // frames f (and f + nsub when FPS == 2) per round; the next round's
    // offsets and lengths are fetched behind this round's loads
    static_assert(FPS >= 1 && FPS <= 3, "frames per subgroup");
    const uintptr_t b0 = reinterpret_cast<uintptr_t>(base);
    auto meta = [&](uint32_t g, uint64_t& o, uint32_t& l) {
      o = offs[min(g, n - 1)];
      l = g < n ? uint32_t(lens[min(g, n - 1)]) : 0u;
    };
    uint64_t o0, o1 = 0;
    uint32_t l0, l1 = 0;
    meta(f, o0, l0);
    if constexpr (FPS == 3) {
      // software pipeline over the subgroup's frames f, f + nsub, ...: the
      // next frame's loads are issued before this one is summed
      FrameChunks<FG, FU> fa;
      load_frame<FG, FU, NT>(b0 + o0, l0, lane, fa);
      while (true) {
        const uint32_t fn = f + nsub;
        meta(fn, o1, l1);
        FrameChunks<FG, FU> fb;
        load_frame<FG, FU, NT>(b0 + o1, l1, lane, fb); // (clamped: frame n - 1 past the end)
        one(fa, f, b0 + o0, l0);
        if (fn >= n) {
          break;
        }
        f = fn;
        o0 = o1;
        l0 = l1;
        fa = fb;
      }
    }
    if constexpr (FPS == 2) {
      meta(f + nsub, o1, l1);
    }
    while (FPS != 3) {
      FrameChunks<FG, FU> fc0, fc1;
      load_frame<FG, FU, NT>(b0 + o0, l0, lane, fc0);
      if constexpr (FPS == 2) {
        load_frame<FG, FU, NT>(b0 + o1, l1, lane, fc1);
      }
      const uint32_t fn = f + uint32_t(FPS) * nsub;
      uint64_t p0, p1 = 0;
      uint32_t q0, q1 = 0;
      meta(fn, p0, q0);
      if constexpr (FPS == 2) {
        meta(fn + nsub, p1, q1);
      }
      one(fc0, f, b0 + o0, l0);
      if constexpr (FPS == 2) {
        if (f + nsub < n) {
          one(fc1, f + nsub, b0 + o1, l1);
        }
      }
      if (fn >= n) {
        break;
      }
      f = fn;
      o0 = p0;
      l0 = q0;
      o1 = p1;
      l1 = q1;
    }
  }
  if (count) {
    __syncthreads();
    if (threadIdx.x < 4) {
      const uint32_t v = s_cnt[threadIdx.x];
      if (v) {
        atomicAdd(shards + CNT_LINE * (blockIdx.x % CNT_SHARDS) + threadIdx.x, v);
      }
    }
  }
}

// ---- low-latency receive validation (zc_mailbox.h) --------------------------
//
// One workgroup of 64 16-lane subgroups serves the context's mailbox. Every
// subgroup validates frames f, f + 64, ... of a request exactly as
// frame_kernel<VALIDATE> does, reading them from the caller's page-locked
// arena over PCIe; the flags and counters go back into the mailbox before
// `done` is published with a system-scope release. RESIDENT: wave 0 polls
// the doorbell (system-scope acquire loads) and the workgroup serves one
// request after another until `stop` or ZC_IDLE_TICKS without one (every
// wave leaves through the same barrier); otherwise the workgroup serves the
// request `seq` (already posted) and exits. Control flow around the
// barriers is wave-uniform (readfirstlane), so every wave takes every
// barrier.
template<bool RESIDENT>
__global__ __launch_bounds__(1024) void
zc_server_kernel(ZcMailbox* mb, ZcArgs args)
{
  constexpr int FG = 16, FU = 6;
  __shared__ uint64_t s_req[ZC_REQ_WORDS];
  __shared__ uint32_t s_exit;
  __shared__ uint32_t s_cnt[4];
  const int lane64 = threadIdx.x & 63;
  const int lane = lane64 & (FG - 1);
  const int sub0 = lane64 - lane;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // subgroup g of workgroup w takes frames (w * nsub + g) + k * gridDim.x * nsub
  const uint32_t wg = blockIdx.x;
  const uint32_t sub = wg * (blockDim.x / FG) + threadIdx.x / FG;
  const uint32_t nsub = gridDim.x * (blockDim.x / FG);
  // the last tag this workgroup served (resident) / the request (one launch)
  uint32_t served = RESIDENT ? uint32_t(__hip_atomic_load(&mb->done[wg], __ATOMIC_ACQUIRE,
                                                          __HIP_MEMORY_SCOPE_SYSTEM))
                             : 0u;
  for (;;) {
    if (wave == 0) {
      uint32_t ex = 0;
      uint64_t w = 0;
      if (RESIDENT) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (uint32_t polls = 1;; ++polls) {
          w = __hip_atomic_load(&mb->req[lane64], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          const uint32_t tag = uint32_t(w >> 48);
          const uint32_t tag0 = __builtin_amdgcn_readfirstlane(tag);
          if ((polls & 1023u) == 0 && lane64 == 0 && wg == 0) {
            __hip_atomic_store(&mb->beat, uint64_t(polls >> 10), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&mb->seen, uint64_t(tag0), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
          }
          if (tag0 != (served & 0xffffu)) {
            // a new request: every word it needs must carry its tag
            const uint32_t n0 = __builtin_amdgcn_readfirstlane(uint32_t(w & 0xffffu));
            const uint32_t need = 2u + (n0 <= ZC_REQ_FRAMES ? n0 : 0u);
            if (__builtin_amdgcn_ballot_w64(uint32_t(lane64) < need && tag != tag0) == 0) {
              break;
            }
            continue; // caught the host mid-write
          }
          const uint32_t stop = __builtin_amdgcn_readfirstlane(uint32_t(
            __hip_atomic_load(&mb->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)));
          if (stop != 0 || __builtin_amdgcn_s_memrealtime() - t0 > ZC_IDLE_TICKS) {
            ex = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      } else {
        // the request as kernel arguments, in the same word format
        const uint32_t tag = uint32_t(args.seq);
        const uint32_t k = uint32_t(lane64) - 2u;
        w = lane64 == 0   ? zc_word(tag, args.n)
            : lane64 == 1 ? zc_word(tag, args.base)
            : k < min(args.inline_n, ZC_ARG_FRAMES)
              ? zc_word(tag, (uint64_t(args.off[k]) << 16) | args.len[k])
              : 0ull;
      }
      s_req[lane64] = w;
      if (lane64 == 0) {
        s_exit = ex;
        s_cnt[0] = s_cnt[1] = s_cnt[2] = s_cnt[3] = 0;
      }
      // the frames (and any descriptor arrays) as the host left them: one
      // invalidate of this CU's L1 and of L2 serves every wave of the
      // workgroup (they load only after the barrier)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(s_exit) != 0) {
      break;
    }
    const uint64_t t_req = __builtin_amdgcn_s_memrealtime();
    const uint32_t tag = uint32_t(s_req[0] >> 48);
    const uint32_t n = min(uint32_t(s_req[0] & 0xffffu), ZC_MAX_FRAMES);
    const uintptr_t base = uintptr_t(s_req[1] & 0xffffffffffffull);
    const bool inl = RESIDENT ? n <= ZC_REQ_FRAMES : args.inline_n != 0;
    for (uint32_t f = sub; f < n; f += nsub) {
      uint64_t off;
      uint32_t flen;
      if (inl) {
        const uint64_t d = s_req[2 + f];
        off = (d >> 16) & 0xffffffffull;
        flen = uint32_t(d & 0xffffu);
      } else {
        off = mb->offs[f];
        flen = mb->lens[f];
      }
      const uintptr_t fa = base + off;
      FrameChunks<FG, FU> fc;
      load_frame<FG, FU, false>(fa, flen, lane, fc);
      uint32_t ipsum = 0; // (as frame_kernel: from the header words)
      const Header h = frame_header_ip(fc, flen, sub0, ipsum);
      const int h0 = fc.h0;
      const bool do_l4 = h.tcp && !h.trunc;
      const uint32_t ip_part = h.ipv4 ? ipsum : 0u;
      const uint32_t l4_part = sub_sum<FG>(
        do_l4 ? tcp_range_part<FG, FU, false>(fc, lane, h0 + 34, h0 + 34 + int(h.tcplen)) : 0u);
      if (lane == 0) {
        const bool ip_ok = h.ipv4 && finish(ip_part, false, MODE_INET, 0, 0, 0, 20) == 0xffffu;
        const bool l4_ok = do_l4 && finish(l4_part, ((fa + 34) & 1) != 0, MODE_TCP, 0, h.src,
                                           h.dst, h.tcplen) == 0xffffu;
        mb->flags[f] = uint8_t(frame_flags(h, ip_ok, l4_ok));
        if (h.ipv4) {
          atomicAdd(&s_cnt[0], 1u);
          if (!ip_ok) {
            atomicAdd(&s_cnt[1], 1u);
          }
        }
        if (h.tcp) {
          atomicAdd(&s_cnt[2], 1u);
          if (!l4_ok) {
            atomicAdd(&s_cnt[3], 1u);
          }
        }
      }
    }
    // this wave's flag stores (to the uncached, host-coherent mailbox) are
    // complete before the barrier; thread 0's system-scope release then
    // publishes them with `done`
    __builtin_amdgcn_s_waitcnt(0x0f70); // vmcnt(0) expcnt(7) lgkmcnt(15)
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int k = 0; k < 4; ++k) {
        __hip_atomic_store(&mb->counters[wg][k], s_cnt[k], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (wg == 0) {
        __hip_atomic_store(&mb->t_req, t_req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&mb->t_done, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
      __hip_atomic_store(&mb->done[wg], uint64_t(tag), __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (!RESIDENT) {
      break;
    }
    served = tag;
    __syncthreads(); // s_req / s_cnt are rewritten by the next poll
  }
}

// Sums the shards into the caller's counters and zeroes them for the next
// call on this stream (atomic exchange: read and cleared where the adds
// landed).
__global__ __launch_bounds__(64) void
frame_counters_finalize(uint32_t* __restrict__ shards, uint32_t* __restrict__ counters,
                        uint32_t nout)
{
  // lane l takes counter l & 3 of shards l >> 2 and (l >> 2) + 16: all 128
  // exchanges in flight at once, then a sum over the lanes of each counter
  static_assert(CNT_SHARDS == 32, "64 lanes x 2 shards");
  const uint32_t l = threadIdx.x, k = l & 3u, j = l >> 2;
  const uint32_t a = atomicExch(shards + CNT_LINE * j + k, 0u);
  const uint32_t b = atomicExch(shards + CNT_LINE * (j + 16) + k, 0u);
  uint32_t sum = a + b;
#pragma unroll
  for (int m = 4; m < 64; m <<= 1) {
    sum += __shfl_xor(sum, m);
  }
  if (l < nout) {
    counters[k] = sum;
  }
}

constexpr int DEFAULT_G = 16, DEFAULT_U = 6;

template<int OP, int G, int U, bool NT>
hipError_t
launch_one(uint8_t* base, const uint64_t* offs, const uint16_t* lens, uint32_t n,
           uint8_t* flags, uint32_t* counters, uint32_t* fields, const FrameLaunch& fl,
           hipStream_t stream)
{
  const uint32_t block = fl.block ? fl.block : 256;
  const bool tuned = OP == OP_VALIDATE && G == 16 && U == 6;
  const uint32_t fps = (tuned && (fl.fps == 2 || fl.fps == 3)) ? uint32_t(fl.fps) : 1u;
  // fps 3 (pipelined): about four frames per subgroup
  const uint32_t per_block = block / G * (fps == 1 ? 1u : fps == 2 ? 2u : 4u);
  uint64_t blocks = (uint64_t(n) + per_block - 1) / per_block;
  const uint64_t cap = fl.max_blocks ? fl.max_blocks : 65535;
  if (blocks > cap) {
    blocks = cap;
  }
  (void)hipGetLastError();
  if constexpr (OP == OP_VALIDATE && G == 16 && U == 6) {
    if (fps == 2) {
      hipLaunchKernelGGL((frame_kernel<OP, G, U, NT, 2>), dim3(uint32_t(blocks)),
                         dim3(block), 0, stream, base, offs, lens, n, flags, counters, fields);
      return hipGetLastError();
    }
    if (fps == 3) {
      hipLaunchKernelGGL((frame_kernel<OP, G, U, NT, 3>), dim3(uint32_t(blocks)),
                         dim3(block), 0, stream, base, offs, lens, n, flags, counters, fields);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((frame_kernel<OP, G, U, NT>), dim3(uint32_t(blocks)),
                     dim3(block), 0, stream, base, offs, lens, n, flags, counters, fields);
  return hipGetLastError();
}

template<int OP>
hipError_t
dispatch(uint8_t* base, const uint64_t* offs, const uint16_t* lens, uint32_t n,
         uint8_t* flags, uint32_t* counters, uint32_t* fields, const FrameLaunch& fl,
         hipStream_t stream)
{
  const int g = fl.group ? fl.group : DEFAULT_G, u = fl.unroll ? fl.unroll : DEFAULT_U;
  const bool nt = fl.nontemporal != 0;
#define TCS_F(G, U)                                                            \
  if (g == G && u == U) {                                                      \
    return nt ? launch_one<OP, G, U, true>(base, offs, lens, n, flags, counters, \
                                           fields, fl, stream)                 \
              : launch_one<OP, G, U, false>(base, offs, lens, n, flags, counters,\
                                            fields, fl, stream);               \
  }
  TCS_F(16, 4)
  TCS_F(16, 6)
  TCS_F(16, 8)
  TCS_F(8, 8)
  TCS_F(8, 16)
  TCS_F(32, 3)
  TCS_F(32, 4)
  TCS_F(64, 2)
#undef TCS_F
  return hipErrorInvalidValue;
}

} // namespace

bool
frame_geometry_ok(int group, int unroll, uint32_t block)
{
  const int g = group ? group : DEFAULT_G, u = unroll ? unroll : DEFAULT_U;
  const bool geo = (g == 16 && (u == 4 || u == 6 || u == 8)) ||
                   (g == 8 && (u == 8 || u == 16)) || (g == 32 && (u == 3 || u == 4)) ||
                   (g == 64 && u == 2);
  return geo && (block == 0 || block == 64 || block == 128 || block == 256 || block == 512 ||
                 block == 1024);
}

hipError_t
launch_zc_server(ZcMailbox* mb, const ZcArgs* oneshot, hipStream_t stream)
{
  (void)hipGetLastError();
  if (oneshot) {
    // a burst of up to 62 frames: one workgroup of a 16-lane subgroup per
    // frame; more: one 1024-thread workgroup per 64 frames
    const uint32_t n = oneshot->n;
    const uint32_t threads =
      oneshot->inline_n ? min(1024u, 64u * ((oneshot->inline_n + 3) / 4)) : 1024u;
    const uint32_t wgs = oneshot->inline_n ? 1u : min(ZC_MAX_WG, (n + 63) / 64);
    hipLaunchKernelGGL(zc_server_kernel<false>, dim3(wgs), dim3(threads), 0, stream, mb,
                       *oneshot);
  } else {
    hipLaunchKernelGGL(zc_server_kernel<true>, dim3(ZC_RES_WG), dim3(1024), 0, stream, mb,
                       ZcArgs{});
  }
  return hipGetLastError();
}

hipError_t
launch_counters_finalize(uint32_t* shards, uint32_t* out, uint32_t nout,
                         hipStream_t stream)
{
  hipLaunchKernelGGL(frame_counters_finalize, dim3(1), dim3(64), 0, stream, shards,
                     out, nout);
  return hipGetLastError();
}

// counters (device uint32[4], may be null) are overwritten with this call's
// totals, in stream order (zeroed for n == 0). The count kernel and the
// finalize are queued under the stream's call mutex (stream_state.h).
hipError_t
launch_frames(const uint8_t* base, const uint64_t* offs, const uint16_t* lens,
              uint32_t n, uint8_t* flags, uint32_t* counters, hipStream_t stream,
              const FrameLaunch& fl)
{
  if (n == 0) {
    return counters ? hipMemsetAsync(counters, 0, 4 * sizeof(uint32_t), stream)
                    : hipSuccess;
  }
  if (!counters) {
    return dispatch<OP_VALIDATE>(const_cast<uint8_t*>(base), offs, lens, n, flags, nullptr,
                                 nullptr, fl, stream);
  }
  std::shared_ptr<StreamState> ss;
  hipError_t e = stream_state(stream, &ss);
  if (e != hipSuccess) {
    return e;
  }
  const bool capturing = stream_capturing(stream);
  std::lock_guard<std::recursive_mutex> g(ss->call);
  uint32_t* shards = nullptr;
  if ((e = call_shards(*ss, capturing, &shards)) != hipSuccess) {
    return e;
  }
  e = dispatch<OP_VALIDATE>(const_cast<uint8_t*>(base), offs, lens, n, flags, shards,
                            nullptr, fl, stream);
  if (e == hipSuccess) {
    e = launch_counters_finalize(shards, counters, 4, stream);
  }
  if (e != hipSuccess && !capturing) {
    drop_shards(*ss, shards);
  }
  return e;
}

hipError_t
launch_generate(uint8_t* base, const uint64_t* offs, const uint16_t* lens,
                uint32_t n, uint8_t* flags, hipStream_t stream, const FrameLaunch& fl,
                uint32_t* fields)
{
  if (n == 0) {
    return hipSuccess;
  }
  return dispatch<OP_GENERATE>(base, offs, lens, n, flags, nullptr, fields, fl, stream);
}

hipError_t
launch_generate_fields(const uint8_t* base, const uint64_t* offs, const uint16_t* lens,
                       uint32_t n, uint32_t* fields, uint8_t* flags, hipStream_t stream,
                       const FrameLaunch& fl)
{
  if (n == 0) {
    return hipSuccess;
  }
  return dispatch<OP_FIELDS>(const_cast<uint8_t*>(base), offs, lens, n, flags, nullptr,
                             fields, fl, stream);
}

} // namespace tulips_amd

extern "C" int
tulips_csum_validate_frames(const uint8_t* base, const uint64_t* offsets,
                            const uint16_t* lengths, uint32_t n, uint8_t* flags,
                            uint32_t* counters, void* stream)
{
  if (n == 0) {
    // counters are still this call's totals (zero), like tulips_csum_verify
    return !counters || hipMemsetAsync(counters, 0, 4 * sizeof(uint32_t),
                                       static_cast<hipStream_t>(stream)) == hipSuccess
             ? TULIPS_STATUS_OK
             : TULIPS_STATUS_HARDWARE_ERROR;
  }
  if (!base || !offsets || !lengths || (!flags && !counters)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  const hipError_t e =
    tulips_amd::launch_frames(base, offsets, lengths, n, flags, counters, st);
  return e == hipSuccess                         ? TULIPS_STATUS_OK
         : e == hipErrorStreamCaptureUnsupported ? TULIPS_STATUS_INVALID_ARGUMENT
                                                 : TULIPS_STATUS_HARDWARE_ERROR;
}

extern "C" int
tulips_csum_generate_frames(uint8_t* base, const uint64_t* offsets,
                            const uint16_t* lengths, uint32_t n, uint8_t* flags,
                            void* stream)
{
  if (n == 0) {
    return TULIPS_STATUS_OK;
  }
  if (!base || !offsets || !lengths) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  const hipError_t e = tulips_amd::launch_generate(
    base, offsets, lengths, n, flags, static_cast<hipStream_t>(stream));
  return e == hipSuccess ? TULIPS_STATUS_OK : TULIPS_STATUS_HARDWARE_ERROR;
}

extern "C" int
tulips_csum_generate_fields(const uint8_t* base, const uint64_t* offsets,
                            const uint16_t* lengths, uint32_t n, uint32_t* fields,
                            uint8_t* flags, void* stream)
{
  if (n == 0) {
    return TULIPS_STATUS_OK;
  }
  if (!base || !offsets || !lengths || !fields) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  const hipError_t e = tulips_amd::launch_generate_fields(
    base, offsets, lengths, n, fields, flags, static_cast<hipStream_t>(stream));
  return e == hipSuccess ? TULIPS_STATUS_OK : TULIPS_STATUS_HARDWARE_ERROR;
}

extern "C" int
tulips_csum_frames_tuned(int op, uint8_t* base, const uint64_t* offsets,
                         const uint16_t* lengths, uint32_t n, uint8_t* flags,
                         uint32_t* counters, const tulips_csum_tuning* tuning,
                         void* stream)
{
  if ((op != 0 && op != 1 && op != 2) || !tuning ||
      !tulips_amd::frame_geometry_ok(tuning->group, tuning->unroll,
                                     uint32_t(tuning->block < 0 ? 0 : tuning->block))) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  // the pipelined validation kernel (sps 3) is compiled for at most 256
  // threads per block (__launch_bounds__ of frame_kernel<..., 3>)
  if (op == 0 && tuning->sps == 3 && tuning->block > 256) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (n == 0 && !(op == 0 && counters)) {
    return TULIPS_STATUS_OK;
  }
  if (n && (!base || !offsets || !lengths || (op == 0 && !flags && !counters) ||
            (op == 2 && !counters))) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  tulips_amd::FrameLaunch fl;
  fl.group = tuning->group;
  fl.unroll = tuning->unroll;
  fl.max_blocks = tuning->max_blocks;
  fl.block = uint32_t(tuning->block < 0 ? 0 : tuning->block);
  fl.nontemporal = tuning->nontemporal < 0 ? 1 : (tuning->nontemporal & 1);
  fl.fps = (tuning->sps == 2 || tuning->sps == 3) ? tuning->sps : 1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e;
  if (op == 0) {
    e = tulips_amd::launch_frames(base, offsets, lengths, n, flags, counters, st, fl);
  } else if (op == 2) {
    // `counters` carries the n-entry fields array
    e = tulips_amd::launch_generate_fields(base, offsets, lengths, n, counters, flags, st, fl);
  } else {
    e = tulips_amd::launch_generate(base, offsets, lengths, n, flags, st, fl);
  }
  return e == hipSuccess                         ? TULIPS_STATUS_OK
         : e == hipErrorStreamCaptureUnsupported ? TULIPS_STATUS_INVALID_ARGUMENT
                                                 : TULIPS_STATUS_HARDWARE_ERROR;
}
