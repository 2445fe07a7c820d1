// rss_route.hip — flow-affine routing of device-resident frames
// (tulips_csum_mctx_validate_frames_rss_device, csum_multi.hip): the GPU
// side of what a NIC does with RSS and an indirection table
// (src/transport/ena/RedirectionTable.cpp:74-98, hash per
// src/stack/Utils.cpp:86-133), on frames already in the source GPU's HBM.
//
//   route    one thread per frame: parse the 4-tuple from the frame bytes,
//            Toeplitz hash (LDS tables, rss_common.h), table[hash % len] ->
//            device; per-block histogram of frames and of 16-byte-rounded
//            bytes per device
//   scan     per device, exclusive prefix of the block histograms (frame
//            positions and packed-byte positions in device order)
//   scatter  one thread per frame: its position in device-major, arrival-
//            ordered lists (stable: wave ballots + wave scans per device),
//            writes perm / offset / length there
//   gather   one wave per frame bound for another device: its bytes copied
//            into that device's packed run on the source (16-byte aligned
//            starts), which then moves to the peer in one DMA
//   home     flags[perm[j]] = routed flags[j], counters from the flags
//
// Everything here runs on the source device's stream.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/tulips_csum.h"
#include "rss_common.h"
#include "rss_route.h"

namespace tulips_amd {
namespace {

constexpr int RT_BLOCK = 256;

__device__ __forceinline__ uint32_t
ld_byte(const uint8_t* p)
{
  return *reinterpret_cast<const __attribute__((address_space(1))) uint8_t*>(
    reinterpret_cast<uintptr_t>(p));
}

// The device of frame i and whether it has a routable 4-tuple: option-less
// IPv4, protocol 6, not a fragment (tulips_csum_mctx_validate_frames_rss_host
// takes the same decision on the host).
__device__ __forceinline__ uint32_t
route_one(const RssTables& t, const uint8_t* f, uint32_t flen, const uint16_t* table,
          uint32_t table_len, uint32_t init)
{
  if (flen < 38 || ld_byte(f + 12) != 0x08 || ld_byte(f + 13) != 0x00 ||
      ld_byte(f + 14) != 0x45 || ld_byte(f + 23) != 6 || (ld_byte(f + 20) & 0x3f) != 0 ||
      ld_byte(f + 21) != 0) {
    return table[0];
  }
  auto le32 = [&](int o) {
    return ld_byte(f + o) | (ld_byte(f + o + 1) << 8) | (ld_byte(f + o + 2) << 16) |
           (ld_byte(f + o + 3) << 24);
  };
  const uint32_t sp = (ld_byte(f + 34) << 8) | ld_byte(f + 35);
  const uint32_t dp = (ld_byte(f + 36) << 8) | ld_byte(f + 37);
  const uint32_t h = rss_one(t, le32(26), le32(30), sp, dp, init);
  return table[h % table_len];
}

__global__ __launch_bounds__(RT_BLOCK) void
rss_route_kernel(RssWindows win, const uint8_t* __restrict__ base,
                 const uint64_t* __restrict__ offs, const uint16_t* __restrict__ lens,
                 uint32_t n, const uint16_t* __restrict__ table, uint32_t table_len,
                 uint32_t init, uint32_t nd, uint16_t* __restrict__ dev_of,
                 uint32_t* __restrict__ blk_cnt, uint32_t* __restrict__ blk_bytes)
{
  __shared__ RssTables t;
  __shared__ uint32_t s_cnt[RT_MAX_DEV], s_bytes[RT_MAX_DEV];
  build_tables(win, t);
  for (uint32_t d = threadIdx.x; d < nd; d += blockDim.x) {
    s_cnt[d] = 0;
    s_bytes[d] = 0;
  }
  __syncthreads();
  const uint32_t i = blockIdx.x * RT_BLOCK + threadIdx.x;
  if (i < n) {
    const uint32_t flen = lens[i];
    const uint32_t d = route_one(t, base + offs[i], flen, table, table_len, init);
    dev_of[i] = uint16_t(d);
    atomicAdd(&s_cnt[d], 1u);
    atomicAdd(&s_bytes[d], (flen + 15u) & ~15u);
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < nd; d += blockDim.x) {
    blk_cnt[size_t(blockIdx.x) * nd + d] = s_cnt[d];
    blk_bytes[size_t(blockIdx.x) * nd + d] = s_bytes[d];
  }
}

// Block-wide exclusive scan of one value per thread (RT_BLOCK threads, four
// waves); returns the block total in *total.
__device__ __forceinline__ uint64_t
block_exclusive(uint64_t v, uint64_t* s_wave, uint64_t* total)
{
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o, 64);
    x += lane >= o ? y : 0;
  }
  if (lane == 63) {
    s_wave[wave] = x;
  }
  __syncthreads();
  uint64_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < RT_BLOCK / 64; ++w) {
    before += w < wave ? s_wave[w] : 0;
    all += s_wave[w];
  }
  __syncthreads();
  *total = all;
  return before + x - v;
}

// Block d: device d's column of the block histograms -> exclusive bases
// (frames and packed bytes, within the device), and its totals.
__global__ __launch_bounds__(RT_BLOCK) void
rss_route_scan_kernel(const uint32_t* __restrict__ blk_cnt,
                      const uint32_t* __restrict__ blk_bytes, uint32_t nblk, uint32_t nd,
                      uint32_t* __restrict__ base_cnt, uint64_t* __restrict__ base_bytes,
                      uint64_t* __restrict__ totals)
{
  __shared__ uint64_t s_wave[RT_BLOCK / 64];
  const uint32_t d = blockIdx.x;
  uint64_t carry_c = 0, carry_b = 0;
  for (uint32_t b0 = 0; b0 < nblk; b0 += RT_BLOCK) {
    const uint32_t b = b0 + threadIdx.x;
    const uint64_t c = b < nblk ? blk_cnt[size_t(b) * nd + d] : 0;
    const uint64_t y = b < nblk ? blk_bytes[size_t(b) * nd + d] : 0;
    uint64_t tc, ty;
    const uint64_t ec = block_exclusive(c, s_wave, &tc);
    const uint64_t ey = block_exclusive(y, s_wave, &ty);
    if (b < nblk) {
      base_cnt[size_t(b) * nd + d] = uint32_t(carry_c + ec);
      base_bytes[size_t(b) * nd + d] = carry_b + ey;
    }
    carry_c += tc;
    carry_b += ty;
  }
  if (threadIdx.x == 0) {
    totals[d] = carry_c;
    totals[nd + d] = carry_b;
  }
}

// Frame i's place in the device-major lists: device start + block base +
// earlier waves of the block + earlier lanes of the wave, for the frame
// count and (for the packed byte runs) the rounded bytes.
__global__ __launch_bounds__(RT_BLOCK) void
rss_route_scatter_kernel(const uint64_t* __restrict__ offs, const uint16_t* __restrict__ lens,
                         uint32_t n, uint32_t nd, uint32_t home,
                         const uint16_t* __restrict__ dev_of,
                         const uint32_t* __restrict__ base_cnt,
                         const uint64_t* __restrict__ base_bytes,
                         const uint64_t* __restrict__ totals, uint32_t* __restrict__ perm,
                         uint64_t* __restrict__ poff, uint16_t* __restrict__ plen)
{
  constexpr int NW = RT_BLOCK / 64;
  __shared__ uint32_t s_wc[NW][RT_MAX_DEV];
  __shared__ uint32_t s_wb[NW][RT_MAX_DEV];
  __shared__ uint32_t s_start[RT_MAX_DEV];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t i = blockIdx.x * RT_BLOCK + threadIdx.x;
  const bool live = i < n;
  const uint32_t mine = live ? dev_of[i] : 0xffffu;
  const uint32_t alen = live ? (uint32_t(lens[i]) + 15u) & ~15u : 0u;
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (uint32_t d = 0; d < nd; ++d) {
      s_start[d] = acc;
      acc += uint32_t(totals[d]);
    }
  }
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t rank = 0, brank = 0;
  for (uint32_t d = 0; d < nd; ++d) {
    const uint64_t m = __ballot(mine == d);
    if (m == 0) {
      if (lane == 0) {
        s_wc[wave][d] = 0;
        s_wb[wave][d] = 0;
      }
      continue;
    }
    uint32_t x = mine == d ? alen : 0u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      x += lane >= o ? y : 0u;
    }
    if (mine == d) {
      rank = uint32_t(__popcll(m & lt));
      brank = x - alen;
    }
    const uint32_t wtot = __shfl(x, 63, 64);
    if (lane == 0) {
      s_wc[wave][d] = uint32_t(__popcll(m));
      s_wb[wave][d] = wtot;
    }
  }
  __syncthreads();
  if (!live) {
    return;
  }
  uint32_t wc = 0, wb = 0;
  for (int w = 0; w < wave; ++w) {
    wc += s_wc[w][mine];
    wb += s_wb[w][mine];
  }
  const size_t cell = size_t(blockIdx.x) * nd + mine;
  const uint32_t pos = s_start[mine] + base_cnt[cell] + wc + rank;
  perm[pos] = i;
  plen[pos] = lens[i];
  poff[pos] = mine == home ? offs[i] : base_bytes[cell] + wb + brank;
}

// One wave per routed position j whose device is not `home`: the frame's
// bytes from the source arena into `packed` + pk_start[device] + poff[j]
// (a 16-byte aligned start), as dwords funnel-shifted from the aligned
// source dwords (loads clamped to the last dword holding a frame byte).
__global__ __launch_bounds__(RT_BLOCK) void
rss_route_gather_kernel(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
                        uint32_t n, uint32_t home, const uint16_t* __restrict__ dev_of,
                        const uint32_t* __restrict__ perm, const uint64_t* __restrict__ poff,
                        const uint16_t* __restrict__ plen, RouteStarts starts,
                        uint8_t* __restrict__ packed)
{
  typedef const __attribute__((address_space(1))) uint32_t* gdw;
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * (RT_BLOCK / 64);
  for (uint32_t j = blockIdx.x * (RT_BLOCK / 64) + (threadIdx.x >> 6); j < n; j += nwaves) {
    const uint32_t i = perm[j];
    const uint32_t d = dev_of[i];
    const uint32_t len = plen[j];
    if (d == home || len == 0) {
      continue;
    }
    const uintptr_t s = reinterpret_cast<uintptr_t>(base + offs[i]);
    const uintptr_t a = s & ~uintptr_t(3);
    const uint32_t r = uint32_t(s - a);
    const uint32_t last = uint32_t((s + len - 1 - a) >> 2);
    const gdw src = reinterpret_cast<gdw>(a);
    uint32_t* dst = reinterpret_cast<uint32_t*>(packed + starts.at[d] + poff[j]);
    const uint32_t nout = (len + 3) >> 2;
    for (uint32_t k = lane; k < nout; k += 64) {
      const uint32_t lo = src[min(k, last)];
      const uint32_t hi = src[min(k + 1, last)];
      dst[k] = r ? __builtin_amdgcn_alignbyte(hi, lo, r) : lo;
    }
  }
}

// flags[perm[j]] = rflags[j]; counters {IPv4, bad IP, TCP, bad L4} from the
// flags (the same counts tulips_csum_validate_frames keeps).
__global__ __launch_bounds__(RT_BLOCK) void
rss_route_home_kernel(const uint32_t* __restrict__ perm, const uint8_t* __restrict__ rflags,
                      uint32_t n, uint8_t* __restrict__ flags, uint32_t* __restrict__ counters)
{
  __shared__ uint32_t s_c[4];
  if (threadIdx.x < 4) {
    s_c[threadIdx.x] = 0;
  }
  __syncthreads();
  const uint32_t j = blockIdx.x * RT_BLOCK + threadIdx.x;
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  if (j < n) {
    const uint32_t f = rflags[j];
    if (flags) {
      flags[perm[j]] = uint8_t(f);
    }
    c0 = (f & TULIPS_FRAME_IPV4) ? 1u : 0u;
    c1 = c0 && !(f & TULIPS_FRAME_IP_CSUM_OK) ? 1u : 0u;
    c2 = (f & TULIPS_FRAME_TCP) ? 1u : 0u;
    c3 = c2 && !(f & TULIPS_FRAME_L4_CSUM_OK) ? 1u : 0u;
  }
  if (counters) {
    const uint64_t b0 = __ballot(c0), b1 = __ballot(c1), b2 = __ballot(c2), b3 = __ballot(c3);
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(&s_c[0], uint32_t(__popcll(b0)));
      atomicAdd(&s_c[1], uint32_t(__popcll(b1)));
      atomicAdd(&s_c[2], uint32_t(__popcll(b2)));
      atomicAdd(&s_c[3], uint32_t(__popcll(b3)));
    }
    __syncthreads();
    if (threadIdx.x < 4 && s_c[threadIdx.x]) {
      atomicAdd(&counters[threadIdx.x], s_c[threadIdx.x]);
    }
  }
}

} // namespace

bool
rss_route_windows(const uint8_t* key, size_t key_len, RouteWindows* out)
{
  static_assert(sizeof(RouteWindows) == sizeof(RssWindows), "windows");
  RssWindows w;
  if (!rss_windows(key, key_len, w)) {
    return false;
  }
  memcpy(out->w, w.w, sizeof(w.w));
  return true;
}

uint32_t
rss_route_blocks(uint32_t n)
{
  return (n + RT_BLOCK - 1) / RT_BLOCK;
}

hipError_t
launch_rss_route(const RouteWindows& win, const uint8_t* base, const uint64_t* offs,
                 const uint16_t* lens, uint32_t n, const uint16_t* table, uint32_t table_len,
                 uint32_t init, uint32_t nd, uint16_t* dev_of, uint32_t* blk_cnt,
                 uint32_t* blk_bytes, uint32_t* base_cnt, uint64_t* base_bytes,
                 uint64_t* totals, hipStream_t st)
{
  RssWindows w;
  memcpy(w.w, win.w, sizeof(w.w));
  const uint32_t nblk = rss_route_blocks(n);
  (void)hipGetLastError();
  hipLaunchKernelGGL(rss_route_kernel, dim3(nblk), dim3(RT_BLOCK), 0, st, w, base, offs, lens, n,
                     table, table_len, init, nd, dev_of, blk_cnt, blk_bytes);
  hipLaunchKernelGGL(rss_route_scan_kernel, dim3(nd), dim3(RT_BLOCK), 0, st, blk_cnt, blk_bytes,
                     nblk, nd, base_cnt, base_bytes, totals);
  return hipGetLastError();
}

hipError_t
launch_rss_scatter(const uint64_t* offs, const uint16_t* lens, uint32_t n, uint32_t nd,
                   uint32_t home, const uint16_t* dev_of, const uint32_t* base_cnt,
                   const uint64_t* base_bytes, const uint64_t* totals, uint32_t* perm,
                   uint64_t* poff, uint16_t* plen, hipStream_t st)
{
  (void)hipGetLastError();
  hipLaunchKernelGGL(rss_route_scatter_kernel, dim3(rss_route_blocks(n)), dim3(RT_BLOCK), 0, st,
                     offs, lens, n, nd, home, dev_of, base_cnt, base_bytes, totals, perm, poff,
                     plen);
  return hipGetLastError();
}

hipError_t
launch_rss_gather(const uint8_t* base, const uint64_t* offs, uint32_t n, uint32_t home,
                  const uint16_t* dev_of, const uint32_t* perm, const uint64_t* poff,
                  const uint16_t* plen, const RouteStarts& starts, uint8_t* packed,
                  hipStream_t st)
{
  const uint32_t waves = std::min<uint32_t>(n, 256u * 64u);
  const uint32_t blocks = (waves + RT_BLOCK / 64 - 1) / (RT_BLOCK / 64);
  (void)hipGetLastError();
  hipLaunchKernelGGL(rss_route_gather_kernel, dim3(blocks), dim3(RT_BLOCK), 0, st, base, offs, n,
                     home, dev_of, perm, poff, plen, starts, packed);
  return hipGetLastError();
}

hipError_t
launch_rss_home(const uint32_t* perm, const uint8_t* rflags, uint32_t n, uint8_t* flags,
                uint32_t* counters, hipStream_t st)
{
  (void)hipGetLastError();
  if (counters) {
    if (hipMemsetAsync(counters, 0, 4 * sizeof(uint32_t), st) != hipSuccess) {
      return hipGetLastError();
    }
  }
  if (n) {
    hipLaunchKernelGGL(rss_route_home_kernel, dim3(rss_route_blocks(n)), dim3(RT_BLOCK), 0, st,
                       perm, rflags, n, flags, counters);
  }
  return hipGetLastError();
}

} // namespace tulips_amd
