// csum_common.h — arithmetic shared by the host drop-ins and the gfx950
// kernels. Everything here is a restatement of one closed form of the
// reference loop (src/stack/Utils.cpp:14-42):
//
//   S = seed + sum_k BE16(d[2k], d[2k+1]) + (len odd ? d[len-1] << 8 : 0)
//   checksum(seed, d, len) = S == 0 ? 0 : ((S - 1) mod 65535) + 1
//
// i.e. an end-around-carry adder that never turns a non-zero sum into 0.
// Because 2^16 == 1 (mod 65535), any reduction order/width is exact once the
// final fold is applied, and a little-endian word sum equals the big-endian
// one byte-swapped when the segment starts at an even address.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define TCS_HD __host__ __device__ __forceinline__
#else
#define TCS_HD inline
#endif

namespace tulips_amd {

constexpr uint32_t MODE_RAW = 0, MODE_INET = 1, MODE_TCP = 2;
constexpr uint32_t MODE_MASK = 0xff, FLAG_COMPLEMENT = 0x100;

// x mod 65535 with 0 kept distinct from 65535: result in [0, 0x3fffc],
// zero iff x == 0.
TCS_HD uint32_t fold64(uint64_t x)
{
  return uint32_t(x & 0xffff) + uint32_t((x >> 16) & 0xffff) +
         uint32_t((x >> 32) & 0xffff) + uint32_t(x >> 48);
}

// Any 32-bit partial -> [0, 0xffff], zero iff x == 0.
TCS_HD uint32_t fold32(uint32_t x)
{
  x = (x & 0xffff) + (x >> 16);
  x = (x & 0xffff) + (x >> 16);
  return x;
}

TCS_HD uint32_t bswap16(uint32_t v)
{
  return ((v & 0xff) << 8) | ((v >> 8) & 0xff);
}

// One's-complement add of a 16-bit seed to a folded 16-bit partial.
TCS_HD uint32_t add_seed(uint32_t r, uint32_t seed)
{
  uint32_t t = r + seed;
  return (t & 0xffff) + (t >> 16);
}

// Big-endian word sum of 4 wire bytes held as a native (LE) uint32, i.e. an
// ipv4::Address::m_data word (include/tulips/stack/IPv4.h:55).
TCS_HD uint32_t be_words_of_addr(uint32_t a)
{
  return bswap16(a & 0xffff) + bswap16(a >> 16);
}

// a2's pseudo-header seed (src/stack/tcpv4/Processor.cpp:346-351):
// (len + 6) in uint16 arithmetic, then + src words + dst words.
TCS_HD uint32_t tcp_seed(uint32_t src, uint32_t dst, uint32_t len)
{
  uint32_t s = ((len + 6u) & 0xffffu) + be_words_of_addr(src) +
               be_words_of_addr(dst);
  return fold32(s);
}

// Post-processing of a2/a5/a6: `sum == 0 ? 0xffff : htons(sum)`.
TCS_HD uint32_t inet_post(uint32_t r)
{
  return r == 0 ? 0xffffu : bswap16(r);
}

// Finish one segment: `le_partial` is any partial (<= 2^32-1) congruent to the
// little-endian dword sum of the segment's bytes taken at their absolute
// addresses; `start_odd` says whether the first byte sits at an odd address.
TCS_HD uint32_t finish(uint32_t le_partial, bool start_odd, uint32_t mode,
                       uint32_t seed, uint32_t src, uint32_t dst, uint32_t len)
{
  uint32_t r = fold32(le_partial);
  if (!start_odd) {
    r = bswap16(r);
  }
  const uint32_t m = mode & MODE_MASK;
  if (m == MODE_TCP) {
    seed = tcp_seed(src, dst, len);
  }
  r = add_seed(r, seed);
  if (m != MODE_RAW) {
    r = inet_post(r);
  }
  if (mode & FLAG_COMPLEMENT) {
    r = ~r & 0xffffu;
  }
  return r;
}

#if defined(__HIPCC__)
// Workgroups are dealt round-robin over the 8 XCDs (blocks b and b + 8 share
// one; MI355X_MICROARCH.md, "Workgroup dispatch, XCD placement"), each with
// its own L2. Consecutive blocks take consecutive segments, and segments
// that meet inside a 128-byte line both fetch it. Runs of C consecutive
// logical blocks are therefore kept on one XCD, while the runs themselves
// stay dealt over the 8 XCDs (so the chip still streams one address window
// at a time): hardware block b = 8g + x maps to logical block
// (g / C) * 8C + x * C + g % C. Blocks of a last, incomplete group of 8C map
// to themselves. A bijection on [0, nb): results never depend on placement.
template<uint32_t C>
__device__ __forceinline__ uint32_t xcd_block_c(uint32_t b, uint32_t nb)
{
  const uint32_t full = (nb / (8u * C)) * (8u * C);
  if (C <= 1 || b >= full) {
    return b;
  }
  const uint32_t x = b & 7u, g = b >> 3;
  return (g / C) * (8u * C) + x * C + g % C;
}

__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb)
{
  return xcd_block_c<8>(b, nb);
}

// Inclusive u32 add-scan over the 64 lanes of a wave: DPP row shifts inside
// each row of 16 lanes, then the row totals from lanes 15/31/47 (readlane).
// No LDS crossbar (a __shfl_up scan is six dependent ds_bpermute_b32).
__device__ __forceinline__ uint32_t wave_inclusive_sum(uint32_t x)
{
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x111, 0xf, 0xf, false));
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x112, 0xf, 0xf, false));
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x114, 0xf, 0xf, false));
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x118, 0xf, 0xf, false));
  const int lane = threadIdx.x & 63;
  const uint32_t r0 = __builtin_amdgcn_readlane(x, 15);
  const uint32_t r1 = __builtin_amdgcn_readlane(x, 31);
  const uint32_t r2 = __builtin_amdgcn_readlane(x, 47);
  x += lane >= 16 ? r0 : 0u;
  x += lane >= 32 ? r1 : 0u;
  x += lane >= 48 ? r2 : 0u;
  return x;
}

// Sum of x over each aligned G-lane subgroup of the wave (G = 16, 32 or 64),
// returned to every lane of it, without the LDS crossbar. Four DPP row
// rotations (row_ror 8, 4, 2, 1) fold each 16-lane row in VALU; wider
// subgroups add the row totals read with readlane. A __shfl_xor butterfly
// compiles to ds_bpermute_b32, one dependent LDS round trip per step (five
// at G = 32), and that chain sits between a subgroup's last load and its
// result store. Every lane of a subgroup must be active (or none).
template<int G>
__device__ __forceinline__ uint32_t subgroup_total(uint32_t x)
{
  static_assert(G == 16 || G == 32 || G == 64, "rows of 16 lanes");
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x128, 0xf, 0xf, false));
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x124, 0xf, 0xf, false));
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x122, 0xf, 0xf, false));
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x121, 0xf, 0xf, false));
  if constexpr (G == 16) {
    return x;
  } else {
    const uint32_t r0 = __builtin_amdgcn_readlane(x, 0), r1 = __builtin_amdgcn_readlane(x, 16);
    const uint32_t r2 = __builtin_amdgcn_readlane(x, 32), r3 = __builtin_amdgcn_readlane(x, 48);
    if constexpr (G == 32) {
      return (threadIdx.x & 32u) ? r2 + r3 : r0 + r1;
    } else {
      return (r0 + r1) + (r2 + r3);
    }
  }
}
#endif

}
