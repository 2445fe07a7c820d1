// rss_common.h — the Toeplitz RSS hash (src/stack/Utils.cpp:86-133) as the
// GPU evaluates it: key windows derived on the host by running the
// reference's shift register, per-workgroup LDS lookup tables, and the
// per-tuple XOR of table entries. Shared by the tuple batch
// (rss_toeplitz.hip) and the flow router (rss_route.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

namespace tulips_amd {

constexpr int RSS_BITS = 96;
constexpr size_t RSS_MAX_KEY = 4096;

struct RssWindows
{
  uint32_t w[RSS_BITS];
};

// The reference's key shift register, step by step (Utils.cpp:96-126).
inline bool
rss_windows(const uint8_t* key, size_t len, RssWindows& out)
{
  if (!key || len < 4 || len > RSS_MAX_KEY) {
    return false;
  }
  uint8_t tmp[RSS_MAX_KEY];
  memcpy(tmp, key, len);
  for (int k = 0; k < RSS_BITS; ++k) {
    out.w[k] = (uint32_t(tmp[0]) << 24) | (uint32_t(tmp[1]) << 16) |
               (uint32_t(tmp[2]) << 8) | uint32_t(tmp[3]);
    for (size_t i = 0; i < len; ++i) {
      tmp[i] = uint8_t(((tmp[i] << 1) & 0xff) | ((tmp[(i + 1) % len] & 0x80) >> 7));
    }
  }
  return true;
}

inline void
tuple_bytes(uint32_t saddr, uint32_t daddr, uint16_t sport, uint16_t dport,
            uint8_t t[12])
{
  memcpy(t, &saddr, 4);
  memcpy(t + 4, &daddr, 4);
  t[8] = uint8_t(sport >> 8);
  t[9] = uint8_t(sport);
  t[10] = uint8_t(dport >> 8);
  t[11] = uint8_t(dport);
}

inline uint32_t
rss_host(const RssWindows& w, uint32_t saddr, uint32_t daddr, uint16_t sport,
         uint16_t dport, uint32_t init)
{
  uint8_t t[12];
  tuple_bytes(saddr, daddr, sport, dport, t);
  uint32_t h = init;
  for (int k = 0; k < RSS_BITS; ++k) {
    if (t[k >> 3] & (0x80u >> (k & 7))) {
      h ^= w.w[k];
    }
  }
  return h;
}

// One workgroup builds its lookup tables in LDS, then hashes a grid-stride
// share of the tuples (structure of arrays). The hash is
//   h = init ^ XOR over tuple bytes b of T_b[byte b]
// and a lookup costs LDS cycles: a 256-entry table read at 32 random
// addresses per lane group conflicts ~3.5-way (about 7 cycles per wave
// instruction instead of 2), while a 16-entry table spans 16 banks and never
// conflicts but needs two lookups per byte and twice the VALU to form the
// indices. The 4 port bytes use byte tables, the 8 address bytes nibble
// tables: LDS 4 x ~7 + 16 x 2 = 60 cycles and ~36 VALU per 64 tuples, where
// 12 byte lookups cost ~84 LDS cycles (the kernel was LDS-bound).
//   TB[k][v]: byte tables for tuple bytes 8 + k (k = 0..3), v = 0..255
//   TN[p][v]: nibble tables for tuple bits 4p..4p+3 (p = 0..15, MSB first)
struct RssTables
{
  uint32_t TB[4][256];
  uint32_t TN[16][16];
};

__device__ __forceinline__ void
build_tables(const RssWindows& win, RssTables& t)
{
  for (int e = threadIdx.x; e < 4 * 256; e += blockDim.x) {
    const int k = e >> 8, v = e & 255;
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x ^= (v & (0x80 >> j)) ? win.w[8 * (8 + k) + j] : 0u;
    }
    t.TB[k][v] = x;
  }
  for (int e = threadIdx.x; e < 16 * 16; e += blockDim.x) {
    const int p = e >> 4, v = e & 15;
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x ^= (v & (0x8 >> j)) ? win.w[4 * p + j] : 0u;
    }
    t.TN[p][v] = x;
  }
}

// Tuple bytes 4a..4a+3 are the little-endian bytes of word x (the reference
// copies the address words' memory, Utils.cpp:101-104): nibble j of x (bits
// 4j..4j+3) is the low (j even) or high (j odd) nibble of byte 4a + j/2.
__device__ __forceinline__ uint32_t
hash_word(const RssTables& t, uint32_t x, int a)
{
  uint32_t h = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int p = 2 * (4 * a + (j >> 1)) + ((j & 1) ? 0 : 1);
    h ^= t.TN[p][(x >> (4 * j)) & 15u];
  }
  return h;
}

__device__ __forceinline__ uint32_t
rss_one(const RssTables& t, uint32_t s, uint32_t d, uint32_t sp, uint32_t dp, uint32_t init)
{
  return init ^ hash_word(t, s, 0) ^ hash_word(t, d, 1) ^ t.TB[0][(sp >> 8) & 0xffu] ^
         t.TB[1][sp & 0xffu] ^ t.TB[2][(dp >> 8) & 0xffu] ^ t.TB[3][dp & 0xffu];
}

} // namespace tulips_amd
