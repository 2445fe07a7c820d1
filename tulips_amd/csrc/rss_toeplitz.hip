// rss_toeplitz.hip — batched Toeplitz RSS hash.
//
// Reference: tulips::stack::utils::toeplitz, src/stack/Utils.cpp:86-133
// (used by the ENA RSS redirection table, src/transport/ena/
// RedirectionTable.cpp:74-98; KATs tests/stack/utils.cpp:37,54).
//
// The hash is linear over GF(2): with the 96-bit tuple
//   saddr bytes | daddr bytes | htons(sport) | htons(dport)
// consumed MSB first, bit k (k = 0..95) XORs the 32-bit key window the
// reference holds at step k into the result. The windows depend only on the
// key, so the host derives them once per call by running the reference's
// shift register exactly — including its wrap-around, which reads the
// already-shifted first byte (Utils.cpp:123-125) and matters for keys shorter
// than 16 bytes — and the GPU only evaluates
//   h = init ^ XOR_b T_b[tuple byte b],   T_b[v] = XOR of the windows of v's bits
// with the 12 x 256 tables built in LDS by each workgroup (12 KiB).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/tulips_csum.h"

namespace tulips::stack::ipv4 {
class Address; // the reference's 4-byte packed address (IPv4.h:13-62)
}

namespace tulips_amd {
namespace {

constexpr int RSS_BITS = 96;
constexpr size_t RSS_MAX_KEY = 4096;

struct RssWindows
{
  uint32_t w[RSS_BITS];
};

// The reference's key shift register, step by step (Utils.cpp:96-126).
bool
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

uint32_t
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

// One workgroup: build T[12][256] in LDS, then hash a grid-stride share of
// the tuples (structure of arrays, coalesced).
__global__ __launch_bounds__(256) void
rss_kernel(RssWindows win, const uint32_t* __restrict__ saddr,
           const uint32_t* __restrict__ daddr,
           const uint16_t* __restrict__ sport,
           const uint16_t* __restrict__ dport, uint32_t* __restrict__ out,
           uint32_t n, uint32_t init)
{
  __shared__ uint32_t T[12][256];
  for (int e = threadIdx.x; e < 12 * 256; e += blockDim.x) {
    const int b = e >> 8, v = e & 255;
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (v & (0x80 >> j)) {
        x ^= win.w[8 * b + j];
      }
    }
    T[b][v] = x;
  }
  __syncthreads();
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += gridDim.x * blockDim.x) {
    const uint32_t s = saddr[i], d = daddr[i];
    const uint32_t sp = sport[i], dp = dport[i];
    uint32_t h = init;
    h ^= T[0][s & 0xff] ^ T[1][(s >> 8) & 0xff] ^ T[2][(s >> 16) & 0xff] ^
         T[3][s >> 24];
    h ^= T[4][d & 0xff] ^ T[5][(d >> 8) & 0xff] ^ T[6][(d >> 16) & 0xff] ^
         T[7][d >> 24];
    h ^= T[8][(sp >> 8) & 0xff] ^ T[9][sp & 0xff] ^ T[10][(dp >> 8) & 0xff] ^
         T[11][dp & 0xff];
    out[i] = h;
  }
}

} // namespace
} // namespace tulips_amd

using namespace tulips_amd;

// The reference's C++ symbol (include/tulips/stack/Utils.h:25-28):
// _ZN6tulips5stack5utils8toeplitzERKNS0_4ipv47AddressES5_ttmPKhj. An Address
// is its 4 wire bytes (packed), so it is read through a byte pointer.
namespace tulips::stack::utils {
__attribute__((visibility("default"))) uint32_t
toeplitz(stack::ipv4::Address const& saddr, stack::ipv4::Address const& daddr,
         const uint16_t sport, const uint16_t dport, const size_t key_len,
         const uint8_t* const key, const uint32_t init)
{
  RssWindows w;
  if (!rss_windows(key, key_len, w)) {
    return init; // the reference reads out of bounds for len < 4
  }
  uint32_t s, d;
  memcpy(&s, reinterpret_cast<const uint8_t*>(&saddr), 4);
  memcpy(&d, reinterpret_cast<const uint8_t*>(&daddr), 4);
  return rss_host(w, s, d, sport, dport, init);
}
}

extern "C" {

int
tulips_rss_toeplitz_host(uint32_t saddr, uint32_t daddr, uint16_t sport,
                         uint16_t dport, const uint8_t* key, size_t key_len,
                         uint32_t init, uint32_t* out)
{
  RssWindows w;
  if (!out || !rss_windows(key, key_len, w)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  *out = rss_host(w, saddr, daddr, sport, dport, init);
  return TULIPS_STATUS_OK;
}

int
tulips_rss_toeplitz_batch(const uint32_t* saddr, const uint32_t* daddr,
                          const uint16_t* sport, const uint16_t* dport,
                          uint32_t n, const uint8_t* key, size_t key_len,
                          uint32_t init, uint32_t* out, void* stream)
{
  if (n == 0) {
    return TULIPS_STATUS_OK;
  }
  RssWindows w;
  if (!saddr || !daddr || !sport || !dport || !out ||
      !rss_windows(key, key_len, w)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  uint64_t blocks = (uint64_t(n) + 255) / 256;
  if (blocks > 2048) {
    blocks = 2048; // 8 per CU; each builds its LDS tables once
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL(rss_kernel, dim3(uint32_t(blocks)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), w, saddr, daddr, sport,
                     dport, out, n, init);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? TULIPS_STATUS_OK : TULIPS_STATUS_HARDWARE_ERROR;
}

} // extern "C"
