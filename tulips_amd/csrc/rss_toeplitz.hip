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
// with lookup tables built in LDS by each workgroup (rss_kernel).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/tulips_csum.h"
#include "rss_common.h"

namespace tulips::stack::ipv4 {
class Address; // the reference's 4-byte packed address (IPv4.h:13-62)
}

namespace tulips_amd {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// VEC: 4 tuples per thread (16-B address / result vectors, 8-B port
// vectors; the arrays are 16-B / 8-B aligned, n / 4 groups), then the n % 4
// tail one tuple per thread. Otherwise one tuple per thread throughout.
template<bool VEC>
__global__ __launch_bounds__(256) void
rss_kernel(RssWindows win, const uint32_t* __restrict__ saddr,
           const uint32_t* __restrict__ daddr,
           const uint16_t* __restrict__ sport,
           const uint16_t* __restrict__ dport, uint32_t* __restrict__ out,
           uint32_t n, uint32_t init)
{
  __shared__ RssTables t;
  build_tables(win, t);
  __syncthreads();
  const uint32_t stride = gridDim.x * blockDim.x;
  uint32_t i0 = 0;
  if constexpr (VEC) {
    const uint32_t n4 = n / 4;
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < n4; g += stride) {
      const u32x4 s = reinterpret_cast<const u32x4*>(saddr)[g];
      const u32x4 d = reinterpret_cast<const u32x4*>(daddr)[g];
      const u32x2 sp = reinterpret_cast<const u32x2*>(sport)[g];
      const u32x2 dp = reinterpret_cast<const u32x2*>(dport)[g];
      u32x4 h;
      h.x = rss_one(t, s.x, d.x, sp.x & 0xffffu, dp.x & 0xffffu, init);
      h.y = rss_one(t, s.y, d.y, sp.x >> 16, dp.x >> 16, init);
      h.z = rss_one(t, s.z, d.z, sp.y & 0xffffu, dp.y & 0xffffu, init);
      h.w = rss_one(t, s.w, d.w, sp.y >> 16, dp.y >> 16, init);
      reinterpret_cast<u32x4*>(out)[g] = h;
    }
    i0 = 4 * n4;
  }
  for (uint32_t i = i0 + blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    out[i] = rss_one(t, saddr[i], daddr[i], sport[i], dport[i], init);
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
  const bool vec = ((reinterpret_cast<uintptr_t>(saddr) | reinterpret_cast<uintptr_t>(daddr) |
                     reinterpret_cast<uintptr_t>(out)) & 15) == 0 &&
                   ((reinterpret_cast<uintptr_t>(sport) | reinterpret_cast<uintptr_t>(dport)) &
                    7) == 0;
  const uint64_t per_thread = vec ? 4 : 1;
  uint64_t blocks = (uint64_t(n) + 256 * per_thread - 1) / (256 * per_thread);
  if (blocks > 2048) {
    blocks = 2048; // 8 per CU; each builds its LDS tables once
  }
  (void)hipGetLastError();
  if (vec) {
    hipLaunchKernelGGL(rss_kernel<true>, dim3(uint32_t(blocks)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), w, saddr, daddr, sport, dport, out,
                       n, init);
  } else {
    hipLaunchKernelGGL(rss_kernel<false>, dim3(uint32_t(blocks)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), w, saddr, daddr, sport, dport, out,
                       n, init);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? TULIPS_STATUS_OK : TULIPS_STATUS_HARDWARE_ERROR;
}

} // extern "C"
