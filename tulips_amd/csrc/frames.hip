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
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tulips_csum.h"
#include "csum_common.h"
#include "csum_launch.h"

namespace tulips_amd {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4* gchunk_ptr;
typedef const __attribute__((address_space(1))) uint8_t* gbyte_ptr;

__device__ __forceinline__ uint64_t
hsum(u32x4 v)
{
  return (uint64_t(v.x) + uint64_t(v.y)) + (uint64_t(v.z) + uint64_t(v.w));
}

__device__ __forceinline__ uint32_t
byte_mask(int lo, int hi, int b)
{
  int ml = min(max(lo - b, 0), 4);
  int mh = min(max(hi - b, 0), 4);
  return uint32_t((1ull << (8 * mh)) - 1ull) & ~uint32_t((1ull << (8 * ml)) - 1ull);
}

__device__ __forceinline__ uint64_t
masked_hsum(u32x4 v, int lo, int hi)
{
  return (uint64_t(v.x & byte_mask(lo, hi, 0)) +
          uint64_t(v.y & byte_mask(lo, hi, 4))) +
         (uint64_t(v.z & byte_mask(lo, hi, 8)) +
          uint64_t(v.w & byte_mask(lo, hi, 12)));
}

// This lane's LE dword sum of [sa, sa+len) over absolute 16-byte chunks
// (G lanes, U unconditional clamped loads per lane per batch).
template<int G, int U, bool NT>
__device__ __forceinline__ uint64_t
lane_sum(uintptr_t sa, uint32_t len, int lane)
{
  if (len == 0) {
    return 0;
  }
  const uintptr_t a0 = sa & ~uintptr_t(15);
  const int nch = int((sa + len - a0 + 15) >> 4);
  const int last = nch - 1;
  const int head = int(sa - a0);
  const int tail = int(sa + len - a0) - 16 * last;
  const gchunk_ptr p = reinterpret_cast<gchunk_ptr>(a0);
  uint64_t acc = 0;
  for (int c = lane; c < nch; c += U * G) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int cc = min(c + u * G, last);
      v[u] = NT ? __builtin_nontemporal_load(p + cc) : p[cc];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int cc = c + u * G;
      acc += cc <= last ? hsum(v[u]) : 0;
      if (u == 0 && cc == 0 && head != 0) {
        acc -= masked_hsum(v[u], 0, head);
      }
      if (cc == last && tail != 16) {
        acc -= masked_hsum(v[u], tail, 16);
      }
    }
  }
  return acc;
}

template<int G>
__device__ __forceinline__ uint32_t
sub_sum(uint32_t x)
{
#pragma unroll
  for (int m = G / 2; m >= 1; m >>= 1) {
    x += __shfl_xor(x, m, 64);
  }
  return x;
}

constexpr int G = 32; // >= 24 header bytes, one per lane
constexpr int U = 4;  // 128 chunks = a 1514 B frame in one batch per lane

__global__ __launch_bounds__(256) void
frame_kernel(const uint8_t* base, const uint64_t* __restrict__ offs,
             const uint16_t* __restrict__ lens, uint32_t n,
             uint8_t* __restrict__ flags, uint32_t* __restrict__ counters)
{
  const int lane64 = threadIdx.x & 63;
  const int lane = lane64 & (G - 1);
  const int sub0 = lane64 - lane; // first lane of this subgroup
  const uint32_t per_block = blockDim.x / G;
  const uint32_t nsub = gridDim.x * per_block;
  for (uint32_t f = blockIdx.x * per_block + threadIdx.x / G; f < n; f += nsub) {
    const uintptr_t fa = reinterpret_cast<uintptr_t>(base) + offs[f];
    const uint32_t flen = lens[f];
    // header bytes 12..35 (only bytes inside the frame are read)
    uint32_t hb = 0;
    if (lane < 24 && uint32_t(12 + lane) < flen) {
      hb = *reinterpret_cast<gbyte_ptr>(fa + 12 + lane);
    }
    auto byte = [&](int off) { return __shfl(hb, sub0 + off - 12, 64); };
    const uint32_t type = (byte(12) << 8) | byte(13);
    const uint32_t vhl = byte(14);
    const uint32_t total = (byte(16) << 8) | byte(17);
    const uint32_t off0 = byte(20), off1 = byte(21);
    const uint32_t proto = byte(23);
    const uint32_t src = byte(26) | (byte(27) << 8) | (byte(28) << 16) | (byte(29) << 24);
    const uint32_t dst = byte(30) | (byte(31) << 8) | (byte(32) << 16) | (byte(33) << 24);
    const bool eth_ip = flen >= 14 && type == 0x0800u;
    const bool runt = eth_ip && flen < 34;
    const bool ipv4 = eth_ip && !runt && vhl == 0x45u;
    const bool tcp = ipv4 && (off0 & 0x3fu) == 0 && off1 == 0 && proto == 6u;
    const uint32_t tcplen = (total - 20u) & 0xffffu;
    const bool trunc = tcp && (total < 20u || 34u + tcplen > flen);
    const bool do_l4 = tcp && !trunc;
    // IPv4 header [14, 34) and TCP segment [34, 34 + tcplen)
    const uint32_t ip_part =
      sub_sum<G>(fold64(lane_sum<G, 1, false>(fa + 14, ipv4 ? 20u : 0u, lane)));
    const uint32_t l4_part =
      sub_sum<G>(fold64(lane_sum<G, U, true>(fa + 34, do_l4 ? tcplen : 0u, lane)));
    if (lane == 0) {
      const bool ip_ok =
        ipv4 && finish(ip_part, ((fa + 14) & 1) != 0, MODE_INET, 0, 0, 0, 20) == 0xffffu;
      const bool l4_ok =
        do_l4 && finish(l4_part, ((fa + 34) & 1) != 0, MODE_TCP, 0, src, dst,
                        tcplen) == 0xffffu;
      uint32_t fl = 0;
      if (runt) {
        fl = TULIPS_FRAME_TRUNCATED;
      } else if (ipv4) {
        fl = TULIPS_FRAME_IPV4 | (ip_ok ? TULIPS_FRAME_IP_CSUM_OK : 0u) |
             (tcp ? TULIPS_FRAME_TCP : 0u) | (trunc ? TULIPS_FRAME_TRUNCATED : 0u) |
             (l4_ok ? TULIPS_FRAME_L4_CSUM_OK : 0u);
      }
      if (flags) {
        flags[f] = uint8_t(fl);
      }
      if (counters) {
        if (ipv4) {
          atomicAdd(counters + 0, 1u);
          if (!ip_ok) {
            atomicAdd(counters + 1, 1u);
          }
        }
        if (tcp) {
          atomicAdd(counters + 2, 1u);
          if (!l4_ok) {
            atomicAdd(counters + 3, 1u);
          }
        }
      }
    }
  }
}

} // namespace

hipError_t
launch_frames(const uint8_t* base, const uint64_t* offs, const uint16_t* lens,
              uint32_t n, uint8_t* flags, uint32_t* counters, hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  const uint64_t per_block = 256 / G;
  uint64_t blocks = (uint64_t(n) + per_block - 1) / per_block;
  if (blocks > 65535) {
    blocks = 65535;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL(frame_kernel, dim3(uint32_t(blocks)), dim3(256), 0, stream,
                     base, offs, lens, n, flags, counters);
  return hipGetLastError();
}

} // namespace tulips_amd

extern "C" int
tulips_csum_validate_frames(const uint8_t* base, const uint64_t* offsets,
                            const uint16_t* lengths, uint32_t n, uint8_t* flags,
                            uint32_t* counters, void* stream)
{
  if (n == 0) {
    return TULIPS_STATUS_OK;
  }
  if (!base || !offsets || !lengths || (!flags && !counters)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (counters) {
    const hipError_t e = hipMemsetAsync(counters, 0, 4 * sizeof(uint32_t), st);
    if (e != hipSuccess) {
      return TULIPS_STATUS_HARDWARE_ERROR;
    }
  }
  const hipError_t e =
    tulips_amd::launch_frames(base, offsets, lengths, n, flags, counters, st);
  return e == hipSuccess ? TULIPS_STATUS_OK : TULIPS_STATUS_HARDWARE_ERROR;
}
