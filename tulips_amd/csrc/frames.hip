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

#include "../../include/tulips_csum.h"
#include "csum_common.h"
#include "csum_launch.h"
#include "frame_common.h"

namespace tulips_amd {
namespace {

using namespace frame;

constexpr int VG = 32; // validate: >= 24 header bytes, one per lane
constexpr int VU = 4;  // 128 chunks = a 1514 B frame in one batch per lane

__global__ __launch_bounds__(256) void
frame_kernel(const uint8_t* base, const uint64_t* __restrict__ offs,
             const uint16_t* __restrict__ lens, uint32_t n,
             uint8_t* __restrict__ flags, uint32_t* __restrict__ counters)
{
  const int lane64 = threadIdx.x & 63;
  const int lane = lane64 & (VG - 1);
  const int sub0 = lane64 - lane; // first lane of this subgroup
  const uint32_t per_block = blockDim.x / VG;
  const uint32_t nsub = gridDim.x * per_block;
  for (uint32_t f = blockIdx.x * per_block + threadIdx.x / VG; f < n; f += nsub) {
    const uintptr_t fa = reinterpret_cast<uintptr_t>(base) + offs[f];
    const Header h = gather_header<24>(fa, lens[f], lane, sub0);
    const bool do_l4 = h.tcp && !h.trunc;
    // IPv4 header [14, 34) and TCP segment [34, 34 + tcplen)
    const uint32_t ip_part =
      sub_sum<VG>(fold64(lane_sum<VG, 1, false>(fa + 14, h.ipv4 ? 20u : 0u, lane)));
    const uint32_t l4_part =
      sub_sum<VG>(fold64(lane_sum<VG, VU, true>(fa + 34, do_l4 ? h.tcplen : 0u, lane)));
    if (lane == 0) {
      const bool ip_ok =
        h.ipv4 && finish(ip_part, ((fa + 14) & 1) != 0, MODE_INET, 0, 0, 0, 20) == 0xffffu;
      const bool l4_ok =
        do_l4 && finish(l4_part, ((fa + 34) & 1) != 0, MODE_TCP, 0, h.src, h.dst,
                        h.tcplen) == 0xffffu;
      if (flags) {
        flags[f] = uint8_t(frame_flags(h, ip_ok, l4_ok));
      }
      if (counters) {
        if (h.ipv4) {
          atomicAdd(counters + 0, 1u);
          if (!ip_ok) {
            atomicAdd(counters + 1, 1u);
          }
        }
        if (h.tcp) {
          atomicAdd(counters + 2, 1u);
          if (!l4_ok) {
            atomicAdd(counters + 3, 1u);
          }
        }
      }
    }
  }
}

// Checksum generation in place (the send side: ipv4/Producer.cpp:79-82
// `ipchksum = ~checksum(header)`, tcpv4/Send.cpp:441-449 `chksum = ~csum`),
// one wave per frame. Each field's current bytes are taken out of the sum
// arithmetically (field_contrib) so the frame is read once and written 4 B.
constexpr int GG = 64; // header window 12..51 covers both checksum fields
constexpr int GU = 2;

__global__ __launch_bounds__(256) void
generate_kernel(uint8_t* base, const uint64_t* __restrict__ offs,
                const uint16_t* __restrict__ lens, uint32_t n,
                uint8_t* __restrict__ flags)
{
  const int lane = threadIdx.x & 63;
  const uint32_t per_block = blockDim.x / GG;
  const uint32_t nsub = gridDim.x * per_block;
  for (uint32_t f = blockIdx.x * per_block + threadIdx.x / GG; f < n; f += nsub) {
    const uintptr_t fa = reinterpret_cast<uintptr_t>(base) + offs[f];
    const uint32_t flen = lens[f];
    const Header h = gather_header<40>(fa, flen, lane, 0);
    // the TCP checksum field (segment bytes 16..17) must lie in the frame
    const bool do_l4 = h.tcp && !h.trunc && h.tcplen >= 18u;
    const uint32_t ip_part =
      sub_sum<GG>(fold64(lane_sum<GG, 1, false>(fa + 14, h.ipv4 ? 20u : 0u, lane)));
    const uint32_t l4_part =
      sub_sum<GG>(fold64(lane_sum<GG, GU, false>(fa + 34, do_l4 ? h.tcplen : 0u, lane)));
    if (lane == 0) {
      if (h.ipv4) {
        const uint32_t p =
          fold32(ip_part) + (0xffffu - field_contrib(fa + 24, h.ipck0, h.ipck1));
        const uint32_t r = finish(p, ((fa + 14) & 1) != 0, MODE_INET, 0, 0, 0, 20);
        store_field(fa + 24, ~r & 0xffffu);
      }
      if (do_l4) {
        const uint32_t p =
          fold32(l4_part) + (0xffffu - field_contrib(fa + 50, h.tcpck0, h.tcpck1));
        const uint32_t r =
          finish(p, ((fa + 34) & 1) != 0, MODE_TCP, 0, h.src, h.dst, h.tcplen);
        store_field(fa + 50, ~r & 0xffffu);
      }
      if (flags) {
        flags[f] = uint8_t(frame_flags(h, h.ipv4, do_l4));
      }
    }
  }
}

uint32_t
grid_for(uint32_t n, uint32_t per_block)
{
  uint64_t blocks = (uint64_t(n) + per_block - 1) / per_block;
  return uint32_t(blocks > 65535 ? 65535 : blocks);
}

} // namespace

hipError_t
launch_frames(const uint8_t* base, const uint64_t* offs, const uint16_t* lens,
              uint32_t n, uint8_t* flags, uint32_t* counters, hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL(frame_kernel, dim3(grid_for(n, 256 / VG)), dim3(256), 0,
                     stream, base, offs, lens, n, flags, counters);
  return hipGetLastError();
}

hipError_t
launch_generate(uint8_t* base, const uint64_t* offs, const uint16_t* lens,
                uint32_t n, uint8_t* flags, hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL(generate_kernel, dim3(grid_for(n, 256 / GG)), dim3(256), 0,
                     stream, base, offs, lens, n, flags);
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
