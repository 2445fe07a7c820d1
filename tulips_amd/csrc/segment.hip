// segment.hip — send-side segmentation with checksum generation, the job the
// reference hands to the NIC as TCP segmentation offload:
// src/transport/ofed/Device.cpp:688-772 posts a super-frame whose header
// length comes from stack::utils::headerLength (src/stack/Utils.cpp:67-84,
// Ethernet 14 + IPv4 20 + TCP data offset * 4) with IBV_WR_TSO and an MSS,
// and the NIC emits MSS-sized frames with their checksums filled in
// (IBV_SEND_IP_CSUM).
//
// Per super-frame (option-less IPv4, unfragmented TCP, complete header and
// segment), payload P = ntohs(len) - 20 - doff*4 is cut into ceil(P / mss)
// segments. Segment k gets the super-frame's header with
//   IPv4 total length = 20 + doff*4 + slice,  IPv4 id = id + k,
//   TCP seq = seq + k*mss,  FIN/PSH only on the last segment, CWR only on
//   the first,
// and both checksums generated as ipv4/Producer.cpp:79-82 and
// tcpv4/Send.cpp:441-449 write them. Other frames (and super-frames whose
// payload fits one segment) are copied whole with checksum generation by the
// rules of tulips_csum_generate_frames. (The reference has no software TSO:
// these fixups are the standard NIC LSO semantics, not a reference
// restatement; the checksum generation is.)
//
// Layout: segment j of the whole batch goes to out + j*stride (16-aligned
// slots); segments of frame i are j = first[i] .. first[i+1]-1, where
// `first` is an exclusive prefix sum of the per-frame segment counts computed
// on the device (first[n] = total). One wave builds one super-frame's
// segments: each lane assembles aligned 16-byte destination chunks from
// funnel-shifted source chunks (v_alignbyte), patches the header fields in
// registers, sums them for both checksums, and stores; the two chunks that
// hold checksum fields are stored after the wave reduction. Reads each source
// byte from HBM once and writes each destination byte once.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "../../include/tulips_csum.h"
#include "csum_common.h"
#include "frame_common.h"

namespace tulips_amd {
namespace {

using namespace frame;

typedef __attribute__((address_space(1))) u32x4* gchunk_wptr;

constexpr uint32_t TCP_FIN = 0x01, TCP_PSH = 0x08, TCP_CWR = 0x80;
constexpr uint32_t MAX_FRAMES = 1u << 24; // 65536 count blocks of 256
constexpr int CB = 256;                   // count/scan block

struct SegInfo
{
  bool seg_ok;
  uint32_t hlen, payload, nseg;
};

__device__ __forceinline__ SegInfo
seg_info(const Header& h, uint32_t mss)
{
  SegInfo s;
  s.seg_ok = h.tcp && !h.trunc && h.doff >= 5 && 20u + 4u * h.doff <= h.total;
  s.hlen = 34u + 4u * h.doff;
  s.payload = s.seg_ok ? h.total - 20u - 4u * h.doff : 0u;
  s.nseg = (s.seg_ok && s.payload > mss) ? (s.payload + mss - 1) / mss : 1u;
  return s;
}

// ---- exclusive scan of segment counts -------------------------------------

template<int NW>
__device__ __forceinline__ uint32_t
block_inclusive_scan(uint32_t x, uint32_t* lds, uint32_t& total)
{
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(x, d, 64);
    if (lane >= d) {
      x += t;
    }
  }
  if (lane == 63) {
    lds[w] = x;
  }
  __syncthreads();
  uint32_t before = 0;
  total = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const uint32_t v = lds[i];
    before += i < w ? v : 0u;
    total += v;
  }
  __syncthreads();
  return x + before;
}

__global__ __launch_bounds__(CB) void
seg_count_kernel(const uint8_t* base, const uint64_t* __restrict__ offs,
                 const uint16_t* __restrict__ lens, uint32_t n, uint32_t mss,
                 uint32_t* __restrict__ first, uint32_t* __restrict__ ws)
{
  __shared__ uint32_t lds[CB / 64];
  const uint32_t i = blockIdx.x * CB + threadIdx.x;
  uint32_t c = 0;
  if (i < n) {
    const uintptr_t fa = reinterpret_cast<uintptr_t>(base) + offs[i];
    c = seg_info(load_header(fa, lens[i]), mss).nseg;
  }
  uint32_t total;
  const uint32_t inc = block_inclusive_scan<CB / 64>(c, lds, total);
  if (i < n) {
    first[i] = inc - c;
  }
  if (threadIdx.x == 0) {
    ws[blockIdx.x] = total;
  }
}

__global__ __launch_bounds__(1024) void
seg_scan_blocks_kernel(uint32_t* ws, uint32_t nb, uint32_t* total_out)
{
  __shared__ uint32_t lds[16];
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
    const uint32_t i = b0 + threadIdx.x;
    const uint32_t v = i < nb ? ws[i] : 0u;
    uint32_t tile;
    const uint32_t inc = block_inclusive_scan<16>(v, lds, tile);
    if (i < nb) {
      ws[i] = carry + inc - v;
    }
    carry += tile;
  }
  if (threadIdx.x == 0) {
    *total_out = carry;
  }
}

__global__ __launch_bounds__(CB) void
seg_add_kernel(uint32_t n, uint32_t* __restrict__ first, const uint32_t* __restrict__ ws)
{
  const uint32_t i = blockIdx.x * CB + threadIdx.x;
  if (i < n) {
    first[i] += ws[blockIdx.x];
  }
}

// ---- segmentation ----------------------------------------------------------

__device__ __forceinline__ u32x4
load_chunk(uintptr_t q)
{
  return *reinterpret_cast<gchunk_ptr>(q);
}

// Bytes x .. x+15 from two aligned chunk loads clamped to [lo, hi] (bytes
// outside the frame come back unspecified; callers never use them).
__device__ __forceinline__ u32x4
window(uintptr_t x, uintptr_t lo, uintptr_t hi)
{
  const uintptr_t q = x & ~uintptr_t(15);
  const uintptr_t q0 = q < lo ? lo : (q > hi ? hi : q);
  const uintptr_t q1 = q + 16 > hi ? hi : q + 16;
  const u32x4 a = load_chunk(q0), b = load_chunk(q1);
  const uint32_t m = uint32_t(x & 15), r = m & 3;
  uint32_t d0, d1, d2, d3, d4;
  switch (m >> 2) {
    case 0: d0 = a.x; d1 = a.y; d2 = a.z; d3 = a.w; d4 = b.x; break;
    case 1: d0 = a.y; d1 = a.z; d2 = a.w; d3 = b.x; d4 = b.y; break;
    case 2: d0 = a.z; d1 = a.w; d2 = b.x; d3 = b.y; d4 = b.z; break;
    default: d0 = a.w; d1 = b.x; d2 = b.y; d3 = b.z; d4 = b.w; break;
  }
  u32x4 v;
  v.x = __builtin_amdgcn_alignbyte(d1, d0, r);
  v.y = __builtin_amdgcn_alignbyte(d2, d1, r);
  v.z = __builtin_amdgcn_alignbyte(d3, d2, r);
  v.w = __builtin_amdgcn_alignbyte(d4, d3, r);
  return v;
}

// Keep bytes [0, k) of a chunk from `a`, the rest from `b`.
__device__ __forceinline__ u32x4
merge_bytes(u32x4 a, u32x4 b, int k)
{
  u32x4 v;
  const uint32_t m0 = byte_mask(0, k, 0), m1 = byte_mask(0, k, 4);
  const uint32_t m2 = byte_mask(0, k, 8), m3 = byte_mask(0, k, 12);
  v.x = (a.x & m0) | (b.x & ~m0);
  v.y = (a.y & m1) | (b.y & ~m1);
  v.z = (a.z & m2) | (b.z & ~m2);
  v.w = (a.w & m3) | (b.w & ~m3);
  return v;
}

__device__ __forceinline__ u32x4
keep_bytes(u32x4 a, int k)
{
  u32x4 v;
  v.x = a.x & byte_mask(0, k, 0);
  v.y = a.y & byte_mask(0, k, 4);
  v.z = a.z & byte_mask(0, k, 8);
  v.w = a.w & byte_mask(0, k, 12);
  return v;
}

__global__ __launch_bounds__(256) void
segment_kernel(const uint8_t* in, const uint64_t* __restrict__ offs,
               const uint16_t* __restrict__ lens, uint32_t n, uint32_t mss,
               const uint32_t* __restrict__ first, uint8_t* out, uint64_t stride,
               uint32_t capacity, uint16_t* __restrict__ out_lens)
{
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x / 64);
  for (uint32_t i = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; i < n; i += nw) {
    const uintptr_t fa = reinterpret_cast<uintptr_t>(in) + offs[i];
    const uint32_t flen = lens[i];
    const Header h = gather_header<40>(fa, flen, lane, 0);
    const SegInfo si = seg_info(h, mss);
    const uint32_t j0 = first[i];
    const uintptr_t lo = fa & ~uintptr_t(15);
    const uintptr_t hi = flen ? (fa + flen - 1) & ~uintptr_t(15) : lo;
    const bool ip_on = h.ipv4;
    const bool l4_on = si.seg_ok || (h.tcp && !h.trunc && h.tcplen >= 18u);
    for (uint32_t k = 0; k < si.nseg; ++k) {
      const uint32_t j = j0 + k;
      if (j >= capacity) {
        break;
      }
      const uint32_t slice = si.seg_ok ? min(mss, si.payload - k * mss) : 0u;
      const uint32_t dlen = si.nseg == 1 ? flen : si.hlen + slice;
      if (dlen > stride) {
        if (lane == 0) {
          out_lens[j] = 0;
        }
        continue;
      }
      const uint32_t total = si.seg_ok ? 20u + 4u * h.doff + slice : h.total;
      const uint32_t tcp_end = si.seg_ok ? 14u + total : 34u + h.tcplen;
      const uint32_t id = (h.id + k) & 0xffffu;
      const uint32_t seq = h.seq + k * mss;
      uint32_t tfl = h.tflags;
      if (k + 1 < si.nseg) {
        tfl &= ~(TCP_FIN | TCP_PSH);
      }
      if (k > 0) {
        tfl &= ~TCP_CWR;
      }
      const uintptr_t shift = uintptr_t(k) * mss;
      const uintptr_t dst = reinterpret_cast<uintptr_t>(out) + uintptr_t(j) * stride;
      const int nchunks = int((dlen + 15) >> 4);
      uint64_t ip_acc = 0, l4_acc = 0;
      u32x4 keep = {0, 0, 0, 0};
      for (int c = lane; c < nchunks; c += 64) {
        const int cb = 16 * c;
        u32x4 v = window(fa + shift + cb, lo, hi);
        if (shift != 0 && uint32_t(cb) < si.hlen) {
          v = merge_bytes(window(fa + cb, lo, hi), v, int(si.hlen) - cb);
        }
        if (uint32_t(cb + 16) > dlen) {
          v = keep_bytes(v, int(dlen) - cb);
        }
        if (c == 1 && ip_on) {
          if (si.seg_ok) {
            v.x = (total >> 8) | ((total & 0xffu) << 8) | ((id >> 8) << 16) |
                  ((id & 0xffu) << 24);
          }
          v.z &= 0xffff0000u; // ipchksum = 0
        }
        if (c == 2 && si.seg_ok) {
          v.y = (v.y & 0xffffu) | (((seq >> 24) & 0xffu) << 16) |
                (((seq >> 16) & 0xffu) << 24);
          v.z = (v.z & 0xffff0000u) | ((seq >> 8) & 0xffu) | ((seq & 0xffu) << 8);
          v.w = (v.w & 0x00ffffffu) | (tfl << 24);
        }
        if (c == 3 && l4_on) {
          v.x &= 0x0000ffffu; // chksum = 0
        }
        if (ip_on && cb < 34) {
          ip_acc += masked_hsum(v, max(14 - cb, 0), min(34 - cb, 16));
        }
        if (l4_on && cb + 16 > 34 && uint32_t(cb) < tcp_end) {
          l4_acc += masked_hsum(v, max(34 - cb, 0), min(int(tcp_end) - cb, 16));
        }
        if (c == 1 || c == 3) {
          keep = v;
        } else {
          *reinterpret_cast<gchunk_wptr>(dst + cb) = v;
        }
      }
      const uint32_t ip = sub_sum<64>(fold64(ip_acc));
      const uint32_t l4 = sub_sum<64>(fold64(l4_acc));
      if (lane == 1 && nchunks > 1) {
        if (ip_on) {
          keep.z |= ~finish(ip, false, MODE_INET, 0, 0, 0, 20) & 0xffffu;
        }
        *reinterpret_cast<gchunk_wptr>(dst + 16) = keep;
      }
      if (lane == 3 && nchunks > 3) {
        if (l4_on) {
          const uint32_t r = finish(l4, false, MODE_TCP, 0, h.src, h.dst, total - 20u);
          keep.x |= (~r & 0xffffu) << 16;
        }
        *reinterpret_cast<gchunk_wptr>(dst + 48) = keep;
      }
      if (lane == 0) {
        out_lens[j] = uint16_t(dlen);
      }
    }
  }
}

// Per-device scan workspace (one uint32 per count block), made on first use.
std::mutex g_ws_mutex;
uint32_t* g_ws[64] = {};

hipError_t
workspace(uint32_t** ws)
{
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) {
    return e;
  }
  if (dev < 0 || dev >= 64) {
    return hipErrorInvalidDevice;
  }
  std::lock_guard<std::mutex> g(g_ws_mutex);
  if (!g_ws[dev]) {
    e = hipMalloc(reinterpret_cast<void**>(&g_ws[dev]),
                  sizeof(uint32_t) * (MAX_FRAMES / CB));
    if (e != hipSuccess) {
      g_ws[dev] = nullptr;
      return e;
    }
  }
  *ws = g_ws[dev];
  return hipSuccess;
}

} // namespace
} // namespace tulips_amd

extern "C" int
tulips_csum_segment_frames(const uint8_t* in_base, const uint64_t* in_offsets,
                           const uint16_t* in_lengths, uint32_t n, uint32_t mss,
                           uint8_t* out_base, uint64_t out_stride,
                           uint32_t out_capacity, uint16_t* out_lengths,
                           uint32_t* out_first, void* stream)
{
  using namespace tulips_amd;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!out_first || mss == 0 || mss > 0xffffu || n > MAX_FRAMES) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (n == 0) {
    return hipMemsetAsync(out_first, 0, sizeof(uint32_t), st) == hipSuccess
             ? TULIPS_STATUS_OK
             : TULIPS_STATUS_HARDWARE_ERROR;
  }
  if (!in_base || !in_offsets || !in_lengths ||
      (out_capacity && (!out_base || !out_lengths ||
                        (reinterpret_cast<uintptr_t>(out_base) & 15) ||
                        out_stride < 16 || (out_stride & 15)))) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  uint32_t* ws = nullptr;
  hipError_t e = workspace(&ws);
  if (e != hipSuccess) {
    return e == hipErrorOutOfMemory ? TULIPS_STATUS_NO_MORE_RESOURCES
                                    : TULIPS_STATUS_HARDWARE_ERROR;
  }
  const uint32_t nb = (n + CB - 1) / CB;
  (void)hipGetLastError();
  hipLaunchKernelGGL(seg_count_kernel, dim3(nb), dim3(CB), 0, st, in_base,
                     in_offsets, in_lengths, n, mss, out_first, ws);
  hipLaunchKernelGGL(seg_scan_blocks_kernel, dim3(1), dim3(1024), 0, st, ws, nb,
                     out_first + n);
  hipLaunchKernelGGL(seg_add_kernel, dim3(nb), dim3(CB), 0, st, n, out_first, ws);
  if (out_capacity) {
    const uint32_t blocks = (n + 3) / 4 > 65535 ? 65535 : (n + 3) / 4;
    hipLaunchKernelGGL(segment_kernel, dim3(blocks), dim3(256), 0, st, in_base,
                       in_offsets, in_lengths, n, mss, out_first, out_base,
                       out_stride, out_capacity, out_lengths);
  }
  e = hipGetLastError();
  return e == hipSuccess ? TULIPS_STATUS_OK : TULIPS_STATUS_HARDWARE_ERROR;
}
