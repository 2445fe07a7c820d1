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
// on the device (first[n] = total), plus the frame of every RUN-th segment,
// so the work spreads over output segments (one 16-lane subgroup each, four
// per wave) rather than over super-frames. For a segment, each lane
// assembles aligned 16-byte destination chunks from funnel-shifted source
// chunks (v_alignbyte), patches the header fields in registers, sums them for
// both checksums, and stores; the two chunks that hold checksum fields are
// stored after the subgroup reduction. Reads each source byte from HBM
// once and writes each destination byte once.
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
// outside the frame come back unspecified; callers never use them):
// load_win issues the loads, assemble funnel-shifts them (v_alignbyte).
struct Win
{
  u32x4 a, b;
  uint32_t m;
};

__device__ __forceinline__ Win
load_win(uintptr_t x, uintptr_t lo, uintptr_t hi)
{
  const uintptr_t q = x & ~uintptr_t(15);
  const uintptr_t q0 = q < lo ? lo : (q > hi ? hi : q);
  const uintptr_t q1 = q + 16 > hi ? hi : q + 16;
  Win w;
  w.a = load_chunk(q0);
  w.b = load_chunk(q1);
  w.m = uint32_t(x & 15);
  return w;
}

__device__ __forceinline__ u32x4
assemble(const Win& w)
{
  const u32x4 a = w.a, b = w.b;
  const uint32_t r = w.m & 3;
  uint32_t d0, d1, d2, d3, d4;
  switch (w.m >> 2) {
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

// One input frame as a segment builder sees it.
struct SegFrame
{
  uintptr_t fa, lo, hi;
  uint32_t flen;
  Header h;
  SegInfo si;
  bool ip_on, l4_on;
};

// The frame's header is read by every lane of the subgroup itself
// (load_header: broadcast chunk loads, no cross-lane traffic).
__device__ __forceinline__ SegFrame
seg_frame(uintptr_t fa, uint32_t flen, uint32_t mss)
{
  SegFrame F;
  F.fa = fa;
  F.flen = flen;
  F.lo = fa & ~uintptr_t(15);
  F.hi = flen ? (fa + flen - 1) & ~uintptr_t(15) : F.lo;
  F.h = load_header(fa, flen);
  F.si = seg_info(F.h, mss);
  F.ip_on = F.h.ipv4;
  F.l4_on = F.si.seg_ok || (F.h.tcp && !F.h.trunc && F.h.tcplen >= 18u);
  return F;
}

// Build, checksum and store segment k of frame F as output frame j, on one
// G-lane subgroup (lane = index in the subgroup). SU chunks per lane per
// batch, every load of a batch issued before any is used.
template<int G, int SU>
__device__ __forceinline__ void
build_segment(const SegFrame& F, uint32_t k, uint32_t j, uint32_t mss, uint8_t* out,
              uint64_t stride, uint16_t* __restrict__ out_lens, int lane)
{
  const Header& h = F.h;
  const SegInfo& si = F.si;
  const uint32_t slice = si.seg_ok ? min(mss, si.payload - k * mss) : 0u;
  const uint32_t dlen = si.nseg == 1 ? F.flen : si.hlen + slice;
  if (dlen > stride) {
    if (lane == 0) {
      out_lens[j] = 0;
    }
    return;
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
  for (int c0 = lane; c0 < nchunks; c0 += G * SU) {
    Win pw[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int cb = 16 * min(c0 + G * u, nchunks - 1);
      pw[u] = load_win(F.fa + shift + cb, F.lo, F.hi);
    }
    // header bytes (< hlen <= 94) of segments k > 0 come from the frame's
    // own header: only chunks 0..5, i.e. lanes 0..5 of the first batch
    const Win hw = load_win(F.fa + 16 * min(c0, 5), F.lo, F.hi);
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int c = c0 + G * u;
      if (c >= nchunks) {
        break;
      }
      const int cb = 16 * c;
      u32x4 v = assemble(pw[u]);
      if (shift != 0 && uint32_t(cb) < si.hlen) {
        v = merge_bytes(assemble(hw), v, int(si.hlen) - cb);
      }
      if (uint32_t(cb + 16) > dlen) {
        v = keep_bytes(v, int(dlen) - cb);
      }
      if (c == 1 && F.ip_on) {
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
      if (c == 3 && F.l4_on) {
        v.x &= 0x0000ffffu; // chksum = 0
      }
      if (F.ip_on && cb < 34) {
        ip_acc += masked_hsum(v, max(14 - cb, 0), min(34 - cb, 16));
      }
      if (F.l4_on && cb + 16 > 34 && uint32_t(cb) < tcp_end) {
        l4_acc += masked_hsum(v, max(34 - cb, 0), min(int(tcp_end) - cb, 16));
      }
      if (c == 1 || c == 3) {
        keep = v;
      } else {
        *reinterpret_cast<gchunk_wptr>(dst + cb) = v;
      }
    }
  }
  const uint32_t ip = sub_sum<G>(fold64(ip_acc));
  const uint32_t l4 = sub_sum<G>(fold64(l4_acc));
  if (lane == 1 && nchunks > 1) {
    if (F.ip_on) {
      keep.z |= ~finish(ip, false, MODE_INET, 0, 0, 0, 20) & 0xffffu;
    }
    *reinterpret_cast<gchunk_wptr>(dst + 16) = keep;
  }
  if (lane == 3 && nchunks > 3) {
    if (F.l4_on) {
      const uint32_t r = finish(l4, false, MODE_TCP, 0, h.src, h.dst, total - 20u);
      keep.x |= (~r & 0xffffu) << 16;
    }
    *reinterpret_cast<gchunk_wptr>(dst + 48) = keep;
  }
  if (lane == 0) {
    out_lens[j] = uint16_t(dlen);
  }
}

// Run starts: runs[r] = the frame holding segment r*RUN. A segment-kernel
// block covering segments [jb, jb + S) loads the prefixes of frames
// runs[jb / RUN] .. +RUN+S into LDS and finds each segment's frame there.
constexpr uint32_t RUN = 16;

__device__ __forceinline__ void
mark_runs(uint32_t i, uint32_t a, uint32_t c, uint32_t capacity,
          uint32_t* __restrict__ runs)
{
  const uint32_t b = min(a + c, capacity);
  for (uint32_t r = (a + RUN - 1) / RUN; r * RUN < b; ++r) {
    runs[r] = i;
  }
}

__global__ __launch_bounds__(CB) void
seg_runs_kernel(uint32_t n, const uint32_t* __restrict__ first, uint32_t capacity,
                uint32_t* __restrict__ runs)
{
  const uint32_t i = blockIdx.x * CB + threadIdx.x;
  if (i < n) {
    mark_runs(i, first[i], first[i + 1] - first[i], capacity, runs);
  }
}

// Small batches (n <= SMALL_N): count, scan and run starts in ONE launch of
// one 1024-thread block, in rounds of 1024 frames with a carried prefix
// (each of the 4 kernels of the large path costs ~4-5 us).
constexpr uint32_t SMALL_N = 16384;

__global__ __launch_bounds__(1024) void
seg_prologue_small_kernel(const uint8_t* base, const uint64_t* __restrict__ offs,
                          const uint16_t* __restrict__ lens, uint32_t n, uint32_t mss,
                          uint32_t* __restrict__ first, uint32_t capacity,
                          uint32_t* __restrict__ runs)
{
  __shared__ uint32_t lds[16];
  uint32_t carry = 0;
  for (uint32_t i0 = 0; i0 < n; i0 += 1024) {
    const uint32_t i = i0 + threadIdx.x;
    uint32_t c = 0;
    if (i < n) {
      const uintptr_t fa = reinterpret_cast<uintptr_t>(base) + offs[i];
      c = seg_info(load_header(fa, lens[i]), mss).nseg;
    }
    uint32_t tile;
    const uint32_t a = carry + block_inclusive_scan<16>(c, lds, tile) - c;
    if (i < n) {
      first[i] = a;
      if (runs) {
        mark_runs(i, a, c, capacity, runs);
      }
    }
    carry += tile;
  }
  if (threadIdx.x == 0) {
    first[n] = carry;
  }
}

// Work is spread over output segments: one G-lane subgroup per segment,
// S = 256 / G consecutive segments per block. A batch of 1024 64 KiB
// super-frames at MSS 1460 is 45,056 independent segments.
template<int G, int SU>
__global__ __launch_bounds__(256) void
segment_kernel(const uint8_t* in, const uint64_t* __restrict__ offs,
               const uint16_t* __restrict__ lens, uint32_t mss,
               const uint32_t* __restrict__ first, uint32_t n,
               const uint32_t* __restrict__ runs, uint8_t* out, uint64_t stride,
               uint32_t capacity, uint16_t* __restrict__ out_lens)
{
  constexpr uint32_t S = 256 / G;
  constexpr uint32_t L = RUN + S + 1; // frames [runs[jb/RUN], ...] that can hold jb..jb+S-1
  __shared__ uint32_t pre[L];
  const int lane = threadIdx.x & (G - 1);
  const uint32_t sub = threadIdx.x / G;
  const uint32_t total = min(first[n], capacity);
  for (uint32_t jb = blockIdx.x * S; jb < total; jb += gridDim.x * S) {
    const uint32_t ir = runs[jb / RUN];
    if (threadIdx.x < L) {
      pre[threadIdx.x] = first[min(ir + threadIdx.x, n)];
    }
    __syncthreads();
    const uint32_t j = jb + sub;
    if (j < total) {
      uint32_t f = 0; // pre[f] <= j < pre[f + 1]
#pragma unroll 1
      while (pre[f + 1] <= j) {
        ++f;
      }
      const uint32_t i = ir + f;
      const SegFrame F =
        seg_frame(reinterpret_cast<uintptr_t>(in) + offs[i], lens[i], mss);
      build_segment<G, SU>(F, j - pre[f], j, mss, out, stride, out_lens, lane);
    }
    __syncthreads();
  }
}

// Per-device workspace: the scan's block totals (MAX_FRAMES / CB words) and
// the run starts (one word per RUN output segments). Made on first use
// and grown when a call's capacity needs a longer map; a call that grows it
// cannot be captured in a HIP graph (warm it up outside the capture).
struct Workspace
{
  uint32_t* blocks = nullptr;
  uint32_t* runs = nullptr;
  uint64_t nruns = 0;
};
std::mutex g_ws_mutex;
Workspace g_ws[64];

hipError_t
workspace(uint32_t capacity, uint32_t** blocks, uint32_t** runs)
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
  Workspace& w = g_ws[dev];
  if (!w.blocks) {
    e = hipMalloc(reinterpret_cast<void**>(&w.blocks),
                  sizeof(uint32_t) * (MAX_FRAMES / CB));
    if (e != hipSuccess) {
      w.blocks = nullptr;
      return e;
    }
  }
  const uint64_t need = (uint64_t(capacity) + RUN - 1) / RUN;
  if (need > w.nruns) {
    const uint64_t want = need < 65536 ? 65536 : need;
    uint32_t* p = nullptr;
    e = hipMalloc(reinterpret_cast<void**>(&p), sizeof(uint32_t) * want);
    if (e != hipSuccess) {
      return e;
    }
    if (w.runs) {
      (void)hipDeviceSynchronize(); // the old array may still be in use
      (void)hipFree(w.runs);
    }
    w.runs = p;
    w.nruns = want;
  }
  *blocks = w.blocks;
  *runs = w.runs;
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
  uint32_t* runs = nullptr;
  hipError_t e = workspace(out_capacity, &ws, &runs);
  if (e != hipSuccess) {
    return e == hipErrorOutOfMemory ? TULIPS_STATUS_NO_MORE_RESOURCES
                                    : TULIPS_STATUS_HARDWARE_ERROR;
  }
  const uint32_t nb = (n + CB - 1) / CB;
  (void)hipGetLastError();
  if (n <= SMALL_N) {
    hipLaunchKernelGGL(seg_prologue_small_kernel, dim3(1), dim3(1024), 0, st, in_base,
                       in_offsets, in_lengths, n, mss, out_first, out_capacity,
                       out_capacity ? runs : nullptr);
  } else {
    hipLaunchKernelGGL(seg_count_kernel, dim3(nb), dim3(CB), 0, st, in_base,
                       in_offsets, in_lengths, n, mss, out_first, ws);
    hipLaunchKernelGGL(seg_scan_blocks_kernel, dim3(1), dim3(1024), 0, st, ws, nb,
                       out_first + n);
    hipLaunchKernelGGL(seg_add_kernel, dim3(nb), dim3(CB), 0, st, n, out_first, ws);
    if (out_capacity) {
      hipLaunchKernelGGL(seg_runs_kernel, dim3(nb), dim3(CB), 0, st, n, out_first,
                         out_capacity, runs);
    }
  }
  if (out_capacity) {
    // 16 lanes x 6 chunks = a 1536 B segment per batch (MSS 1460 frames in
    // one batch); whole waves for jumbo MSS.
    const bool small = mss <= 1460;
    const uint32_t per_block = small ? 256 / 16 : 256 / 64; // segments per block
    const uint64_t want = (uint64_t(out_capacity) + per_block - 1) / per_block;
    const uint32_t blocks = uint32_t(want > 65535 ? 65535 : want);
    if (small) {
      hipLaunchKernelGGL((segment_kernel<16, 6>), dim3(blocks), dim3(256), 0, st, in_base,
                         in_offsets, in_lengths, mss, out_first, n, runs, out_base,
                         out_stride, out_capacity, out_lengths);
    } else {
      hipLaunchKernelGGL((segment_kernel<64, 6>), dim3(blocks), dim3(256), 0, st, in_base,
                         in_offsets, in_lengths, mss, out_first, n, runs, out_base,
                         out_stride, out_capacity, out_lengths);
    }
  }
  e = hipGetLastError();
  return e == hipSuccess ? TULIPS_STATUS_OK : TULIPS_STATUS_HARDWARE_ERROR;
}
