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

#include <algorithm>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/tulips_csum.h"
#include "csum_common.h"
#include "frame_common.h"
#include "seg_device.h"
#include "stream_state.h"

namespace tulips_amd {
namespace {

using namespace frame;


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

// Per-frame descriptor written by the prologue (one 16-byte record per input
// frame): everything a segment builder needs to issue its loads, so that
// the segment kernel's chain is run start -> descriptors -> data instead of
// run start -> prefixes -> offsets -> header -> data.
//   x, y: frame address (lo, hi)   z: flen | hlen << 16 | seg_ok << 31
//   w: payload | nseg << 16
__device__ __forceinline__ u32x4
make_desc(uintptr_t fa, uint32_t flen, const SegInfo& si)
{
  u32x4 d;
  d.x = uint32_t(fa);
  d.y = uint32_t(uint64_t(fa) >> 32);
  d.z = (flen & 0xffffu) | (si.hlen << 16) | (si.seg_ok ? 0x80000000u : 0u);
  d.w = (si.payload & 0xffffu) | (si.nseg << 16);
  return d;
}

// ---- exclusive scan of segment counts -------------------------------------

template<int NW>
__device__ __forceinline__ uint32_t
block_inclusive_scan(uint32_t x, uint32_t* lds, uint32_t& total)
{
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  x = wave_inclusive_sum(x);
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
                 uint32_t* __restrict__ first, uint32_t* __restrict__ ws,
                 u32x4* __restrict__ desc)
{
  __shared__ uint32_t lds[CB / 64];
  const uint32_t i = blockIdx.x * CB + threadIdx.x;
  uint32_t c = 0;
  if (i < n) {
    const uintptr_t fa = reinterpret_cast<uintptr_t>(base) + offs[i];
    const uint32_t flen = lens[i];
    const SegInfo si = seg_info(load_seg_header(fa, flen), mss);
    c = si.nseg;
    if (desc) {
      desc[i] = make_desc(fa, flen, si);
    }
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


// Bytes x .. x+15 of a source: two consecutive aligned chunks a, b and the
// offset m = x & 15 (assemble funnel-shifts them with v_alignbyte). Bytes
// outside the frame come back unspecified; callers never use them.
struct Win
{
  u32x4 a, b;
  uint32_t m;
};

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


// One input frame as a segment builder sees it: its prologue descriptor.
struct SegFrame
{
  uintptr_t fa, lo, hi;
  uint32_t flen;
  SegInfo si;
};

__device__ __forceinline__ SegFrame
frame_of(const u32x4& d)
{
  SegFrame F;
  F.fa = uintptr_t((uint64_t(d.y) << 32) | d.x);
  F.flen = d.z & 0xffffu;
  F.lo = F.fa & ~uintptr_t(15);
  F.hi = F.flen ? (F.fa + F.flen - 1) & ~uintptr_t(15) : F.lo;
  F.si.hlen = (d.z >> 16) & 0x7fffu;
  F.si.seg_ok = (d.z >> 31) != 0;
  F.si.payload = d.w & 0xffffu;
  F.si.nseg = d.w >> 16;
  return F;
}

// The aligned chunk after each lane's (lane + 1's, the next batch slot's for
// the subgroup's last lane): lane s hands lane s-1 its chunk, lane 0 hands
// lane G-1 the chunk of the next batch slot.
template<int G>
__device__ __forceinline__ u32x4
next_chunk(const u32x4& cur, const u32x4& nxt, int lane, int sub0)
{
  const u32x4 give = lane == 0 ? nxt : cur;
  const int from = sub0 + ((lane + 1) & (G - 1));
  u32x4 r;
  r.x = __shfl(give.x, from, 64);
  r.y = __shfl(give.y, from, 64);
  r.z = __shfl(give.z, from, 64);
  r.w = __shfl(give.w, from, 64);
  return r;
}



// Build, checksum and store segment k of frame F as output frame j, on one
// G-lane subgroup (lane = index in the subgroup, sub0 = its first lane in the
// wave). Output chunk c holds source bytes [x + 16c, x + 16c + 16), x = the
// segment's source start: lane l loads the 4 source dwords of each of its
// output chunks (one dword-aligned 16-byte load) plus one extra for the batch,
// and takes the fifth dword from lane l+1 for the funnel shift, so a batch of
// SU chunks per lane is SU + 1 loads. The header chunks 0..6 come from one more load per lane and
// are parsed through cross-lane shuffles; everything is issued before the
// first use (the prologue's descriptor is all the addresses need).
//
// KNOWN: F.si comes from the prologue's descriptor. Otherwise (the planned
// entry, no prologue) it is derived here from the header this subgroup loads
// anyway, once the loads are in flight (they need only the frame's address,
// length and k); a k past the frame's segment count (a caller's plan that
// disagrees with the header) writes length 0 and nothing else.
template<int G, int SU, bool KNOWN = true>
__device__ __forceinline__ void
build_segment(const SegFrame& F, uint32_t k, uint32_t j, uint32_t mss, uint8_t* out,
              uint64_t stride, uint16_t* __restrict__ out_lens, int lane, int sub0)
{
  static_assert(G >= 8, "batch slots u > 0 must lie past every header byte");
  SegInfo si = F.si;
  uint32_t slice = 0, dlen = 0;
  if constexpr (KNOWN) {
    slice = si.seg_ok ? min(mss, si.payload - k * mss) : 0u;
    dlen = si.nseg == 1 ? F.flen : si.hlen + slice;
    if (dlen > stride) {
      if (lane == 0) {
        out_lens[j] = 0;
      }
      return;
    }
  }
  const uintptr_t shift = uintptr_t(k) * mss;
  const uintptr_t dst = reinterpret_cast<uintptr_t>(out) + uintptr_t(j) * stride;
  const uintptr_t xs = F.fa + shift;          // source of output byte 0
  // Output chunk c is source bytes [xs + 16c, +16): dwords p0 + 16c .. + 20
  // funnel-shifted by r bytes. Each lane loads the 4 dwords of its chunk at
  // their (4-byte aligned) address and takes the fifth from lane + 1.
  const uintptr_t p0 = xs & ~uintptr_t(3);
  const uint32_t r = uint32_t(xs & 3);
  auto src_chunk = [&](int c, uint32_t& sel) { // clamped to the last chunk
    const uintptr_t p = p0 + 16 * uintptr_t(c);
    const uintptr_t q = p > F.hi ? F.hi : p;   // p >= xs & ~3 >= F.lo
    sel = uint32_t(p - q) >> 2;
    return u32x4(*reinterpret_cast<gdw4_ptr>(q));
  };

  // ---- batch 0 loads: payload chunks (+1), header chunk --------------------
  u32x4 X[SU + 1];
  uint32_t XS[SU + 1];
  auto load_batch = [&](int b0) {
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      X[u] = src_chunk(b0 + lane + G * u, XS[u]);
    }
    X[SU] = src_chunk(lane == 0 ? b0 + G * SU : b0 + lane + G * (SU - 1), XS[SU]);
  };
  uintptr_t hq = F.lo + 16 * uintptr_t(min(lane, 6));
  hq = hq > F.hi ? F.hi : hq;
  const u32x4 H = load_chunk(hq);             // frame chunk min(lane, 6), first
  load_batch(0);
  // every load of the batch is in flight before the header waits for H
  // (left alone, the scheduler trades that overlap for registers); H is
  // issued first, so that wait leaves the payload loads outstanding
  __builtin_amdgcn_sched_barrier(0);

  // ---- header fields (chunks 0..4 from lanes 0..4) -------------------------
  uint32_t FW[13];
  header_words<G>(H, int(F.fa - F.lo), sub0, FW);
  mask_past_end(FW, F.flen);
  const Header h = parse_header<true>(
    [&](int b) -> uint32_t { return (FW[b >> 2] >> (8 * (b & 3))) & 0xffu; }, F.flen);
  if constexpr (!KNOWN) {
    si = seg_info(h, mss);
    slice = si.seg_ok && k < si.nseg ? min(mss, si.payload - k * mss) : 0u;
    dlen = si.nseg == 1 ? F.flen : si.hlen + slice;
    if (k >= si.nseg || dlen > stride) {  // (uniform per subgroup)
      if (lane == 0) {
        out_lens[j] = 0;
      }
      return;
    }
  }
  const int nchunks = int((dlen + 15) >> 4);
  const bool ip_on = h.ipv4;
  const bool l4_on = si.seg_ok || (h.tcp && !h.trunc && h.tcplen >= 18u);
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
  // header window of output chunks 0..5 (segments k > 0 take their header
  // bytes, < hlen <= 94, from the frame's own header)
  Win hw;
  hw.a = H;
  hw.b = next_chunk<G>(H, H, lane, sub0);
  hw.m = uint32_t(F.fa & 15);

  uint32_t l4_acc = 0; // 16-bit halves, 32-bit v_dot2 accumulation (as range_sum32)
  u32x4 keep = {0, 0, 0, 0};
  // first: batch 0, whose slot u = 0 holds output chunks c = lane < G, the
  // only ones that can touch a header byte (hlen <= 94 < 16 * 16 <= 16 * G);
  // every other slot is plain payload.
  auto consume = [&](int c0, bool first) {
    realign(X[0], XS[0]);
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      realign(X[u + 1], XS[u + 1]);
      const uint32_t d4 = next_dword<G>(X[u].x, X[u + 1].x, lane, sub0);
      const int c = c0 + G * u;
      if (c >= nchunks) {
        continue;   // (no break: the shuffles above need every lane)
      }
      const int cb = 16 * c;
      const u32x4 a = X[u];
      u32x4 v;
      v.x = __builtin_amdgcn_alignbyte(a.y, a.x, r);
      v.y = __builtin_amdgcn_alignbyte(a.z, a.y, r);
      v.z = __builtin_amdgcn_alignbyte(a.w, a.z, r);
      v.w = __builtin_amdgcn_alignbyte(d4, a.w, r);
      if (!(first && u == 0)) {
        if (uint32_t(cb + 16) > dlen) {
          v = keep_bytes(v, int(dlen) - cb);
        }
        if (l4_on && uint32_t(cb) < tcp_end) {
          l4_acc = uint32_t(cb + 16) <= tcp_end ? chunk_dot2(v, l4_acc)
                                                 : masked_dot2(v, 0, int(tcp_end) - cb, l4_acc);
        }
        store_chunk(dst + cb, v);
        continue;
      }
      if (shift != 0 && uint32_t(cb) < si.hlen) {
        v = merge_bytes(assemble(hw), v, int(si.hlen) - cb);
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

      if (l4_on && cb + 16 > 34 && uint32_t(cb) < tcp_end) {
        l4_acc = masked_dot2(v, max(34 - cb, 0), min(int(tcp_end) - cb, 16), l4_acc);
      }
      if (c < 4) {
        keep = v;   // line 0 (chunks 0..3) is stored whole after the sums
      } else {
        store_chunk(dst + cb, v);
      }
    }
  };
  // further batches: jumbo segments only (> G*SU chunks); uniform per subgroup
  for (int b0 = 0;;) {
    consume(b0 + lane, b0 == 0);
    b0 += G * SU;
    if (b0 >= nchunks) {
      break;
    }
    load_batch(b0);
  }
  // The output IPv4 header's sum from the frame's header words every lane
  // holds: bytes 14..33 with total length and id as written (bytes 16..19)
  // and the checksum field zero (the output is 16-byte aligned, so the word
  // grids agree); no masked sums over chunks 0..2 and no subgroup reduction
  // for it (as frame_kernel; profiles/ab_frame_ip_header_r06.txt: 0.2-1.5 %
  // per call serially here).
  const uint32_t len_id = si.seg_ok ? (total >> 8) | ((total & 0xffu) << 8) |
                                        ((id >> 8) << 16) | ((id & 0xffu) << 24)
                                    : FW[4];
  const uint32_t ip = fold64(uint64_t(FW[3] >> 16) + len_id + FW[5] +
                             (FW[6] & 0xffff0000u) + FW[7] + (FW[8] & 0xffffu));
  const uint32_t l4 = sub_sum<G>(fold32(l4_acc));
  // lanes 0..3 write the first 64 bytes in one instruction: nontemporal
  // stores are not merged in L2, and separate stores of chunks 1 and 3 wrote
  // that line to HBM three times
  if (lane < 4 && lane < nchunks) {
    if (lane == 1 && ip_on) {
      keep.z |= ~finish(ip, false, MODE_INET, 0, 0, 0, 20) & 0xffffu;
    }
    if (lane == 3 && l4_on) {
      const uint32_t r = finish(l4, false, MODE_TCP, 0, h.src, h.dst, total - 20u);
      keep.x |= (~r & 0xffffu) << 16;
    }
    store_chunk(dst + 16 * uintptr_t(lane), keep);
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
                          uint32_t* __restrict__ runs, u32x4* __restrict__ desc)
{
  __shared__ uint32_t lds[16];
  uint32_t carry = 0;
  for (uint32_t i0 = 0; i0 < n; i0 += 1024) {
    const uint32_t i = i0 + threadIdx.x;
    uint32_t c = 0;
    if (i < n) {
      const uintptr_t fa = reinterpret_cast<uintptr_t>(base) + offs[i];
      const uint32_t flen = lens[i];
      const SegInfo si = seg_info(load_seg_header(fa, flen), mss);
      c = si.nseg;
      if (desc) {
        desc[i] = make_desc(fa, flen, si);
      }
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
segment_kernel(const u32x4* __restrict__ desc, uint32_t mss,
               const uint32_t* __restrict__ first, uint32_t n,
               const uint32_t* __restrict__ runs, uint8_t* out, uint64_t stride,
               uint32_t capacity, uint16_t* __restrict__ out_lens)
{
  constexpr uint32_t S = 256 / G;
  constexpr uint32_t L = RUN + S + 1; // frames [runs[jb/RUN], ...] that can hold jb..jb+S-1
  __shared__ uint32_t pre[L];
  __shared__ u32x4 dsc[L];
  const int lane = threadIdx.x & (G - 1);
  const uint32_t sub = threadIdx.x / G;
  const uint32_t total = min(first[n], capacity);
  for (uint32_t jb = xcd_block(blockIdx.x, gridDim.x) * S; jb < total; jb += gridDim.x * S) {
    const uint32_t ir = runs[jb / RUN];
    if (threadIdx.x < L) {
      pre[threadIdx.x] = first[min(ir + threadIdx.x, n)];
      dsc[threadIdx.x] = desc[min(ir + threadIdx.x, n - 1)];
    }
    __syncthreads();
    const uint32_t j = jb + sub;
    if (j < total) {
      uint32_t f = 0; // pre[f] <= j < pre[f + 1]
#pragma unroll 1
      while (pre[f + 1] <= j) {
        ++f;
      }
      // (opaque per iteration: keeps LLVM from hoisting ~30 lane-derived
      // values out of this loop, which nearly always runs once, into VGPRs
      // that stay live across the whole segment build)
      int l = lane;
      asm volatile("" : "+v"(l));
      build_segment<G, SU>(frame_of(dsc[f]), j - pre[f], j, mss, out, stride, out_lens,
                           l, int(threadIdx.x & 63) & ~(G - 1));
    }
    __syncthreads();
  }
}

// ---- planned segmentation: the caller's first[], no prologue ---------------
//
// The reference decides the TSO split on the host: the transport posts each
// super-frame with its header length (stack::utils::headerLength,
// src/stack/Utils.cpp:67-84) and the MSS (src/transport/ofed/Device.cpp:
// 688-700), and the segment count follows. A caller that has that plan passes
// first[] (n + 1 entries, the exclusive prefix of the per-frame counts) and
// the segment kernel runs alone: each block finds the frames of its S output
// segments in first[] itself and parses their headers from the loads it
// issues for the segments anyway.
//
// Frame search, per block, by wave 0: ONE round trip brings a speculative
// window of PW frames (first[], offsets, lengths) where an evenly cut batch
// would put segment jb (frame jb * n / capacity, a few frames of slack
// before it). A window that does not cover the block's segments (uneven
// counts, capacity far above the total) falls back to a 64-ary search over
// first[] (one round trip per 64x, n <= 2^24: at most 4) and then loads the
// window at the frame found.
constexpr uint32_t PW = 64;     // window frames
constexpr uint32_t PW_BACK = 8; // of which before the guessed frame

template<int G, int SU>
__global__ __launch_bounds__(256) void
segment_planned_kernel(const uint8_t* base, const uint64_t* __restrict__ offs,
                       const uint16_t* __restrict__ lens, uint32_t n, uint32_t mss,
                       const uint32_t* __restrict__ first, uint8_t* out, uint64_t stride,
                       uint32_t capacity, uint16_t* __restrict__ out_lens)
{
  constexpr uint32_t S = 256 / G;
  static_assert(S + 16 <= PW, "the window holds every frame of a block's segments");
  __shared__ uint32_t pre[PW + 1];
  __shared__ uint64_t fadr[PW];
  __shared__ uint32_t flen[PW];
  __shared__ uint32_t total_s, f0_s;
  const uint32_t tid = threadIdx.x;
  const int lane = int(tid) & (G - 1);
  const uint32_t sub = tid / G;
  const uintptr_t b0 = reinterpret_cast<uintptr_t>(base);
  for (uint32_t jb = xcd_block(blockIdx.x, gridDim.x) * S; jb < capacity;
       jb += gridDim.x * S) {
    if (tid < 64) {
      // the window at frame w0: lane t holds frame w0 + t (first[], offset,
      // length), lane 0 also first[w0 + PW] and first[n]
      auto load_window = [&](uint32_t w0, uint32_t& p, uint32_t& pend, uint64_t& o, uint32_t& l) {
        const uint32_t f = w0 + tid;
        p = first[min(f, n)];
        o = offs[min(f, n - 1)];
        l = lens[min(f, n - 1)];
        pend = first[min(w0 + PW, n)];
      };
      const uint32_t g = uint32_t(uint64_t(jb) * n / capacity);
      uint32_t w0 = g > PW_BACK ? g - PW_BACK : 0u;
      uint32_t p, pend;
      uint64_t o;
      uint32_t l;
      load_window(w0, p, pend, o, l);
      const uint32_t total = min(first[n], capacity);
      const uint32_t jl = min(jb + S, max(total, jb + 1)) - 1; // the block's last segment
      const uint32_t p0 = __shfl(p, 0, 64);
      if (jb < total && !(p0 <= jb && jl < pend)) {
        // the window missed: 64-ary search for the frame of jb (first[lo] <=
        // jb < first[hi]); a span of at most PW - S - 1 frames leaves room
        // for the block's other segments' frames in the window at lo
        uint32_t lo = 0, hi = n;
        while (hi - lo > PW - S - 1) {
          const uint32_t span = hi - lo;
          const uint32_t v = first[lo + uint32_t(uint64_t(span) * tid / 64)];
          const uint64_t m = __ballot(v <= jb);
          const uint32_t t = m ? 63u - uint32_t(__builtin_clzll(m)) : 0u;
          const uint32_t nlo = lo + uint32_t(uint64_t(span) * t / 64);
          hi = t == 63 ? hi : lo + uint32_t(uint64_t(span) * (t + 1) / 64);
          lo = nlo;
        }
        w0 = lo;
        load_window(w0, p, pend, o, l);
      }
      pre[tid] = p;
      fadr[tid] = b0 + o;
      flen[tid] = l;
      // the window index of jb's frame (the last entry at or below jb), where
      // every subgroup's scan starts
      const uint64_t at_or_below = __ballot(p <= jb);
      if (tid == 0) {
        pre[PW] = pend;
        total_s = total;
        f0_s = at_or_below ? 63u - uint32_t(__builtin_clzll(at_or_below)) : 0u;
      }
    }
    __syncthreads();
    const uint32_t total = total_s;
    if (jb >= total) {
      break; // (uniform: later tiles lie further past the total)
    }
    const uint32_t j = jb + sub;
    if (j < total) {
      uint32_t f = f0_s; // pre[f] <= j < pre[f + 1] within the window
#pragma unroll 1
      while (f + 1 < PW && pre[f + 1] <= j) {
        ++f;
      }
      SegFrame F;
      F.fa = uintptr_t(fadr[f]);
      F.flen = flen[f];
      F.lo = F.fa & ~uintptr_t(15);
      F.hi = F.flen ? (F.fa + F.flen - 1) & ~uintptr_t(15) : F.lo;
      const uint32_t k = j - pre[f];
      // (a plan with a frame of no segments, which the rule never makes, can
      // put a block's last segments past the window: those get length 0)
      const bool inside = pre[f] <= j && j < pre[f + 1];
      int lv = lane;
      asm volatile("" : "+v"(lv));
      if (inside) {
        build_segment<G, SU, false>(F, k, j, mss, out, stride, out_lens, lv,
                                    int(tid & 63) & ~(G - 1));
      } else if (lane == 0) {
        out_lens[j] = 0; // the caller's first[] is not a prefix for this batch
      }
    }
#ifdef TCS_SEG_LAST_BARRIER
    __syncthreads();
#else
    // the window is rewritten only by a next tile: a block with none (the
    // grid covers the capacity) lets each wave leave as soon as it is done
    if (jb + gridDim.x * S < capacity) {
      __syncthreads();
    }
#endif
  }
}


// Workspace per (device, stream) (stream_state.h): the scan's block totals
// (MAX_FRAMES / CB words), the run starts (one word per RUN output segments)
// and the frame descriptors (16 bytes per input frame). Direct calls on one
// stream run in order, so they share one, grown when a call needs more (the
// old arrays are freed once the stream is idle: no graph holds them). The
// calls one capture records on a stream share a workspace made for that
// capture and owned by its graph, so a later direct call can neither free it
// under the graph nor race a replay on it. The caller holds the stream's call
// mutex.
hipError_t
ws_alloc(int device, uint64_t nruns, uint64_t ndesc, StreamState::SegWs* w,
         std::vector<void*>* made)
{
  struct Part
  {
    void** p;
    size_t bytes;
  };
  const Part parts[3] = { { reinterpret_cast<void**>(&w->blocks),
                            sizeof(uint32_t) * (MAX_FRAMES / CB) },
                          { reinterpret_cast<void**>(&w->runs), sizeof(uint32_t) * nruns },
                          { &w->desc, sizeof(u32x4) * ndesc } };
  for (const Part& q : parts) {
    if (*q.p) {
      continue;
    }
    const hipError_t e = device_malloc(device, q.p, q.bytes);
    if (e != hipSuccess) {
      *q.p = nullptr;
      return e;
    }
    made->push_back(*q.p);
  }
  w->nruns = nruns;
  w->ndesc = ndesc;
  return hipSuccess;
}

hipError_t
workspace(StreamState& s, bool capturing, uint32_t capacity, uint32_t n,
          uint32_t** blocks, uint32_t** runs, u32x4** desc)
{
  const uint64_t need_runs = (uint64_t(capacity) + RUN - 1) / RUN;
  const uint64_t need_desc = capacity ? uint64_t(n) : 0;
  StreamState::SegWs* w = nullptr;
  if (capturing) {
    StreamState::Capture* c = nullptr;
    if (capture_record(s, &c) != hipSuccess) {
      return hipErrorStreamCaptureUnsupported;
    }
    if (!c->seg.blocks || c->seg.nruns < need_runs || c->seg.ndesc < need_desc) {
      // a fresh one sized for this call (the graph keeps it; an earlier one
      // of this capture stays with the calls recorded on it)
      StreamState::SegWs fresh;
      std::vector<void*> made;
      const hipError_t e = ws_alloc(s.device, need_runs ? need_runs : 1,
                                    need_desc ? need_desc : 1, &fresh, &made);
      capture_keep(s, made);
      if (e != hipSuccess) {
        return e;
      }
      c->seg = fresh;
    }
    w = &c->seg;
  } else {
    w = &s.seg;
    if (!w->blocks || need_runs > w->nruns || need_desc > w->ndesc) {
      StreamState::SegWs grown;
      grown.blocks = w->blocks;
      if (need_runs <= w->nruns) {
        grown.runs = w->runs;
      }
      if (need_desc <= w->ndesc) {
        grown.desc = w->desc;
      }
      std::vector<void*> made;
      const uint64_t nr = std::max<uint64_t>(std::max<uint64_t>(need_runs, 65536), w->nruns);
      const uint64_t nd = std::max<uint64_t>(std::max<uint64_t>(need_desc, 65536), w->ndesc);
      hipError_t e = ws_alloc(s.device, grown.runs ? w->nruns : nr,
                              grown.desc ? w->ndesc : nd, &grown, &made);
      if (e == hipSuccess) {
        e = sync_stream(s.stream); // the arrays replaced are idle
      }
      if (e != hipSuccess) {
        device_free(s.device, made);
        return e;
      }
      device_free(s.device, { grown.runs != w->runs ? w->runs : nullptr,
                              grown.desc != w->desc ? w->desc : nullptr });
      *w = grown;
    }
  }
  *blocks = w->blocks;
  *runs = w->runs;
  *desc = static_cast<u32x4*>(w->desc);
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
  std::shared_ptr<StreamState> ss;
  hipError_t e = stream_state(st, &ss);
  if (e != hipSuccess) {
    return TULIPS_STATUS_HARDWARE_ERROR;
  }
  // the prologue and the segment kernel share the stream's workspace: queue
  // them as one sequence (stream_state.h)
  std::lock_guard<std::recursive_mutex> g(ss->call);
  uint32_t* ws = nullptr;
  uint32_t* runs = nullptr;
  u32x4* desc = nullptr;
  e = workspace(*ss, stream_capturing(st), out_capacity, n, &ws, &runs, &desc);
  if (e != hipSuccess) {
    return e == hipErrorOutOfMemory                ? TULIPS_STATUS_NO_MORE_RESOURCES
           : e == hipErrorStreamCaptureUnsupported ? TULIPS_STATUS_INVALID_ARGUMENT
                                                   : TULIPS_STATUS_HARDWARE_ERROR;
  }
  const uint32_t nb = (n + CB - 1) / CB;
  (void)hipGetLastError();
  if (n <= SMALL_N) {
    hipLaunchKernelGGL(seg_prologue_small_kernel, dim3(1), dim3(1024), 0, st, in_base,
                       in_offsets, in_lengths, n, mss, out_first, out_capacity,
                       out_capacity ? runs : nullptr, out_capacity ? desc : nullptr);
  } else {
    hipLaunchKernelGGL(seg_count_kernel, dim3(nb), dim3(CB), 0, st, in_base,
                       in_offsets, in_lengths, n, mss, out_first, ws,
                       out_capacity ? desc : nullptr);
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
      hipLaunchKernelGGL((segment_kernel<16, 6>), dim3(blocks), dim3(256), 0, st, desc,
                         mss, out_first, n, runs, out_base, out_stride, out_capacity,
                         out_lengths);
    } else {
      hipLaunchKernelGGL((segment_kernel<64, 6>), dim3(blocks), dim3(256), 0, st, desc,
                         mss, out_first, n, runs, out_base, out_stride, out_capacity,
                         out_lengths);
    }
  }
  e = hipGetLastError();
  return e == hipSuccess ? TULIPS_STATUS_OK : TULIPS_STATUS_HARDWARE_ERROR;
}

extern "C" int
tulips_csum_segment_frames_planned(const uint8_t* in_base, const uint64_t* in_offsets,
                                   const uint16_t* in_lengths, uint32_t n, uint32_t mss,
                                   const uint32_t* first, uint8_t* out_base,
                                   uint64_t out_stride, uint32_t out_capacity,
                                   uint16_t* out_lengths, void* stream)
{
  using namespace tulips_amd;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (mss == 0 || mss > 0xffffu || n > MAX_FRAMES) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (n == 0 || out_capacity == 0) {
    return TULIPS_STATUS_OK;
  }
  if (!in_base || !in_offsets || !in_lengths || !first || !out_base || !out_lengths ||
      (reinterpret_cast<uintptr_t>(out_base) & 15) || out_stride < 16 || (out_stride & 15)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  const bool small = mss <= 1460;
  const uint32_t per_block = small ? 256 / 16 : 256 / 64;
  const uint64_t want = (uint64_t(out_capacity) + per_block - 1) / per_block;
  const uint32_t blocks = uint32_t(want > 65535 ? 65535 : want);
  (void)hipGetLastError();
  if (small) {
    hipLaunchKernelGGL((segment_planned_kernel<16, 6>), dim3(blocks), dim3(256), 0, st,
                       in_base, in_offsets, in_lengths, n, mss, first, out_base, out_stride,
                       out_capacity, out_lengths);
  } else {
    hipLaunchKernelGGL((segment_planned_kernel<64, 6>), dim3(blocks), dim3(256), 0, st,
                       in_base, in_offsets, in_lengths, n, mss, first, out_base, out_stride,
                       out_capacity, out_lengths);
  }
  return hipGetLastError() == hipSuccess ? TULIPS_STATUS_OK : TULIPS_STATUS_HARDWARE_ERROR;
}

extern "C" int
tulips_csum_segment_plan_host(const uint8_t* base, const uint64_t* offsets,
                              const uint16_t* lengths, uint32_t n, uint32_t mss,
                              uint32_t* first)
{
  if (!first || mss == 0 || mss > 0xffffu || (n && (!base || !offsets || !lengths))) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  // seg_info of the device prologue, on bytes read in place (0 past the frame)
  uint64_t acc = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t* f = base + offsets[i];
    const uint32_t flen = lengths[i];
    auto at = [&](uint32_t k) -> uint32_t { return k < flen ? f[k] : 0u; };
    const bool eth_ip = flen >= 14 && ((at(12) << 8) | at(13)) == 0x0800u;
    const bool runt = eth_ip && flen < 34;
    const bool ipv4 = eth_ip && !runt && at(14) == 0x45u;
    const bool tcp = ipv4 && (at(20) & 0x3fu) == 0 && at(21) == 0 && at(23) == 6u;
    const uint32_t total = (at(16) << 8) | at(17);
    const uint32_t tcplen = (total - 20u) & 0xffffu;
    const bool trunc = tcp && (total < 20u || 34u + tcplen > flen);
    const uint32_t doff = at(46) >> 4;
    const bool seg_ok = tcp && !trunc && doff >= 5 && 20u + 4u * doff <= total;
    const uint32_t payload = seg_ok ? total - 20u - 4u * doff : 0u;
    first[i] = uint32_t(acc);
    acc += (seg_ok && payload > mss) ? (payload + mss - 1) / mss : 1u;
    if (acc > 0xffffffffull) {
      return TULIPS_STATUS_INVALID_ARGUMENT;
    }
  }
  first[n] = uint32_t(acc);
  return TULIPS_STATUS_OK;
}

