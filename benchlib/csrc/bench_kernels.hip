// bench_kernels.hip — libtulips_csum_bench.so: the measurement and
// test-data entry points of include/tulips_csum_bench.h, kept out of the
// product library (which exports include/tulips_csum.h only). The ceiling
// kernels repeat the product kernels' load/store patterns without their
// arithmetic, from the same device headers, so a ceiling moves with the
// kernel it bounds.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/tulips_csum_bench.h"
#include "../../tulips_amd/csrc/csum_common.h"
#include "../../tulips_amd/csrc/csum_device.h"
#include "../../tulips_amd/csrc/seg_device.h"

namespace tulips_bench {
using namespace tulips_amd;

namespace {

__device__ __forceinline__ uint64_t
splitmix_mix(uint64_t z)
{
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Thread t produces draw k = k0 + t (8 arena bytes) and stores the part of
// it that falls in [byte_off, byte_off + nbytes).
__global__ __launch_bounds__(256) void
fill_splitmix_kernel(uint8_t* __restrict__ dst, uint64_t nbytes, uint64_t seed,
                     uint64_t byte_off, uint64_t ndraws)
{
  const uint64_t k0 = byte_off >> 3;
  for (uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
       t < ndraws; t += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t k = k0 + t;
    const uint64_t z = splitmix_mix(seed + (k + 1) * 0x9E3779B97F4A7C15ull);
    const int64_t rel = int64_t(k * 8) - int64_t(byte_off); // dst index of byte 0
    if (rel >= 0 && uint64_t(rel) + 8 <= nbytes && ((rel & 7) == 0) &&
        ((reinterpret_cast<uintptr_t>(dst) & 7) == 0)) {
      *reinterpret_cast<uint64_t*>(dst + rel) = z;
    } else {
      for (int b = 0; b < 8; ++b) {
        const int64_t i = rel + b;
        if (i >= 0 && uint64_t(i) < nbytes) {
          dst[i] = uint8_t(z >> (8 * b));
        }
      }
    }
  }
}

// Plain streaming read of [p, p+nbytes) (16-byte chunks, nbytes % 16 == 0):
// the calibration ceiling for the checksum kernels' HBM read rate. It reads
// exactly as the fastest checksum geometry does (the F9000 kernel: one wave
// per contiguous 12 KiB tile = 64 lanes x 12 nt dwordx4 loads issued back to
// back, 256-thread blocks in the XCD-clustered order of csum_common.h) and
// only XORs what it loaded, so it bounds that kernel from above.
__global__ __launch_bounds__(256) void
stream_read_kernel(uintptr_t base, uint64_t nchunks,
                   uint32_t* __restrict__ sink)
{
  constexpr int U = 12;
  const gchunk_ptr p = reinterpret_cast<gchunk_ptr>(base);
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave =
    (uint64_t(xcd_block(blockIdx.x, gridDim.x)) * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = (uint64_t(gridDim.x) * blockDim.x) >> 6;
  const uint64_t ntiles = nchunks / (64 * U);
  uint32_t x = 0;
  for (uint64_t t = wave; t < ntiles; t += nwaves) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u] = __builtin_nontemporal_load(p + t * (64 * U) + u * 64 + lane);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
  }
  for (uint64_t i = ntiles * (64 * U) + wave * 64 + lane; i < nchunks;
       i += nwaves * 64) {
    const u32x4 a = p[i];
    x ^= a.x ^ a.y ^ a.z ^ a.w;
  }
  if (x == 0x9e3779b9u) { // practically never; keeps the loads live
    sink[0] = x;
  }
}

// The F9000 checksum kernel's exact read pattern without its arithmetic:
// wave w reads the 16-byte chunks of tile [w * tile, (w + 1) * tile) at
// absolute alignment, 64 lanes x 12 unconditional loads, slots past the
// tile re-reading its last chunk (as csum_kernel<64, 12> does for one
// segment per wave), in the same XCD-clustered block order. Bounds that
// kernel from above.
__global__ __launch_bounds__(256) void
stream_tiles_kernel(uintptr_t base, uint64_t tile, uint32_t ntiles, uint32_t* __restrict__ sink)
{
  constexpr int U = 12;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = (xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x) >> 6;
  if (wave >= ntiles) {
    return;
  }
  const uintptr_t sa = base + uint64_t(wave) * tile;
  const uintptr_t a0 = sa & ~uintptr_t(15);
  const int last = int((sa + tile - a0 + 15) >> 4) - 1;
  const gchunk_ptr p = reinterpret_cast<gchunk_ptr>(a0);
  uint32_t x = 0;
  for (int c = int(lane); c <= last; c += U * 64) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u] = __builtin_nontemporal_load(p + min(c + u * 64, last));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
  }
  if (x == 0x9e3779b9u) { // practically never; keeps the loads live
    sink[0] = x;
  }
}

// The frame kernels' read pattern without their arithmetic: slot k's bytes
// [base + k * stride, + bytes) read by one G-lane subgroup, U clamped 16-byte
// nontemporal loads per lane per pass (frame_kernel<., 16, 6>: a 1514 B frame
// is one pass), 256-thread blocks in the XCD-clustered order. Bounds the
// frame kernels from above for frames in fixed receive slots.
template<int G, int U>
__global__ __launch_bounds__(256) void
stream_slots_kernel(uintptr_t base, uint64_t stride, uint32_t bytes, uint32_t n,
                    uint32_t* __restrict__ sink)
{
  const uint32_t t = xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const uint32_t k = t / G, lane = t % G;
  if (k >= n) {
    return;
  }
  const uintptr_t sa = base + uint64_t(k) * stride;
  const uintptr_t a0 = sa & ~uintptr_t(15);
  const int last = int((sa + bytes - a0 + 15) >> 4) - 1;
  const gchunk_ptr p = reinterpret_cast<gchunk_ptr>(a0);
  uint32_t x = 0;
  for (int c = int(lane); c <= last; c += U * G) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u] = __builtin_nontemporal_load(p + min(c + u * G, last));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
  }
  if (x == 0x9e3779b9u) { // practically never; keeps the loads live
    sink[0] = x;
  }
}

} // namespace

hipError_t
launch_stream_slots(const uint8_t* p, uint64_t stride, uint32_t bytes, uint32_t n, int group,
                    int unroll, uint32_t* sink, hipStream_t stream)
{
  if (n == 0 || bytes == 0) {
    return hipSuccess;
  }
  const uint32_t blocks = uint32_t((uint64_t(n) * uint32_t(group) + 255) / 256);
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  (void)hipGetLastError();
  if (group == 16 && unroll == 6) {
    hipLaunchKernelGGL((stream_slots_kernel<16, 6>), dim3(blocks), dim3(256), 0, stream, a,
                       stride, bytes, n, sink);
  } else if (group == 32 && unroll == 3) {
    hipLaunchKernelGGL((stream_slots_kernel<32, 3>), dim3(blocks), dim3(256), 0, stream, a,
                       stride, bytes, n, sink);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t
launch_stream_tiles(const uint8_t* p, uint64_t tile, uint32_t ntiles, uint32_t* sink,
                    hipStream_t stream)
{
  if (ntiles == 0 || tile == 0) {
    return hipSuccess;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL(stream_tiles_kernel, dim3((ntiles + 3) / 4), dim3(256), 0, stream,
                     reinterpret_cast<uintptr_t>(p), tile, ntiles, sink);
  return hipGetLastError();
}

hipError_t
launch_fill_splitmix(uint8_t* dst, uint64_t nbytes, uint64_t seed,
                     uint64_t byte_off, hipStream_t stream)
{
  if (nbytes == 0) {
    return hipSuccess;
  }
  const uint64_t first = byte_off >> 3;
  const uint64_t last = (byte_off + nbytes - 1) >> 3;
  const uint64_t ndraws = last - first + 1;
  uint64_t blocks = (ndraws + 255) / 256;
  if (blocks > 8192) {
    blocks = 8192;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL(fill_splitmix_kernel, dim3(uint32_t(blocks)), dim3(256),
                     0, stream, dst, nbytes, seed, byte_off, ndraws);
  return hipGetLastError();
}

hipError_t
launch_stream_read(const uint8_t* p, uint64_t nbytes, uint32_t* sink,
                   uint32_t max_blocks, hipStream_t stream)
{
  const uint64_t nchunks = nbytes / 16;
  if (nchunks == 0) {
    return hipSuccess;
  }
  // one 12 KiB tile per wave (4 waves per block), as the checksum kernel's
  // one 9000 B segment per wave: no grid-stride cap by default
  uint64_t blocks = (nchunks + 4 * 64 * 12 - 1) / (4 * 64 * 12);
  const uint64_t cap = max_blocks ? max_blocks : (1u << 30);
  if (blocks > cap) {
    blocks = cap;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL(stream_read_kernel, dim3(uint32_t(blocks)), dim3(256), 0,
                     stream, reinterpret_cast<uintptr_t>(p), nchunks, sink);
  return hipGetLastError();
}

namespace {

// One wave that returns after `ticks` of the 100 MHz realtime counter.
__global__ __launch_bounds__(64) void
gpu_sleep_kernel(uint64_t ticks)
{
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
  }
}


namespace seg {
using namespace tulips_amd::frame;

// The segment kernels' data movement without their header work: slot k
// copies source bytes [src + (k / per) * gstride + (k % per) * step, + bytes)
// to out + k * ostride, one G-lane subgroup per slot, SU + 1 dword-aligned
// 16-byte loads per lane per batch (clamped to the source's last 16-byte
// chunk), funnel shift, nontemporal 16-byte stores: build_segment's loads and
// stores with no header chunk, parse, patch or sums. The ceiling the
// segmentation figures are held against (bench.py extras.segment_*).
template<int G, int SU>
__global__ __launch_bounds__(256) void
copy_slots_kernel(uintptr_t src, uint64_t gstride, uint32_t per, uint32_t step, uint32_t bytes,
                  uint32_t n, uint8_t* out, uint64_t ostride)
{
  const uint32_t t = xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const uint32_t k = t / G;
  if (k >= n) {
    return; // (whole subgroups: their shuffles stay inside the subgroup)
  }
  const int lane = int(t % G), sub0 = int(threadIdx.x & 63) & ~(G - 1);
  const uintptr_t xs = src + uint64_t(k / per) * gstride + uint64_t(k % per) * step;
  const uintptr_t hi = (xs + bytes - 1) & ~uintptr_t(15);
  const uintptr_t p0 = xs & ~uintptr_t(3);
  const uint32_t r = uint32_t(xs & 3);
  const uintptr_t dst = reinterpret_cast<uintptr_t>(out) + uint64_t(k) * ostride;
  const int nchunks = int((bytes + 15) >> 4);
  auto src_chunk = [&](int c, uint32_t& sel) {
    const uintptr_t p = p0 + 16 * uintptr_t(c);
    const uintptr_t q = p > hi ? hi : p;
    sel = uint32_t(p - q) >> 2;
    return u32x4(*reinterpret_cast<gdw4_ptr>(q));
  };
  for (int b0 = 0; b0 < nchunks; b0 += G * SU) {
    u32x4 X[SU + 1];
    uint32_t XS[SU + 1];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      X[u] = src_chunk(b0 + lane + G * u, XS[u]);
    }
    X[SU] = src_chunk(lane == 0 ? b0 + G * SU : b0 + lane + G * (SU - 1), XS[SU]);
    realign(X[0], XS[0]);
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      realign(X[u + 1], XS[u + 1]);
      const uint32_t d4 = next_dword<G>(X[u].x, X[u + 1].x, lane, sub0);
      const int c = b0 + lane + G * u;
      if (c >= nchunks) {
        continue;
      }
      const u32x4 a = X[u];
      u32x4 v;
      v.x = __builtin_amdgcn_alignbyte(a.y, a.x, r);
      v.y = __builtin_amdgcn_alignbyte(a.z, a.y, r);
      v.z = __builtin_amdgcn_alignbyte(a.w, a.z, r);
      v.w = __builtin_amdgcn_alignbyte(d4, a.w, r);
      if (uint32_t(16 * c + 16) > bytes) {
        v = keep_bytes(v, int(bytes) - 16 * c);
      }
      store_chunk(dst + 16 * uintptr_t(c), v);
    }
  }
}

} // namespace seg

thread_local char last_error[160] = "";

int
status_of(hipError_t e)
{
  if (e != hipSuccess) {
    snprintf(last_error, sizeof(last_error), "%s (%d): %s", hipGetErrorName(e), int(e),
             hipGetErrorString(e));
  }
  switch (e) {
    case hipSuccess:
      return TULIPS_STATUS_OK;
    case hipErrorOutOfMemory:
      return TULIPS_STATUS_NO_MORE_RESOURCES;
    case hipErrorInvalidValue:
      return TULIPS_STATUS_INVALID_ARGUMENT;
    default:
      return TULIPS_STATUS_HARDWARE_ERROR;
  }
}

} // namespace
} // namespace tulips_bench

using namespace tulips_bench;

extern "C" {

int
tulips_csum_gpu_sleep(uint32_t us, void* stream)
{
  if (us > 1000000u) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL(gpu_sleep_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream),
                     uint64_t(us) * 100u);
  return status_of(hipGetLastError());
}

int
tulips_csum_fill_splitmix(uint8_t* dst, uint64_t nbytes, uint64_t seed,
                          uint64_t byte_off, void* stream)
{
  if (nbytes && !dst) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return status_of(launch_fill_splitmix(dst, nbytes, seed, byte_off,
                                        static_cast<hipStream_t>(stream)));
}

int
tulips_csum_stream_read(const uint8_t* p, uint64_t nbytes, uint32_t* sink,
                        uint32_t max_blocks, void* stream)
{
  if ((nbytes && (!p || !sink)) || (reinterpret_cast<uintptr_t>(p) & 15)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return status_of(launch_stream_read(p, nbytes, sink, max_blocks,
                                      static_cast<hipStream_t>(stream)));
}

int
tulips_csum_stream_read_tiles(const uint8_t* p, uint64_t tile_bytes, uint32_t ntiles,
                              uint32_t* sink, void* stream)
{
  if (ntiles && (!p || !sink || tile_bytes == 0 || tile_bytes > TULIPS_CSUM_MAX_SEGMENT)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return status_of(
    launch_stream_tiles(p, tile_bytes, ntiles, sink, static_cast<hipStream_t>(stream)));
}

int
tulips_csum_stream_read_slots(const uint8_t* p, uint64_t slot_bytes, uint32_t read_bytes,
                              uint32_t nslots, uint32_t* sink, void* stream)
{
  if (nslots && (!p || !sink || read_bytes == 0 || read_bytes > TULIPS_CSUM_MAX_SEGMENT ||
                 slot_bytes < read_bytes)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return status_of(launch_stream_slots(p, slot_bytes, read_bytes, nslots, 16, 6, sink,
                                       static_cast<hipStream_t>(stream)));
}

int
tulips_csum_stream_read_slots_geom(const uint8_t* p, uint64_t slot_bytes, uint32_t read_bytes,
                                   uint32_t nslots, int group, int unroll, uint32_t* sink,
                                   void* stream)
{
  const bool geom = (group == 16 && unroll == 6) || (group == 32 && unroll == 3);
  if (!geom || (nslots && (!p || !sink || read_bytes == 0 ||
                           read_bytes > TULIPS_CSUM_MAX_SEGMENT || slot_bytes < read_bytes))) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return status_of(launch_stream_slots(p, slot_bytes, read_bytes, nslots, group, unroll, sink,
                                       static_cast<hipStream_t>(stream)));
}

int
tulips_csum_stream_copy_slots(const uint8_t* src, uint64_t group_stride, uint32_t per_group,
                              uint32_t step, uint32_t bytes, uint32_t nslots, uint8_t* out,
                              uint64_t out_stride, void* stream)
{
  if (nslots == 0) {
    return TULIPS_STATUS_OK;
  }
  if (!src || !out || per_group == 0 || bytes == 0 || bytes > 0xffffu ||
      (reinterpret_cast<uintptr_t>(out) & 15) || (out_stride & 15) || out_stride < bytes) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  constexpr int G = 16, SU = 6;
  const uint64_t blocks = (uint64_t(nslots) * G + 255) / 256;
  if (blocks > 0xffffffffull) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL((seg::copy_slots_kernel<G, SU>), dim3(uint32_t(blocks)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), reinterpret_cast<uintptr_t>(src),
                     group_stride, per_group, step, bytes, nslots, out, out_stride);
  return hipGetLastError() == hipSuccess ? TULIPS_STATUS_OK : TULIPS_STATUS_HARDWARE_ERROR;
}

} // extern "C"
