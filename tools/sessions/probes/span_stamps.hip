// span_stamps.hip — the product span kernel (tulips_amd/csrc/span_kernel.h)
// instantiated for measurement:
//   * with a probe that records, per wave, the realtime clock (100 MHz) at
//     the kernel's marks: 0 start, 1 window + range loads issued, 2 window
//     counted (first barrier), 3 range scanned (data arrived, second
//     barrier), 4 in-range results stored, 5 end (split parts sent,
//     finisher's result stored), 7 rare path entered; slot 6 holds the
//     wave's XCC id;
//   * without stamps at other XCD run lengths (XC) and window sizes (NWIN);
//   * read_shape_kernel: the kernel's loads alone (the window of NWIN
//     entries, then U = 6 chunks per thread of the range, same block order),
//     xor-reduced, to price the window's requests apart from everything else.
// Measurement only (tools/probes/span_stamps.py); not part of the product.
#include "../../tulips_amd/csrc/span_kernel.h"

namespace tulips_amd {
namespace {

struct StampProbe
{
  static constexpr int stop = 0;
  static constexpr bool data_mark = false;
  uint64_t* buf;
  __device__ __forceinline__ void keep(uint32_t) const {}
  __device__ __forceinline__ void mark(uint32_t k, uint32_t w, uint32_t lane, int point) const
  {
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
      uint64_t* row = buf + (uint64_t(k) * 4u + w) * 8u;
      row[point] = t;
      if (point == 0) {
        row[6] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((16 - 1) << 11)); // XCC_ID
      }
    }
  }
};

// Diagnostic builds of the product kernel: stop after phase STOP (1: loads
// and window, 2: + scans, 3: + results stored, no atomics), values kept live
// through a store that never happens.
template<int STOP>
struct DiagProbe
{
  static constexpr int stop = STOP;
  static constexpr bool data_mark = false;
  uint32_t* sink;
  __device__ __forceinline__ void mark(uint32_t, uint32_t, uint32_t, int) const {}
  __device__ __forceinline__ void keep(uint32_t x) const
  {
    if (x == 0x9e3779b9u) {
      sink[0] = x;
    }
  }
};

template<int STOP, int MH>
void
launch_diag(const SpanArgs& sp, uint32_t grid, uint32_t* sink, hipStream_t st)
{
  hipLaunchKernelGGL((csum_span_kernel<6, DiagProbe<STOP>, 8, 1024, MH>), dim3(grid),
                     dim3(256), 0, st, sp, DiagProbe<STOP>{sink});
}

template<uint32_t NWIN>
__global__ __launch_bounds__(256, 7) void
read_shape_kernel(SpanArgs p, uint32_t* sink)
{
  constexpr int U = 6;
  constexpr uint64_t W = 4096ull * U;
  constexpr int RW = NWIN / 256;
  const uint32_t t = threadIdx.x;
  const uint32_t k = xcd_block(blockIdx.x, gridDim.x);
  const uintptr_t b = reinterpret_cast<uintptr_t>(p.base);
  const uintptr_t A = b & ~uintptr_t(15);
  const uintptr_t x0 = A + uint64_t(k) * W;
  const uintptr_t last = (b + p.arena - 1) & ~uintptr_t(15);
  const uint32_t n = p.n;
  const gu64_ptr offs = reinterpret_cast<gu64_ptr>(reinterpret_cast<uintptr_t>(p.offs));
  const gu16_ptr lens = reinterpret_cast<gu16_ptr>(reinterpret_cast<uintptr_t>(p.lens));
  const uint64_t mid = uint64_t(k) * W + W / 2;
  const uint64_t guess = uint64_t(double(n) * double(mid) / double(p.arena));
  const uint32_t gmax = n > NWIN ? n - NWIN : 0u;
  const uint32_t G = uint32_t(min(guess > NWIN / 2 ? guess - NWIN / 2 : 0ull, uint64_t(gmax)));
  uint64_t acc = 0;
  if constexpr (RW > 0) {
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const uint32_t i = min(G + t + 256u * r, n - 1);
      acc += offs[i] + lens[i];
    }
  }
  u32x4 v[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    v[j] = load_chunk<false>(
      reinterpret_cast<gchunk_ptr>(min(x0 + 16u * (uint32_t(j) * 256u + t), last)));
  }
  uint32_t x = uint32_t(acc) ^ uint32_t(acc >> 32);
#pragma unroll
  for (int j = 0; j < U; ++j) {
    x ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  }
  if (x == 0x9e3779b9u) { // practically never; keeps the loads live
    sink[0] = x;
  }
}

template<int U, uint32_t XC, uint32_t NWIN, int MH>
void
launch_v(const SpanArgs& sp, uint32_t grid, uint64_t* stamps, hipStream_t st)
{
  if (stamps) {
    hipLaunchKernelGGL((csum_span_kernel<U, StampProbe, XC, NWIN, MH>), dim3(grid), dim3(256),
                       0, st, sp, StampProbe{stamps});
  } else {
    hipLaunchKernelGGL((csum_span_kernel<U, NoProbe, XC, NWIN, MH>), dim3(grid), dim3(256), 0,
                       st, sp, NoProbe{});
  }
}

} // namespace
} // namespace tulips_amd

// One launch of the product kernel with `u` chunks per lane, `xc` ranges per
// XCD run, an `nwin`-entry window and `mh` range chunks issued before the
// window is counted (6 / 8 / 1024 / 3 = the product default), with per-wave
// stamps when `stamps` is not NULL. `slots` must hold `ranges` zeroed words;
// `stamps` ranges * 4 * 8 uint64.
extern "C" int
span_probe_launch(const uint8_t* base, uint64_t arena, const uint64_t* offs,
                  const uint16_t* lens, uint16_t* out, uint32_t n, uint64_t* slots,
                  uint64_t nslots, uint32_t salt, uint64_t* stamps, uint32_t u, uint32_t xc,
                  uint32_t nwin, uint32_t mh, void* stream)
{
  using namespace tulips_amd;
  const uint64_t ranges = span_ranges(base, arena, 4096ull * u);
  if (n == 0 || arena == 0 || ranges > nslots) {
    return 1;
  }
  SpanArgs sp{base, arena, offs, lens, nullptr, nullptr, nullptr, out, nullptr,
              n, 0u, 0u, slots, nslots, salt, 0};
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const uint32_t g = uint32_t(ranges);
  (void)hipGetLastError();
  const uint32_t key = u * 1000000 + xc * 10000 + (nwin / 256) * 100 + mh;
  switch (key) {
  case 6080406: launch_v<6, 8, 1024, 6>(sp, g, stamps, st); break;
  case 6080403: launch_v<6, 8, 1024, 3>(sp, g, stamps, st); break;
  case 6080402: launch_v<6, 8, 1024, 2>(sp, g, stamps, st); break;
  case 7080402: launch_v<7, 8, 1024, 2>(sp, g, stamps, st); break;
  case 7080403: launch_v<7, 8, 1024, 3>(sp, g, stamps, st); break;
  case 7080404: launch_v<7, 8, 1024, 4>(sp, g, stamps, st); break;
  case 8080403: launch_v<8, 8, 1024, 3>(sp, g, stamps, st); break;
  case 8080404: launch_v<8, 8, 1024, 4>(sp, g, stamps, st); break;
  case 7080303: launch_v<7, 8, 768, 3>(sp, g, stamps, st); break;
  default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// The kernel's loads alone (window of `nwin` entries: 0, 256, 1024, 2048).
extern "C" int
read_shape_launch(const uint8_t* base, uint64_t arena, const uint64_t* offs,
                  const uint16_t* lens, uint32_t n, uint32_t nwin, uint32_t* sink, void* stream)
{
  using namespace tulips_amd;
  const uint64_t ranges = span_ranges(base, arena, 4096ull * 6);
  if (n < 2048 || arena == 0) {
    return 1;
  }
  SpanArgs sp{base, arena, offs, lens, nullptr, nullptr, nullptr, nullptr, nullptr,
              n, 0u, 0u, nullptr, 0, 0, 0};
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 grid{uint32_t(ranges), 1, 1};
  (void)hipGetLastError();
  switch (nwin) {
  case 0: hipLaunchKernelGGL((read_shape_kernel<0>), grid, dim3(256), 0, st, sp, sink); break;
  case 256: hipLaunchKernelGGL((read_shape_kernel<256>), grid, dim3(256), 0, st, sp, sink); break;
  case 1024:
    hipLaunchKernelGGL((read_shape_kernel<1024>), grid, dim3(256), 0, st, sp, sink);
    break;
  case 2048:
    hipLaunchKernelGGL((read_shape_kernel<2048>), grid, dim3(256), 0, st, sp, sink);
    break;
  default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// The product kernel (U = 6, `mh` 3 or 6) stopped after phase `stop` (1-3).
extern "C" int
span_diag_launch(const uint8_t* base, uint64_t arena, const uint64_t* offs,
                 const uint16_t* lens, uint16_t* out, uint32_t n, uint64_t* slots,
                 uint64_t nslots, uint32_t stop, uint32_t mh, uint32_t* sink, void* stream)
{
  using namespace tulips_amd;
  const uint64_t ranges = span_ranges(base, arena, 4096ull * 6);
  if (n == 0 || arena == 0 || ranges > nslots) {
    return 1;
  }
  SpanArgs sp{base, arena, offs, lens, nullptr, nullptr, nullptr, out, nullptr,
              n, 0u, 0u, slots, nslots, 0, 0};
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const uint32_t g = uint32_t(ranges);
  (void)hipGetLastError();
  const uint32_t key = stop * 10 + mh;
  switch (key) {
  case 13: launch_diag<1, 3>(sp, g, sink, st); break;
  case 16: launch_diag<1, 6>(sp, g, sink, st); break;
  case 23: launch_diag<2, 3>(sp, g, sink, st); break;
  case 26: launch_diag<2, 6>(sp, g, sink, st); break;
  case 33: launch_diag<3, 3>(sp, g, sink, st); break;
  case 36: launch_diag<3, 6>(sp, g, sink, st); break;
  default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" uint64_t
span_stamps_ranges(const uint8_t* base, uint64_t arena)
{
  return tulips_amd::span_ranges(base, arena, 4096ull * 6);
}
