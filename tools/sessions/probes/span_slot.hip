// span_slot.hip — A/B builds of the span kernel (span_kernel.h) for the ZIPF
// serial launch: the product split form (boundary chunks
// loaded by the entry holders between the range's first rows and the rest)
// against the boundary-slot split form (csum_span_slot_kernel: every row
// issued with the window, boundary chunks handed over in LDS by their
// owners). Same exports as span_early.hip, so tools/probes/span_early.py
// drives it (SPAN_LIB=libspan_slot.so). Measured slower and not kept: the
// kernel lives in tools/variants/span_slot_r03.patch (apply it to
// tulips_amd/csrc/span_kernel.h to rebuild). Measurement only; built with
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared \
//     -o tools/probes/libspan_slot.so tools/probes/span_slot.hip
#include "../../tulips_amd/csrc/span_kernel.h"

namespace tulips_amd {
namespace {

template<int U, bool SLOT>
void
launch_e(const SpanArgs& sp, uint32_t grid, hipStream_t st)
{
  if constexpr (SLOT) {
    hipLaunchKernelGGL((csum_span_slot_kernel<U>), dim3(grid), dim3(256), 0, st, sp, NoProbe{});
  } else {
    hipLaunchKernelGGL((csum_span_kernel<U>), dim3(grid), dim3(256), 0, st, sp, NoProbe{});
  }
}

struct EStampProbe
{
  static constexpr int stop = 0;
  static constexpr bool data_mark = true;
  uint64_t* buf;
  __device__ __forceinline__ void keep(uint32_t) const {}
  __device__ __forceinline__ void mark(uint32_t k, uint32_t w, uint32_t lane, int point) const
  {
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
      buf[(uint64_t(k) * 4u + w) * 8u + point] = t;
    }
  }
};

template<bool SLOT>
void
launch_s(const SpanArgs& sp, uint32_t grid, uint64_t* stamps, hipStream_t st)
{
  if constexpr (SLOT) {
    hipLaunchKernelGGL((csum_span_slot_kernel<7, EStampProbe>), dim3(grid), dim3(256), 0, st, sp,
                       EStampProbe{stamps});
  } else {
    hipLaunchKernelGGL((csum_span_kernel<7, EStampProbe>), dim3(grid), dim3(256), 0, st, sp,
                       EStampProbe{stamps});
  }
}

} // namespace
} // namespace tulips_amd

// Stamped launches of variants 0 (product), 1 (slot), U = 7.
extern "C" int
span_early_stamped(const uint8_t* base, uint64_t arena, const uint64_t* offs,
                   const uint16_t* lens, uint16_t* out, uint32_t n, uint64_t* slots,
                   uint64_t nslots, uint32_t salt, uint32_t variant, uint64_t* stamps,
                   void* stream)
{
  using namespace tulips_amd;
  const uint64_t ranges = span_ranges(base, arena, 4096ull * 7);
  if (n == 0 || ranges > nslots) {
    return 1;
  }
  SpanArgs sp{base, arena, offs, lens, nullptr, nullptr, nullptr, out, nullptr,
              n, 0u, 0u, slots, nslots, salt, 0};
  const hipStream_t st = static_cast<hipStream_t>(stream);
  (void)hipGetLastError();
  switch (variant) {
  case 0: launch_s<false>(sp, uint32_t(ranges), stamps, st); break;
  case 1: launch_s<true>(sp, uint32_t(ranges), stamps, st); break;
  default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// variant: 0 product U 7, 1 slot U 7, 2 slot U 6, 3 slot U 8
extern "C" int
span_early_launch(const uint8_t* base, uint64_t arena, const uint64_t* offs,
                  const uint16_t* lens, const uint32_t* src, const uint32_t* dst, uint16_t* out,
                  uint32_t n, uint32_t mode, uint64_t* slots, uint64_t nslots, uint32_t salt,
                  uint32_t variant, void* stream)
{
  using namespace tulips_amd;
  static const uint32_t us[4] = {7, 7, 6, 8};
  if (variant >= 4) {
    return 1;
  }
  const uint64_t ranges = span_ranges(base, arena, 4096ull * us[variant]);
  if (n == 0 || ranges > nslots) {
    return 1;
  }
  SpanArgs sp{base, arena, offs, lens, nullptr, src, dst, out, nullptr,
              n, mode, 0u, slots, nslots, salt, 0};
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const uint32_t g = uint32_t(ranges);
  (void)hipGetLastError();
  switch (variant) {
  case 0: launch_e<7, false>(sp, g, st); break;
  case 1: launch_e<7, true>(sp, g, st); break;
  case 2: launch_e<6, true>(sp, g, st); break;
  case 3: launch_e<8, true>(sp, g, st); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
