// span_early.hip — A/B builds of the span kernel (span_kernel.h) for the ZIPF
// serial launch: compare-and-swap + re-zero words against
// one exchange per part (XCHG, the product since r03), and the exchange form
// at 24 and 32 KiB ranges; stamped launches with a data-arrival mark.
// Measured here before and not kept (profiles/probe_span_early_r03.txt):
// EARLY, the crossing segments' parts sent from rows loaded first
// (tools/variants/span_early_r03.patch), and raised issue priority until the
// window (and first rows) are issued (s_setprio). Measurement only (tools/probes/span_early.py); built with
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared \
//     -o tools/probes/libspan_early.so tools/probes/span_early.hip
#include "../../tulips_amd/csrc/span_kernel.h"

namespace tulips_amd {
namespace {

template<int U, int MH, bool X>
void
launch_e(const SpanArgs& sp, uint32_t grid, hipStream_t st)
{
  hipLaunchKernelGGL((csum_span_kernel<U, NoProbe, 8, 1024, MH, X>), dim3(grid), dim3(256), 0,
                     st, sp, NoProbe{});
}

// per-wave realtime stamps at the kernel's marks (as span_stamps.hip)
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

template<bool X>
void
launch_s(const SpanArgs& sp, uint32_t grid, uint64_t* stamps, hipStream_t st)
{
  hipLaunchKernelGGL((csum_span_kernel<7, EStampProbe, 8, 1024, 2, X>), dim3(grid), dim3(256),
                     0, st, sp, EStampProbe{stamps});
}

} // namespace
} // namespace tulips_amd

// Stamped launches of variants 0, 1 (U = 7): `stamps` holds
// ranges * 4 waves * 8 uint64 (marks 0-5, 7).
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

// variant: 0 compare-and-swap + re-zero (the r03f product), 1 exchange (the
// product since), 2 exchange U 6, 3 exchange U 8, all MH = U / 3. `mode` as the library's (RAW/INET/TCP |
// COMPLEMENT); src/dst for TCP.
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
  case 0: launch_e<7, 2, false>(sp, g, st); break;
  case 1: launch_e<7, 2, true>(sp, g, st); break;
  case 2: launch_e<6, 2, true>(sp, g, st); break;
  case 3: launch_e<8, 2, true>(sp, g, st); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
