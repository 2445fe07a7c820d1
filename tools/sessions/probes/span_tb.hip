// span_tb.hip — A/B of the span kernel's workgroup size for the ZIPF launch
// (read traffic <= 1.04x, WRITE_SIZE <= 1.5x the results):
// the product's 256-thread workgroups over 28 KiB ranges against 512 and
// 1024-thread workgroups over proportionally longer ranges (one offsets
// window and at most two split words per range, so fewer of both per byte).
// Same exports as span_early.hip; tools/probes/span_early.py drives it
// (SPAN_LIB=libspan_tb.so STAMPS=0). Measurement only; built with
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared \
//     -o tools/probes/libspan_tb.so tools/probes/span_tb.hip
#include "../../tulips_amd/csrc/span_kernel.h"

namespace tulips_amd {
namespace {

template<int U, uint32_t TB>
void
launch_e(const SpanArgs& sp, uint32_t grid, hipStream_t st)
{
  hipLaunchKernelGGL((csum_span_kernel<U, NoProbe, 8, 1024, U / 3, true, TB>), dim3(grid),
                     dim3(TB), 0, st, sp, NoProbe{});
}

} // namespace
} // namespace tulips_amd

extern "C" int
span_early_stamped(const uint8_t*, uint64_t, const uint64_t*, const uint16_t*, uint16_t*,
                   uint32_t, uint64_t*, uint64_t, uint32_t, uint32_t, uint64_t*, void*)
{
  return 1;
}

// variant: 0 product (256 threads, U 7: 28 KiB), 1 512 threads U 7 (56 KiB),
// 2 512 threads U 6 (48 KiB), 3 1024 threads U 4 (64 KiB)
extern "C" int
span_early_launch(const uint8_t* base, uint64_t arena, const uint64_t* offs,
                  const uint16_t* lens, const uint32_t* src, const uint32_t* dst, uint16_t* out,
                  uint32_t n, uint32_t mode, uint64_t* slots, uint64_t nslots, uint32_t salt,
                  uint32_t variant, void* stream)
{
  using namespace tulips_amd;
  static const uint64_t wb[4] = {16ull * 256 * 7, 16ull * 512 * 7, 16ull * 512 * 6,
                                 16ull * 1024 * 4};
  if (variant >= 4) {
    return 1;
  }
  const uint64_t ranges = span_ranges(base, arena, wb[variant]);
  if (n == 0 || ranges > nslots) {
    return 1;
  }
  SpanArgs sp{base, arena, offs, lens, nullptr, src, dst, out, nullptr,
              n, mode, 0u, slots, nslots, salt, 0};
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const uint32_t g = uint32_t(ranges);
  (void)hipGetLastError();
  switch (variant) {
  case 0: launch_e<7, 256>(sp, g, st); break;
  case 1: launch_e<7, 512>(sp, g, st); break;
  case 2: launch_e<6, 512>(sp, g, st); break;
  case 3: launch_e<4, 1024>(sp, g, st); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
