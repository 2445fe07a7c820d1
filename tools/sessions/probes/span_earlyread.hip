// span_earlyread.hip — A/B of the span kernel's EARLY option for the ZIPF
// launch: the holder of a two-part segment reads the segment's word behind
// the range's last rows, so a partner part published before this range's
// data arrived is in hand without an exchange round trip after the data.
// Same exports as span_early.hip; tools/probes/span_early.py drives it
// (SPAN_LIB=libspan_earlyread.so STAMPS=0). Measured slower, not kept: needs
// tools/variants/span_earlyread_r03.patch applied. Measurement only; built with
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared \
//     -o tools/probes/libspan_earlyread.so tools/probes/span_earlyread.hip
#include "../../tulips_amd/csrc/span_kernel.h"

namespace tulips_amd {
namespace {

template<int U, bool E>
void
launch_e(const SpanArgs& sp, uint32_t grid, hipStream_t st)
{
  hipLaunchKernelGGL((csum_span_kernel<U, NoProbe, 8, 1024, U / 3, true, 256, E>), dim3(grid),
                     dim3(256), 0, st, sp, NoProbe{});
}

} // namespace
} // namespace tulips_amd

extern "C" int
span_early_stamped(const uint8_t*, uint64_t, const uint64_t*, const uint16_t*, uint16_t*,
                   uint32_t, uint64_t*, uint64_t, uint32_t, uint32_t, uint64_t*, void*)
{
  return 1;
}

// variant: 0 product (U 7), 1 EARLY U 7, 2 EARLY U 6, 3 EARLY U 8
extern "C" int
span_early_launch(const uint8_t* base, uint64_t arena, const uint64_t* offs,
                  const uint16_t* lens, const uint32_t* src, const uint32_t* dst, uint16_t* out,
                  uint32_t n, uint32_t mode, uint64_t* slots, uint64_t nslots, uint32_t salt,
                  uint32_t variant, void* stream)
{
  using namespace tulips_amd;
  static const uint64_t wb[4] = {16ull * 256 * 7, 16ull * 256 * 7, 16ull * 256 * 6,
                                 16ull * 256 * 8};
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
  case 0: launch_e<7, false>(sp, g, st); break;
  case 1: launch_e<7, true>(sp, g, st); break;
  case 2: launch_e<6, true>(sp, g, st); break;
  case 3: launch_e<8, true>(sp, g, st); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
