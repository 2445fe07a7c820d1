// frames_slots.hip — the frame kernels in SLOTS mode (frame i at base + i *
// slot, chunk loads issued with the length load) for A/B against the
// offsets form on bench.py's frame workload. Needs tools/variants/frames_slots_r03.patch
// applied (measured equal, not kept). Measurement only
// (tools/probes/frames_slots.py); built with
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o tools/probes/libframes_slots.so \
//     tools/probes/frames_slots.hip -Ltulips_amd -ltulips_csum
#include "../../tulips_amd/csrc/frames.hip"

extern "C" int
frames_slots(int op, uint8_t* base, uint64_t slot, const uint16_t* lens, uint32_t n,
             uint8_t* flags, uint32_t* fields, void* stream)
{
  using namespace tulips_amd;
  const uint32_t blocks = (n + 15) / 16;
  const hipStream_t st = static_cast<hipStream_t>(stream);
  (void)hipGetLastError();
  switch (op) {
  case 0:
    hipLaunchKernelGGL((frame_kernel<0, 16, 6, true, true>), dim3(blocks), dim3(256), 0, st,
                       base, nullptr, lens, n, flags, nullptr, nullptr, slot);
    break;
  case 1:
    hipLaunchKernelGGL((frame_kernel<1, 16, 6, true, true>), dim3(blocks), dim3(256), 0, st,
                       base, nullptr, lens, n, flags, nullptr, nullptr, slot);
    break;
  default:
    hipLaunchKernelGGL((frame_kernel<2, 16, 6, true, true>), dim3(blocks), dim3(256), 0, st,
                       base, nullptr, lens, n, nullptr, nullptr, fields, slot);
    break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
