// occ_frames.hip — the product's frame kernels (validate / generate / fields,
// 16 lanes x 6 chunks) with dynamic LDS added to cap the workgroups per CU,
// i.e. the waves per SIMD below the 6 their registers allow. Measurement only
// (tools/probes/occ_frames.py); built with
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o tools/probes/libocc_frames.so \
//     tools/probes/occ_frames.hip -Ltulips_amd -ltulips_csum
#include "../../tulips_amd/csrc/frames.hip"

extern "C" int
occ_frames(int op, uint8_t* base, const uint64_t* offs, const uint16_t* lens, uint32_t n,
           uint8_t* flags, uint32_t* fields, uint32_t lds_bytes, void* stream)
{
  using namespace tulips_amd;
  const uint32_t blocks = (n + 15) / 16;
  const hipStream_t st = static_cast<hipStream_t>(stream);
  (void)hipGetLastError();
  switch (op) {
  case 0:
    hipLaunchKernelGGL((frame_kernel<0, 16, 6, true>), dim3(blocks), dim3(256), lds_bytes, st,
                       base, offs, lens, n, flags, nullptr, nullptr);
    break;
  case 1:
    hipLaunchKernelGGL((frame_kernel<1, 16, 6, true>), dim3(blocks), dim3(256), lds_bytes, st,
                       base, offs, lens, n, flags, nullptr, nullptr);
    break;
  default:
    hipLaunchKernelGGL((frame_kernel<2, 16, 6, true>), dim3(blocks), dim3(256), lds_bytes, st,
                       base, offs, lens, n, nullptr, nullptr, fields);
    break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
