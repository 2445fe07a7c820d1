// occ_probe.hip — F1500 through the product's csum_kernel<32, 4> with
// dynamic LDS added to cap the workgroups per CU (waves per SIMD), to see
// whether fewer resident waves stream a single launch faster (the frame
// kernels ran slower at 7 waves per SIMD than at 6). Measurement only
// (tools/probes/occ_probe.py); built with
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o tools/probes/libocc_probe.so \
//     tools/probes/occ_probe.hip -Ltulips_amd -ltulips_csum
#include "../../tulips_amd/csrc/csum_kernels.hip"

extern "C" int
occ_launch(const uint8_t* base, uint16_t* out, uint32_t n, uint32_t lds_bytes, void* stream)
{
  using namespace tulips_amd;
  const FixedSegs segs{base, 1500, 1500};
  const uint32_t blocks = (n + 7) / 8;
  (void)hipGetLastError();
  hipLaunchKernelGGL((csum_kernel<32, 4, true, FixedSegs>), dim3(blocks), dim3(256), lds_bytes,
                     static_cast<hipStream_t>(stream), segs, nullptr, nullptr, nullptr, out,
                     nullptr, n, 0u, false);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
