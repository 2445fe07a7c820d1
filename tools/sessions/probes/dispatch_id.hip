// Probe: is the AQL dispatch id (llvm.amdgcn.dispatch.id) filled in on
// gfx950, distinct per launch on one stream, across streams and across
// replays of one HIP graph? (Candidate per-launch tag for the arena
// kernel's split words.)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

extern "C" __device__ uint64_t dispatch_id_intrinsic() __asm("llvm.amdgcn.dispatch.id");

__global__ void
did_kernel(uint64_t* out, int slot)
{
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[slot] = dispatch_id_intrinsic();
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int
main()
{
  uint64_t* d = nullptr;
  CK(hipMalloc(&d, 64 * sizeof(uint64_t)));
  CK(hipMemset(d, 0xff, 64 * sizeof(uint64_t)));
  hipStream_t s1, s2;
  CK(hipStreamCreate(&s1));
  CK(hipStreamCreate(&s2));
  for (int i = 0; i < 4; ++i) {
    hipLaunchKernelGGL(did_kernel, dim3(1), dim3(64), 0, s1, d, i);
  }
  for (int i = 0; i < 4; ++i) {
    hipLaunchKernelGGL(did_kernel, dim3(1), dim3(64), 0, s2, d, 4 + i);
  }
  CK(hipDeviceSynchronize());
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
  hipLaunchKernelGGL(did_kernel, dim3(1), dim3(64), 0, s1, d, 8);
  CK(hipStreamEndCapture(s1, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  uint64_t h[64];
  for (int r = 0; r < 3; ++r) {
    CK(hipGraphLaunch(ge, s1));
    CK(hipStreamSynchronize(s1));
    CK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
    printf("graph replay %d: dispatch id %llu\n", r, (unsigned long long)h[8]);
  }
  for (int i = 0; i < 8; ++i) {
    printf("%s launch %d: dispatch id %llu\n", i < 4 ? "s1" : "s2", i % 4,
           (unsigned long long)h[i]);
  }
  return 0;
}
