// Probe: round-trip latency of a GPU load from page-locked host memory, by
// allocation flags, measured inside one kernel with s_memrealtime (100 MHz):
// relaxed/acquire system-scope loads, 200 dependent loads each.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <vector>

template<int ORDER>
__global__ void
lat_kernel(uint64_t* p, uint64_t* ticks, int reps)
{
  if (threadIdx.x != 0) {
    return;
  }
  uint64_t acc = 0;
  for (int i = 0; i < reps; ++i) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t v = __hip_atomic_load(p + (acc & 1), ORDER, __HIP_MEMORY_SCOPE_SYSTEM);
    acc += v;
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime() + (acc & 0);
    ticks[i] = t1 - t0;
  }
  ticks[reps] = acc;
}

int
main()
{
  struct Case { const char* name; unsigned flags; };
  Case cases[] = { { "default (0)", 0u },
                   { "Mapped", hipHostMallocMapped },
                   { "Coherent|Mapped", hipHostMallocCoherent | hipHostMallocMapped },
                   { "NonCoherent|Mapped", hipHostMallocNonCoherent | hipHostMallocMapped } };
  const int reps = 200;
  uint64_t* dticks = nullptr;
  if (hipMalloc(&dticks, (reps + 1) * 8) != hipSuccess) {
    return 1;
  }
  std::vector<uint64_t> t(reps + 1);
  for (auto& c : cases) {
    uint64_t* h = nullptr;
    if (hipHostMalloc(&h, 4096, c.flags) != hipSuccess) {
      printf("%s: alloc failed\n", c.name);
      continue;
    }
    memset(h, 0, 4096);
    for (int order = 0; order < 2; ++order) {
      for (int round = 0; round < 2; ++round) {
        if (order == 0) {
          hipLaunchKernelGGL(lat_kernel<__ATOMIC_RELAXED>, dim3(1), dim3(64), 0, 0, h, dticks,
                             reps);
        } else {
          hipLaunchKernelGGL(lat_kernel<__ATOMIC_ACQUIRE>, dim3(1), dim3(64), 0, 0, h, dticks,
                             reps);
        }
        if (hipMemcpy(t.data(), dticks, (reps + 1) * 8, hipMemcpyDeviceToHost) != hipSuccess) {
          return 1;
        }
        std::vector<uint64_t> v(t.begin(), t.begin() + reps);
        std::sort(v.begin(), v.end());
        printf("%-22s %-8s round %d: load round trip median %.2f us, min %.2f, p90 %.2f\n",
               c.name, order ? "acquire" : "relaxed", round, v[reps / 2] / 100.0,
               v[0] / 100.0, v[reps * 9 / 10] / 100.0);
      }
    }
    (void)hipHostFree(h);
  }
  return 0;
}
