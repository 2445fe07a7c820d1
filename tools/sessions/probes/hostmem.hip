// Probe: can a kernel on gfx950 read and write page-locked host memory
// directly (zero-copy), and does a host spin see its stores? Each case has
// a 2 s limit on the host side.
#include <hip/hip_runtime.h>
#include <chrono>
#include <stdio.h>
#include <stdint.h>
#include <string.h>

__global__ void
write_kernel(uint64_t* p, uint64_t v)
{
  if (threadIdx.x == 0) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void
copy_kernel(const uint64_t* src, uint64_t* dst)
{
  if (threadIdx.x == 0) {
    const uint64_t v = __hip_atomic_load(src, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dst, v + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static bool
wait_value(volatile uint64_t* p, uint64_t v, hipStream_t s, const char* what)
{
  auto t0 = std::chrono::steady_clock::now();
  while (__atomic_load_n(p, __ATOMIC_ACQUIRE) != v) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
      printf("%-40s TIMEOUT (value %llu, query %d)\n", what, (unsigned long long)*p,
             int(hipStreamQuery(s)));
      fflush(stdout);
      return false;
    }
  }
  auto us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0);
  printf("%-40s ok in %.1f us (query %d)\n", what, us.count(), int(hipStreamQuery(s)));
  fflush(stdout);
  return true;
}

int
main()
{
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  struct Case { const char* name; unsigned flags; };
  Case cases[] = { { "hipHostMalloc default", 0u },
                   { "hipHostMalloc Mapped", hipHostMallocMapped },
                   { "hipHostMalloc Coherent|Mapped", hipHostMallocCoherent | hipHostMallocMapped },
                   { "hipHostMalloc NonCoherent|Mapped",
                     hipHostMallocNonCoherent | hipHostMallocMapped } };
  for (auto& c : cases) {
    uint64_t* h = nullptr;
    if (hipHostMalloc(&h, 4096, c.flags) != hipSuccess) {
      printf("%-40s alloc failed\n", c.name);
      continue;
    }
    memset(h, 0, 4096);
    void* d = nullptr;
    hipHostGetDevicePointer(&d, h, 0);
    printf("%s: host %p dev %p\n", c.name, (void*)h, d);
    hipLaunchKernelGGL(write_kernel, dim3(1), dim3(64), 0, s, (uint64_t*)d, 42ull);
    printf("  launch: %s\n", hipGetErrorString(hipGetLastError()));
    if (!wait_value(h, 42, s, "  kernel store seen by host spin")) {
      return 1;
    }
    hipStreamSynchronize(s);
    h[8] = 77;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    hipLaunchKernelGGL(copy_kernel, dim3(1), dim3(64), 0, s, (uint64_t*)d + 8,
                       (uint64_t*)d + 16);
    if (!wait_value(h + 16, 78, s, "  kernel load of host value")) {
      return 1;
    }
    hipStreamSynchronize(s);
    // launch latency: 20 write kernels, host spin on each
    double tot = 0;
    for (int i = 0; i < 20; ++i) {
      auto t0 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(write_kernel, dim3(1), dim3(64), 0, s, (uint64_t*)d, 100ull + i);
      while (__atomic_load_n(h, __ATOMIC_ACQUIRE) != 100ull + i) {
      }
      tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
               .count();
    }
    printf("  launch + store seen: %.1f us mean of 20\n", tot / 20);
    hipStreamSynchronize(s);
    hipHostFree(h);
  }
  return 0;
}
