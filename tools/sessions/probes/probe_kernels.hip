// probe_kernels.hip — diagnostic kernels (tuning tool, not product code).
// Plain streaming read of [base, base+nbytes) in 8 KiB wave tiles, optionally
// followed by one u16 store per `store_every` bytes read (store_mode 0 = none,
// 1 = plain, 2 = nontemporal), to price what output stores add to a launch.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4* gptr;

__global__ __launch_bounds__(256) void
read_store(uintptr_t base, uint64_t nchunks, uint16_t* out, uint64_t nout,
           int store_mode)
{
  constexpr int U = 8;
  const gptr p = reinterpret_cast<gptr>(base);
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = (uint64_t(gridDim.x) * blockDim.x) >> 6;
  const uint64_t ntiles = nchunks / (64 * U);
  uint32_t x = 0;
  for (uint64_t t = wave; t < ntiles; t += nwaves) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u] = __builtin_nontemporal_load(p + t * (64 * U) + u * 64 + lane);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (store_mode) {
      // this tile's share of outputs: nout * tile / ntiles .. next
      const uint64_t o0 = nout * t / ntiles, o1 = nout * (t + 1) / ntiles;
      for (uint64_t o = o0 + lane; o < o1; o += 64) {
        if (store_mode == 1) {
          out[o] = uint16_t(x);
        } else {
          __builtin_nontemporal_store(uint16_t(x), out + o);
        }
      }
    }
  }
  if (x == 0x9e3779b9u) {
    out[0] = 1;
  }
}

extern "C" int
probe_read_store(const void* base, uint64_t nbytes, uint16_t* out, uint64_t nout,
                 int store_mode, uint32_t blocks, void* stream)
{
  hipLaunchKernelGGL(read_store, dim3(blocks), dim3(256), 0,
                     static_cast<hipStream_t>(stream),
                     reinterpret_cast<uintptr_t>(base), nbytes / 16, out, nout,
                     store_mode);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
