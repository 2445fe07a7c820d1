// seg_device.h — the chunk-movement primitives of the segmentation kernels
// (segment.hip), shared with the copy-ceiling kernel of the measurement
// library (benchlib/csrc/bench_kernels.hip), which must move bytes exactly
// as the segment builders do.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "frame_common.h"

namespace tulips_amd {
namespace frame {

typedef __attribute__((address_space(1))) u32x4* gchunk_wptr;

// Output chunks are written once and read next by the NIC, not by this GPU:
// nontemporal stores stream them out instead of leaving ~68 MB per call dirty
// in L2 for the kernel boundary to write back (per call 41.0 -> 31.5 us in
// bench.py's serial chain, 30.0 -> 23.4 us on 4 branches; the kernel's own
// duration is unchanged).
__device__ __forceinline__ void
store_chunk(uintptr_t a, u32x4 v)
{
  __builtin_nontemporal_store(v, reinterpret_cast<gchunk_wptr>(a));
}

__device__ __forceinline__ u32x4
keep_bytes(u32x4 a, int k)
{
  u32x4 v;
  v.x = a.x & byte_mask(0, k, 0);
  v.y = a.y & byte_mask(0, k, 4);
  v.z = a.z & byte_mask(0, k, 8);
  v.w = a.w & byte_mask(0, k, 12);
  return v;
}

// The dword after each lane's chunk: lane l + 1's first dword, the next batch
// slot's for the subgroup's last lane (lane 0 hands it nxt).
template<int G>
__device__ __forceinline__ uint32_t
next_dword(uint32_t cur, uint32_t nxt, int lane, int sub0)
{
  const uint32_t give = lane == 0 ? nxt : cur;
  if constexpr (G == 16) {
    // a 16-lane subgroup is one DPP row: row_ror:15 hands lane l the value of
    // lane (l + 1) mod 16 in one VALU move
    return uint32_t(__builtin_amdgcn_update_dpp(0, int(give), 0x12F, 0xF, 0xF, false));
  } else {
    return __shfl(give, sub0 + ((lane + 1) & (G - 1)), 64);
  }
}

typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef const __attribute__((address_space(1))) u32x4_a4* gdw4_ptr;

// A payload chunk whose dwords start past the frame's last aligned chunk is
// loaded from that chunk instead (reads never leave the 16-byte chunks the
// frame touches), sel dwords early: move its dwords down. Dwords that would
// come from beyond that chunk lie past the frame and are never used.
__device__ __forceinline__ void
realign(u32x4& d, uint32_t sel)
{
  if (sel != 0) {
    const u32x4 e = d;
    d.x = sel == 1 ? e.y : (sel == 2 ? e.z : e.w);
    d.y = sel == 1 ? e.z : e.w;
    d.z = e.w;
  }
}

} // namespace frame
} // namespace tulips_amd
