// rss_route.h — launchers of the flow router (rss_route.hip) for
// tulips_csum_mctx_validate_frames_rss_device (csum_multi.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace tulips_amd {

constexpr uint32_t RT_MAX_DEV = 64; // = the mctx device limit

struct RouteWindows
{
  uint32_t w[96]; // the key's 32-bit window at each tuple bit (rss_common.h)
};

// Per device, where its packed run starts in the source's gather buffer.
struct RouteStarts
{
  uint64_t at[RT_MAX_DEV];
};

bool rss_route_windows(const uint8_t* key, size_t key_len, RouteWindows* out);
uint32_t rss_route_blocks(uint32_t n);

// route + scan: dev_of[n]; blk_cnt / blk_bytes / base_cnt / base_bytes
// [rss_route_blocks(n) * nd]; totals[2 * nd] = frames then packed bytes
// per device. `table` is a device array of table_len entries < nd.
hipError_t launch_rss_route(const RouteWindows& win, const uint8_t* base, const uint64_t* offs,
                            const uint16_t* lens, uint32_t n, const uint16_t* table,
                            uint32_t table_len, uint32_t init, uint32_t nd, uint16_t* dev_of,
                            uint32_t* blk_cnt, uint32_t* blk_bytes, uint32_t* base_cnt,
                            uint64_t* base_bytes, uint64_t* totals, hipStream_t st);
// perm / poff / plen [n] in device-major, arrival order; poff = the source
// offset for frames of `home`, else the packed offset within its device's run
hipError_t launch_rss_scatter(const uint64_t* offs, const uint16_t* lens, uint32_t n, uint32_t nd,
                              uint32_t home, const uint16_t* dev_of, const uint32_t* base_cnt,
                              const uint64_t* base_bytes, const uint64_t* totals, uint32_t* perm,
                              uint64_t* poff, uint16_t* plen, hipStream_t st);
hipError_t launch_rss_gather(const uint8_t* base, const uint64_t* offs, uint32_t n, uint32_t home,
                             const uint16_t* dev_of, const uint32_t* perm, const uint64_t* poff,
                             const uint16_t* plen, const RouteStarts& starts, uint8_t* packed,
                             hipStream_t st);
// counters (nullable) zeroed then summed from the flags; flags (nullable)
hipError_t launch_rss_home(const uint32_t* perm, const uint8_t* rflags, uint32_t n,
                           uint8_t* flags, uint32_t* counters, hipStream_t st);

} // namespace tulips_amd
