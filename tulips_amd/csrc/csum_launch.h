// csum_launch.h — internal launcher interface between the C ABI
// (csum_capi.hip) and the kernels (csum_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tulips_amd {

// The calling thread's stream-capture mode, relaxed for the guard's scope.
// In global mode (the default) a hipMalloc, hipFree or hipStreamSynchronize
// from any thread invalidates every other thread's global-mode capture
// (tools/probe_capture_modes.py, profiles/capture_modes_r06o.jsonl); the
// library's own allocations, frees and waits never touch such a capture, so
// they are made relaxed.
struct RelaxedCapture
{
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  RelaxedCapture() { (void)hipThreadExchangeStreamCaptureMode(&mode); }
  ~RelaxedCapture() { (void)hipThreadExchangeStreamCaptureMode(&mode); }
  RelaxedCapture(const RelaxedCapture&) = delete;
  RelaxedCapture& operator=(const RelaxedCapture&) = delete;
};

struct LaunchArgs
{
  const uint16_t* seeds; // nullable
  const uint32_t* src;   // TCP only
  const uint32_t* dst;   // TCP only
  uint16_t* out;         // nullable when only counting
  uint32_t* bad;         // nullable: counter shards (stream_state.h) that
                         // results != 0xffff are counted into
  uint32_t n;
  uint32_t mode;
  int kind;              // TULIPS_CSUM_KIND_* (never DEFAULT here)
  int group;             // lanes per segment / short subgroup / segs per wave
  int unroll;            // chunks in flight per lane: 2, 4, 8
  bool nontemporal;      // nt loads
  bool nt_store;         // nt (streaming) result stores
  uint32_t max_blocks;   // grid cap (0 = one subgroup per segment)
  int block;             // threads per workgroup: 256, 512, 1024 (0 = 256)
  int spw;               // packed: 2 = double-buffered windows
  uint64_t offs_bias;    // span: segment i starts at base + offs[i] - offs_bias
};

// Counter shards: CNT_SHARDS zeroed 128-B lines per (device,
// stream), counter k of a block's shard at shards[CNT_LINE * shard + k].
// Kernels add per-block totals to their shard; launch_counters_finalize
// writes the sums of counters 0..nout-1 to `out` and zeroes the shards again.
// Spreading the adds keeps same-address device atomics (~11 ns each,
// serialised) off the critical path.
// The shards come from the stream's state (stream_state.h call_shards).
constexpr uint32_t CNT_SHARDS = 32, CNT_LINE = 32;
hipError_t launch_counters_finalize(uint32_t* shards, uint32_t* out, uint32_t nout,
                                    hipStream_t stream);

hipError_t launch_fixed(const uint8_t* base, uint64_t stride, uint32_t len,
                        const LaunchArgs& a, hipStream_t stream);
hipError_t launch_var(const uint8_t* base, const uint64_t* offs,
                      const uint16_t* lens, const LaunchArgs& a,
                      hipStream_t stream);
// Whether launch_span has a kernel for (unroll, group) (checked on the CPU
// before any HIP call).
bool span_geometry_ok(int unroll, int group);
// Chunks per lane of the default arena geometry: 28 KiB per workgroup range
// (tools/sessions/probes/span_stamps.py, profiles/probe_span_geometry_r03.txt: ZIPF
// 11.3 us serial and 7.8 us per launch on 4 branches, against 11.5 / 8.0 at
// 6 and 11.6 / 8.0 at 8).
constexpr int SPAN_DEFAULT_UNROLL = 7;
// In-order arena (KIND_SPAN): segments lie in order in [base, base + arena);
// a.unroll = chunks per lane (4 KiB of arena per workgroup each), a.group the
// form (include/tulips_csum.h).
hipError_t launch_span(const uint8_t* base, uint64_t arena, const uint64_t* offs,
                       const uint16_t* lens, const LaunchArgs& a,
                       hipStream_t stream);
// frames.hip: per-frame TULIPS_FRAME_* flags (and optional counters[4]) /
// in-place checksum generation. Zero fields = defaults.
struct FrameLaunch
{
  int group = 0;           // lanes per frame: 16, 32, 64
  int unroll = 0;          // chunks in flight per lane
  uint32_t max_blocks = 0; // grid cap
  uint32_t block = 0;      // threads per workgroup
  int nontemporal = 1;     // nt chunk loads
  int fps = 1;             // validation at 16 x 6: 1, 2 (two frames in flight), 3 (pipelined)
};
bool frame_geometry_ok(int group, int unroll, uint32_t block);
// fields (nullable): per frame, the IPv4 (low 16 bits) and TCP (high 16)
// checksum values as stored, 0 where not written (see flags)
hipError_t launch_generate(uint8_t* base, const uint64_t* offs,
                           const uint16_t* lens, uint32_t n, uint8_t* flags,
                           hipStream_t stream, const FrameLaunch& fl = {},
                           uint32_t* fields = nullptr);
// compact generation: fields[i] only (IPv4 field low 16 bits, TCP high),
// frames not modified
hipError_t launch_generate_fields(const uint8_t* base, const uint64_t* offs,
                                  const uint16_t* lens, uint32_t n, uint32_t* fields,
                                  uint8_t* flags, hipStream_t stream,
                                  const FrameLaunch& fl = {});
hipError_t launch_frames(const uint8_t* base, const uint64_t* offs,
                         const uint16_t* lens, uint32_t n, uint8_t* flags,
                         uint32_t* counters, hipStream_t stream,
                         const FrameLaunch& fl = {});

// the low-latency validation server (zc_mailbox.h) on `stream`: one
// resident workgroup until mb->stop or an idle timeout, or (oneshot = a
// posted request's seq) one workgroup that serves that request and exits
struct ZcMailbox;
struct ZcArgs;
hipError_t launch_zc_server(ZcMailbox* mb, const ZcArgs* oneshot, hipStream_t stream);


}
