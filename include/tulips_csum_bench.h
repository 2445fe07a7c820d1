/*
 * tulips_csum_bench.h — measurement and test-data entry points, in their own
 * library (benchlib/libtulips_csum_bench.so) so the product library exports
 * only include/tulips_csum.h. bench.py, tools/ and tests/ load it beside the
 * product; nothing in the product calls it.
 *
 * The ceiling kernels here are the product kernels' load (and store)
 * patterns without their arithmetic: the roofline each kernel is compared
 * against in bench.py's `summary` and DESIGN.md §1 / §5 ("ceiling").
 */
#ifndef TULIPS_CSUM_BENCH_H
#define TULIPS_CSUM_BENCH_H

#include <stdint.h>

#include "tulips_csum.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Device fill with the SplitMix64 byte stream of SURVEY.md §8c: dst[i] =
 * stream byte (byte_off + i). Used to materialise synthetic arenas in HBM. */
int tulips_csum_fill_splitmix(uint8_t* dst, uint64_t nbytes, uint64_t seed,
                              uint64_t byte_off, void* stream);

/* Occupy `stream` for `us` microseconds (<= 1 s) with one sleeping wave: a
 * timed region queued behind it starts on the GPU only once the host has
 * submitted it (bench.py), so host-side launch latency is not timed. */
int tulips_csum_gpu_sleep(uint32_t us, void* stream);

/* Diagnostics: on SIGSEGV, SIGBUS, SIGILL, SIGFPE or SIGABRT write the
 * signal, the faulting address and the native call stack
 * (backtrace_symbols_fd) to stderr, then hand the signal to the handler that
 * was installed before (e.g. Python's faulthandler, which adds the
 * interpreter's stack) and let it terminate the process as it would have.
 * enable = 0 restores the previous handlers. */
int tulips_csum_debug_crash_backtrace(int enable);

/* Plain 16-byte streaming read of [p, p + nbytes): the measured read
 * ceiling that the checksum kernel's HBM rate is compared against. */
int tulips_csum_stream_read(const uint8_t* p, uint64_t nbytes, uint32_t* sink,
                            uint32_t max_blocks, void* stream);

/* The F9000 checksum kernel's read pattern without its arithmetic: tile k =
 * [p + k * tile_bytes, p + (k + 1) * tile_bytes) read by one wave, 64 lanes x
 * 12 clamped 16-byte loads (tile_bytes <= 65535). The ceiling that kernel is
 * compared against (bench.py extras.F9000.read_same_bytes). */
int tulips_csum_stream_read_tiles(const uint8_t* p, uint64_t tile_bytes, uint32_t ntiles,
                                  uint32_t* sink, void* stream);

/* The frame kernels' read pattern without their arithmetic: slot k's first
 * read_bytes bytes, [p + k * slot_bytes, + read_bytes), read by one 16-lane
 * subgroup, 6 clamped 16-byte loads per lane per pass (read_bytes <= 65535,
 * slot_bytes >= read_bytes). The ceiling the frame kernels are compared
 * against (bench.py extras.frames_validate_F1514.read_same_bytes). */
int tulips_csum_stream_read_slots(const uint8_t* p, uint64_t slot_bytes, uint32_t read_bytes,
                                  uint32_t nslots, uint32_t* sink, void* stream);

/* The same with the subgroup geometry named: group lanes per slot, unroll
 * clamped loads per lane per pass; (16, 6) as above, or (32, 3), the F1500
 * checksum kernel's (csum_kernel<32, 3>: slot_bytes = read_bytes = 1500 is
 * that kernel's exact load pattern, bench.py extras.F1500.read_same_bytes).
 * Other geometries: InvalidArgument. */
int tulips_csum_stream_read_slots_geom(const uint8_t* p, uint64_t slot_bytes, uint32_t read_bytes,
                                       uint32_t nslots, int group, int unroll, uint32_t* sink,
                                       void* stream);

/* The segmentation kernels' data movement without their header work: slot k
 * copies the `bytes` source bytes at src + (k / per_group) * group_stride +
 * (k % per_group) * step to out + k * out_stride (one 16-lane subgroup per
 * slot, dword-aligned 16-byte loads clamped to the source's last 16-byte
 * chunk, funnel shift, nontemporal 16-byte stores; the last chunk's bytes
 * past `bytes` are written as 0). out 16-byte aligned, out_stride a multiple
 * of 16 and >= bytes, bytes <= 65535. The ceiling the segmentation figures
 * are compared against (bench.py extras.segment_TSO_64K_mss1460
 * .copy_same_bytes). */
int tulips_csum_stream_copy_slots(const uint8_t* src, uint64_t group_stride, uint32_t per_group,
                                  uint32_t step, uint32_t bytes, uint32_t nslots, uint8_t* out,
                                  uint64_t out_stride, void* stream);

/* Latency of `reps` back-to-back receive validations of one burst of
 * host-resident frames, timed in C with a steady clock around each call
 * (no interpreter in the loop): path 0 = tulips_csum_validate_frames_host
 * (staged), 1 = tulips_csum_validate_frames_zc, 2 =
 * tulips_csum_validate_frames_cpu (host code, no GPU), 3 = the gpucsum
 * decorator's default choice per burst (2 when
 * tulips_csum_burst_prefers_cpu, else 1). out[0..3] = median, p99, min and
 * mean (us). `flags` (n bytes) holds the last call's flags. */
int tulips_csum_time_validate(tulips_csum_ctx* ctx, int path, const uint8_t* base,
                              const uint64_t* offsets, const uint16_t* lengths, uint32_t n,
                              uint32_t reps, uint8_t* flags, double* out);
/* The same over a ring of `nbursts` bursts laid `burst_stride` bytes apart
 * (call r validates the burst at ring + (r % nbursts) * burst_stride, same
 * offsets and lengths): with a ring larger than the host caches every call
 * meets frames that are not in them. */
int tulips_csum_time_validate_ring(tulips_csum_ctx* ctx, int path, const uint8_t* ring,
                                   uint64_t burst_stride, uint32_t nbursts,
                                   const uint64_t* offsets, const uint16_t* lengths,
                                   uint32_t n, uint32_t reps, uint8_t* flags, double* out);

#ifdef __cplusplus
}
#endif

#endif /* TULIPS_CSUM_BENCH_H */
