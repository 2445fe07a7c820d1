/*
 * tulips_csum_util.h — tuning and measurement entry points of the checksum
 * library (not part of the reference surface; used by bench.py and tests).
 */
#ifndef TULIPS_CSUM_UTIL_H
#define TULIPS_CSUM_UTIL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Kernel families (tulips_csum_tuning.kind). Kinds 2 and 4 (hybrid,
   workgroup-balanced) and the other span forms are measured variants kept
   outside the library (tools/variants/); the library rejects them. */
#define TULIPS_CSUM_KIND_DEFAULT 0
#define TULIPS_CSUM_KIND_SUBGROUP 1 /* `group` lanes (16/32/64) per segment,
                                       `unroll` chunks per lane in flight
                                       (16/32: 2/4/8; 32: 3; 64: 4/8/9/10/12) */
#define TULIPS_CSUM_KIND_PACKED 3   /* variable only: one wave per `group`
                                       segments (8/16), their chunks packed
                                       end to end, `unroll` 64-chunk windows
                                       per batch (2/4), double-buffered
                                       (`sps` 2) */
#define TULIPS_CSUM_KIND_SPAN 5     /* in-order arenas only
                                       (tulips_csum_batch_arena): a workgroup
                                       per 4 KiB * `unroll` (4..8) of arena
                                       bytes; a segment crossing ranges is
                                       summed in parts that meet in a
                                       per-range word of the stream's state.
                                       `group` 0 (or 7: the same form);
                                       `group` 9 (unroll 6..8): the
                                       tail-shaped cut, the last `sps` %
                                       (0 = 12) of the arena in ranges of
                                       unroll / 2 rows (measured variant);
                                       `group` 10 (unroll 6..8): the uniform
                                       cut with each quarter of the ranges at
                                       instruction priority 3..0 (measured
                                       variant) */

/* Explicit kernel geometry. Zero fields pick the library default. */
typedef struct tulips_csum_tuning
{
  int32_t kind;        /* TULIPS_CSUM_KIND_* */
  int32_t group;       /* see kind */
  int32_t unroll;      /* see kind */
  int32_t nontemporal; /* bit 0: nt loads, bit 1: nt result stores; -1 = default */
  uint32_t max_blocks; /* grid cap; 0 = default */
  int32_t block;       /* threads per workgroup: 256, 512 or 1024 (fixed-length
                          batches and frames also 64 or 128); 0 = default */
  int32_t sps;         /* PACKED: 2 = double-buffered windows (the only
                          form; 0 = default) */
} tulips_csum_tuning;

/* The geometry tulips_csum_batch_fixed / tulips_csum_batch would pick. */
int tulips_csum_default_tuning(uint32_t fixed_length, int variable,
                               tulips_csum_tuning* out);

int tulips_csum_batch_fixed_tuned(const uint8_t* base, uint64_t stride,
                                  uint32_t length, const uint16_t* seeds,
                                  const uint32_t* src, const uint32_t* dst,
                                  uint16_t* out, uint32_t n, uint32_t mode,
                                  const tulips_csum_tuning* tuning,
                                  void* stream);

int tulips_csum_batch_tuned(const uint8_t* base, const uint64_t* offsets,
                            const uint16_t* lengths, const uint16_t* seeds,
                            const uint32_t* src, const uint32_t* dst,
                            uint16_t* out, uint32_t n, uint32_t mode,
                            const tulips_csum_tuning* tuning, void* stream);

int tulips_csum_batch_arena_tuned(const uint8_t* base, uint64_t arena_bytes,
                                  const uint64_t* offsets, const uint16_t* lengths,
                                  const uint16_t* seeds, const uint32_t* src,
                                  const uint32_t* dst, uint16_t* out, uint32_t n,
                                  uint32_t mode, const tulips_csum_tuning* tuning,
                                  void* stream);

/* Frame kernels (include/tulips_csum.h) with an explicit geometry: op 0 =
 * tulips_csum_validate_frames, op 1 = tulips_csum_generate_frames (counters
 * ignored), op 2 = tulips_csum_generate_fields (`counters` is the n-entry
 * fields array). Uses tuning->group (lanes per frame, 0 = 16), unroll
 * (chunks in flight per lane, 0 = 6; supported pairs 16x4, 16x6, 16x8, 8x8,
 * 8x16, 32x4, 64x2), nontemporal (bit 0: nt loads, -1 = on), max_blocks and
 * block (64, 128, 256, 512 or 1024 threads; 0 = 256); sps 2 = two frames per subgroup in flight, 3 = a software pipeline
 * (the next frame's loads issued before this one is summed, ~4 frames per
 * subgroup) (validation at 16 x 6 only; otherwise ignored); kind is ignored. */
int tulips_csum_frames_tuned(int op, uint8_t* base, const uint64_t* offsets,
                             const uint16_t* lengths, uint32_t n,
                             uint8_t* flags, uint32_t* counters,
                             const tulips_csum_tuning* tuning, void* stream);

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
 * enable = 0 restores the previous handlers. Not for use in a product
 * process that installs its own signal handlers after this call. */
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
 * tulips_csum_burst_prefers_cpu, else 1). out[0..4] = median, p99,
 * min, mean (us) and, for path 1, the median GPU service time (request
 * picked up -> flags out, from the server's realtime clock; 0 otherwise).
 * `flags` (n bytes) holds the last call's flags. */
typedef struct tulips_csum_ctx tulips_csum_ctx;
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

/* Test hooks. tulips_csum_ctx_debug_set_seq: the sequence number of the
 * context's last zero-copy request (its low 16 bits tag the next request's
 * doorbell and completion words), to reach tag wrap-around in a test.
 * tulips_csum_mctx_set_peer_mode: how device-resident mctx calls move a
 * piece to a device other than the source: 0 = over xGMI (peer DMA) where
 * hipDeviceCanAccessPeer allows it, else staged through page-locked host
 * memory (the default); 1 = always staged. */
int tulips_csum_ctx_debug_set_seq(tulips_csum_ctx* ctx, uint64_t seq);
typedef struct tulips_csum_mctx tulips_csum_mctx;
int tulips_csum_mctx_set_peer_mode(tulips_csum_mctx* ctx, int mode);

#ifdef __cplusplus
}
#endif

#endif /* TULIPS_CSUM_UTIL_H */
