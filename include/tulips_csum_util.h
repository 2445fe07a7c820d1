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

/* Kernel families (tulips_csum_tuning.kind). */
#define TULIPS_CSUM_KIND_DEFAULT 0
#define TULIPS_CSUM_KIND_SUBGROUP 1 /* `group` lanes (16/32/64) per segment */
#define TULIPS_CSUM_KIND_HYBRID 2   /* variable only: `group`-lane subgroups
                                       (8/16/32) for short segments, `sps`
                                       of them in flight per subgroup; whole
                                       wave for long ones */
#define TULIPS_CSUM_KIND_PACKED 3   /* variable only: one wave per `group`
                                       segments (8/16/32/64), their chunks
                                       packed end to end, `unroll` 64-chunk
                                       windows in flight (2/4/8) */
#define TULIPS_CSUM_KIND_BALANCED 4 /* variable only: a workgroup of `block`/64
                                       waves (4 or 8) owns 8 segments per wave;
                                       the workgroup's chunks are packed end to
                                       end and split evenly over its waves,
                                       `unroll` windows (2/4) per batch,
                                       double-buffered; `group` must be 8 */
#define TULIPS_CSUM_KIND_SPAN 5     /* in-order arenas only
                                       (tulips_csum_batch_arena): a workgroup
                                       per 4 KiB * `unroll` of arena bytes.
                                       `group` 0 or 7 = split form (default,
                                       `unroll` 4..8): a segment crossing
                                       ranges is summed in parts that meet in
                                       a per-range word of the stream's state,
                                       only chunk prefixes in LDS; 6 = the same
                                       with the chunks staged in LDS
                                       (`unroll` 2/4/5/6/7/8/10/12); 1/2 =
                                       segments finished where they start,
                                       with 1/2 rows of 4 KiB read past the
                                       range (`unroll` 2/4/6/8/10/12 for 2,
                                       2/4/6/8 for 1); 3 = no halo, the
                                       crossing segment's wave reads its own
                                       tail (`unroll` 6/7/8); 4/5 =
                                       boundary-slot form with 2/1 halo rows
                                       (`unroll` 4/6/8/10/12 for 4, 8 for 5) */

/* Explicit kernel geometry. Zero fields pick the library default. */
typedef struct tulips_csum_tuning
{
  int32_t kind;        /* TULIPS_CSUM_KIND_* */
  int32_t group;       /* see kind */
  int32_t unroll;      /* 16-byte chunks in flight per lane: 2, 4 or 8 */
  int32_t nontemporal; /* bit 0: nt loads, bit 1: nt result stores; -1 = default */
  uint32_t max_blocks; /* grid cap; 0 = default */
  int32_t block;       /* threads per workgroup: 256, 512 or 1024; 0 = default */
  int32_t sps;         /* HYBRID: short segments per subgroup issued together
                          (1, 2, 4); PACKED: 1 = one batch of windows at a
                          time, 2 = double-buffered, 3 = double-buffered with
                          the next group's metadata prefetched (grid-stride;
                          pays with max_blocks below one group per wave);
                          0 = default */
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
 * ignored). Uses tuning->group (lanes per frame, 0 = 16), unroll (chunks
 * in flight per lane, 0 = 6; supported pairs 16x4, 16x6, 16x8, 8x8, 8x16,
 * 32x4, 64x2), nontemporal (bit 0: nt loads, -1 = on), max_blocks and
 * block; kind and sps are ignored. */
int tulips_csum_frames_tuned(int op, uint8_t* base, const uint64_t* offsets,
                             const uint16_t* lengths, uint32_t n,
                             uint8_t* flags, uint32_t* counters,
                             const tulips_csum_tuning* tuning, void* stream);

/* Device fill with the SplitMix64 byte stream of SURVEY.md §8c: dst[i] =
 * stream byte (byte_off + i). Used to materialise synthetic arenas in HBM. */
int tulips_csum_fill_splitmix(uint8_t* dst, uint64_t nbytes, uint64_t seed,
                              uint64_t byte_off, void* stream);

/* Plain 16-byte streaming read of [p, p + nbytes): the measured read
 * ceiling that the checksum kernel's HBM rate is compared against. */
int tulips_csum_stream_read(const uint8_t* p, uint64_t nbytes, uint32_t* sink,
                            uint32_t max_blocks, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* TULIPS_CSUM_UTIL_H */
