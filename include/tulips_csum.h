/*
 * tulips_csum.h — C ABI of the MI355X-native TULIPS checksum path.
 *
 * This is the drop-in boundary for TULIPS' Internet/TCP one's-complement
 * checksum (xenogenics/tulips @ 2024-12-20, src/stack). Every entry point
 * takes plain pointers and sizes; no HIP or torch types appear here, so the
 * header can be bound from C, C++, ctypes, cgo or JNI unchanged. Streams are
 * passed as `void*` (a hipStream_t; NULL = the legacy default stream).
 *
 * What each entry point replaces in the reference:
 *
 *   tulips_csum_host          tulips::stack::utils::checksum
 *                             (include/tulips/stack/Utils.h:10-11,
 *                              src/stack/Utils.cpp:14-42). The library also
 *                             exports that exact C++ symbol,
 *                             _ZN6tulips5stack5utils8checksumEtPKht.
 *   tulips_csum_ipv4_host     tulips::stack::ipv4::checksum
 *                             (include/tulips/stack/IPv4.h:90-92,
 *                              src/stack/IPv4.cpp:75-82); C++ symbol exported.
 *   tulips_csum_icmpv4_host   tulips::stack::icmpv4::checksum
 *                             (include/tulips/stack/ICMPv4.h:37,
 *                              src/stack/ICMPv4.cpp:10-15); C++ symbol exported.
 *   tulips_csum_tcp_host      tulips::stack::tcpv4::Processor::checksum
 *                             (private static, include/tulips/stack/tcpv4/
 *                              Processor.h:142-145, src/stack/tcpv4/
 *                              Processor.cpp:337-357).
 *   tulips_csum_batch         the per-frame loop of those calls
 *   tulips_csum_batch_fixed   (src/stack/tcpv4/Processor.cpp:121 verify,
 *                             src/stack/tcpv4/Send.cpp:448 generate,
 *                             src/stack/ipv4/Processor.cpp:95 verify,
 *                             src/stack/ipv4/Producer.cpp:81 generate), done
 *                             for a whole batch of device-resident segments by
 *                             HIP kernels on gfx950.
 *   tulips_csum_batch_host    the same for host-resident segments (pinned
 *                             staging, H2D, kernel, D2H), the path a transport
 *                             poll burst would take (src/transport/ofed/
 *                             Device.cpp:505-545).
 *
 * Semantics (bit-exact with the reference):
 *   RAW   out = utils::checksum(seed, seg, len)          (uncomplemented, host order)
 *   INET  out = r == 0 ? 0xffff : htons(r), r = RAW      (ipv4/icmpv4 wrappers)
 *   TCP   r = utils::checksum(pseudo, seg, len) with pseudo = checksum(
 *         checksum((len + 6) & 0xffff, src, 4), dst, 4); out as INET
 *   | TULIPS_CSUM_COMPLEMENT stores ~out (what the generate sites write into
 *         the header field, src/stack/tcpv4/Send.cpp:449, ipv4/Producer.cpp:81)
 *   A received segment verifies iff its INET/TCP result is 0xffff
 *   (src/stack/tcpv4/Processor.cpp:122, src/stack/ipv4/Processor.cpp:96).
 *
 * Return values are tulips::Status values (include/tulips/api/Status.h:8-44).
 *
 * Ownership: device pointers are borrowed until the work queued on `stream`
 * completes; nothing is retained after that. Threading: all entry points are
 * reentrant; a context (tulips_csum_ctx) must be used by one thread at a time.
 */
#ifndef TULIPS_CSUM_H
#define TULIPS_CSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* tulips::Status (include/tulips/api/Status.h:8-44) */
#define TULIPS_STATUS_OK 0
#define TULIPS_STATUS_INVALID_ARGUMENT 1
#define TULIPS_STATUS_HARDWARE_ERROR 2
#define TULIPS_STATUS_NO_MORE_RESOURCES 3
#define TULIPS_STATUS_UNSUPPORTED_OPERATION 18

/* Modes (low byte) and flags. */
#define TULIPS_CSUM_RAW 0u
#define TULIPS_CSUM_INET 1u
#define TULIPS_CSUM_TCP 2u
#define TULIPS_CSUM_MODE_MASK 0xffu
#define TULIPS_CSUM_COMPLEMENT 0x100u

/* Largest segment: the reference's `const uint16_t len` parameter. */
#define TULIPS_CSUM_MAX_SEGMENT 65535u

/* ---- host scalar drop-ins (no GPU involved) ------------------------------ */

uint16_t tulips_csum_host(uint16_t seed, const uint8_t* data, uint16_t len);
uint16_t tulips_csum_ipv4_host(const uint8_t* header20);
uint16_t tulips_csum_icmpv4_host(const uint8_t* header8);
/* src/dst: ipv4::Address::m_data, i.e. the 4 wire bytes as a native uint32. */
uint16_t tulips_csum_tcp_host(uint32_t src, uint32_t dst, uint16_t len,
                              const uint8_t* segment);

/* ---- device-resident batches --------------------------------------------- */

/*
 * Segment i is base[offsets[i] .. offsets[i] + lengths[i]).
 * `seeds` (RAW/INET only) may be NULL = all zero. `src`/`dst` are required
 * for TULIPS_CSUM_TCP and ignored otherwise. All arrays are device pointers.
 * n == 0 is a no-op returning OK. Segments may overlap and start at any byte.
 */
int tulips_csum_batch(const uint8_t* base, const uint64_t* offsets,
                      const uint16_t* lengths, const uint16_t* seeds,
                      const uint32_t* src, const uint32_t* dst, uint16_t* out,
                      uint32_t n, uint32_t mode, void* stream);

/*
 * In-order arena: the same batch when its segments lie in order inside one
 * allocation, offsets[i] + lengths[i] <= offsets[i+1] and
 * offsets[n-1] + lengths[n-1] <= arena_bytes (a receive ring, a packed
 * staging buffer). The work is then cut by arena bytes instead of by
 * segments (every workgroup gets the same bytes whatever the length mix).
 * Bytes of [base, base + arena_bytes) between segments may be read. A batch
 * that breaks the order gets undefined results but no access outside the
 * arena's 16-byte-aligned hull.
 */
int tulips_csum_batch_arena(const uint8_t* base, uint64_t arena_bytes,
                            const uint64_t* offsets, const uint16_t* lengths,
                            const uint16_t* seeds, const uint32_t* src,
                            const uint32_t* dst, uint16_t* out, uint32_t n,
                            uint32_t mode, void* stream);

/* Segment i is base[i*stride .. i*stride + length); length <= 65535. */
int tulips_csum_batch_fixed(const uint8_t* base, uint64_t stride,
                            uint32_t length, const uint16_t* seeds,
                            const uint32_t* src, const uint32_t* dst,
                            uint16_t* out, uint32_t n, uint32_t mode,
                            void* stream);

/*
 * Number of segments in [0, n) whose result (as selected by mode, INET or
 * TCP) is not 0xffff, i.e. that fail verification; written to *bad_count
 * (device pointer, uint32). `out` may be NULL when only the count is wanted.
 */
int tulips_csum_verify(const uint8_t* base, const uint64_t* offsets,
                       const uint16_t* lengths, const uint32_t* src,
                       const uint32_t* dst, uint16_t* out,
                       uint32_t* bad_count, uint32_t n, uint32_t mode,
                       void* stream);

/* tulips_csum_verify over an in-order arena (see tulips_csum_batch_arena). */
int tulips_csum_verify_arena(const uint8_t* base, uint64_t arena_bytes,
                             const uint64_t* offsets, const uint16_t* lengths,
                             const uint32_t* src, const uint32_t* dst, uint16_t* out,
                             uint32_t* bad_count, uint32_t n, uint32_t mode,
                             void* stream);

/* ---- host-resident batches (end-to-end path) ----------------------------- */

typedef struct tulips_csum_ctx tulips_csum_ctx;

/* A context owns a stream, pinned staging and device buffers sized for
 * `chunk_bytes` of segment bytes per pipeline stage (0 = 16 MiB; three
 * stages), and a pool of threads for the staging copy. */
int tulips_csum_ctx_create(int device, uint64_t chunk_bytes,
                           tulips_csum_ctx** ctx);
int tulips_csum_ctx_destroy(tulips_csum_ctx* ctx);

/* Page-locked host memory (hipHostMalloc): an arena staged here is DMA'd
 * straight to HBM by the *_host entry points, skipping their packing copy. */
int tulips_csum_host_alloc(size_t bytes, void** ptr);
int tulips_csum_host_free(void* ptr);

/* All pointers are host pointers; blocks until `out` holds every result. */
int tulips_csum_batch_host(tulips_csum_ctx* ctx, const uint8_t* base,
                           const uint64_t* offsets, const uint16_t* lengths,
                           const uint16_t* seeds, const uint32_t* src,
                           const uint32_t* dst, uint16_t* out, uint32_t n,
                           uint32_t mode);

/* ---- several GPUs, one process ---------------------------- */
/*
 * Byte-balanced contiguous split of a batch into `nshards` shards: bounds
 * (nshards + 1 entries) gets shard k = segments [bounds[k], bounds[k+1]),
 * each holding about 1/nshards of the bytes (prefix sum of lengths; shard k
 * starts at the first segment whose prefix reaches k/nshards of the total).
 * lengths is a host array.
 */
int tulips_csum_shard_plan(const uint16_t* lengths, uint32_t n, uint32_t nshards,
                           uint32_t* bounds);

typedef struct tulips_csum_mctx tulips_csum_mctx;

/* One host context (tulips_csum_ctx_create) per listed device, the CPUs
 * shared among them; a device may be listed more than once (independent
 * pipelines on one GPU). */
int tulips_csum_mctx_create(const int* devices, uint32_t ndevices,
                            uint64_t chunk_bytes, tulips_csum_mctx** ctx);
int tulips_csum_mctx_destroy(tulips_csum_mctx* ctx);

/* As the single-device *_host calls, over all devices at once: the batch is
 * split by tulips_csum_shard_plan, shard k runs on devices[k], results are
 * written in segment order (counters summed). Blocks until done. */
int tulips_csum_mctx_batch_host(tulips_csum_mctx* ctx, const uint8_t* base,
                                const uint64_t* offsets, const uint16_t* lengths,
                                const uint16_t* seeds, const uint32_t* src,
                                const uint32_t* dst, uint16_t* out, uint32_t n,
                                uint32_t mode);
int tulips_csum_mctx_validate_frames_host(tulips_csum_mctx* ctx,
                                          const uint8_t* base,
                                          const uint64_t* offsets,
                                          const uint16_t* lengths, uint32_t n,
                                          uint8_t* flags, uint32_t* counters);
/*
 * Device-resident batches over the context's devices ("data
 * starts on GPU 0"): every array is a device pointer on the device of
 * `stream` (the source). The batch is cut into contiguous byte-balanced
 * pieces, a run of pieces per listed device; each other device pulls its
 * pieces over xGMI (hipMemcpyPeerAsync on its own copy stream, ~32 MiB
 * pieces so copies overlap its kernels), checksums them, and sends the
 * results back into `out` (on the source device, segment order). The first
 * listed entry on the source device computes its share in place. Ordered
 * after the work already queued on `stream`; `stream` waits for all results
 * before its later work (the call returns before they are done). The arena
 * form requires an in-order arena (tulips_csum_batch_arena's contract) and
 * blocks until its cut plan is read back (one small D2H after the stream's
 * earlier work). Not capturable (InvalidArgument inside a stream capture).
 * Semantics per segment as tulips_csum_batch_fixed / tulips_csum_batch_arena.
 * tulips_csum_mctx_shard_bounds reports the segment range each device got.
 */
int tulips_csum_mctx_batch_fixed_device(tulips_csum_mctx* ctx, const uint8_t* base,
                                        uint64_t stride, uint32_t length,
                                        const uint16_t* seeds, const uint32_t* src,
                                        const uint32_t* dst, uint16_t* out, uint32_t n,
                                        uint32_t mode, void* stream);
int tulips_csum_mctx_batch_arena_device(tulips_csum_mctx* ctx, const uint8_t* base,
                                        uint64_t arena_bytes, const uint64_t* offsets,
                                        const uint16_t* lengths, const uint16_t* seeds,
                                        const uint32_t* src, const uint32_t* dst,
                                        uint16_t* out, uint32_t n, uint32_t mode,
                                        void* stream);
/*
 * Flow-affine receive validation ("enables flow-affine GPU
 * sharding"), the GPU analogue of NIC RSS queues with an indirection table
 * (src/transport/ena/RedirectionTable.cpp:74-98): every option-less,
 * unfragmented IPv4/TCP frame's 4-tuple (saddr | daddr | sport | dport, as
 * tulips_rss_toeplitz_batch takes it) is hashed with the `key_len`-byte
 * Toeplitz key from `init` on the context's first device, and the frame is
 * validated on device table[hash % table_len] (entries index the context's
 * devices); frames without such a tuple (including IPv4 fragments: MF set
 * or a fragment offset) go to table[0]. All frames of one
 * flow therefore land on one device, in arrival order. `flags` (and the
 * summed `counters`) come back in arrival order; `device_of` (host uint16[n],
 * may be NULL) receives each frame's device index. All arrays are host
 * arrays; blocks until done. tulips_csum_mctx_shard_bounds then reports the
 * prefix sums of the per-device frame counts.
 */
int tulips_csum_mctx_validate_frames_rss_host(tulips_csum_mctx* ctx, const uint8_t* base,
                                              const uint64_t* offsets,
                                              const uint16_t* lengths, uint32_t n,
                                              const uint8_t* key, size_t key_len,
                                              uint32_t init, const uint16_t* table,
                                              uint32_t table_len, uint8_t* flags,
                                              uint32_t* counters, uint16_t* device_of);
/*
 * The same for frames resident in the HBM of `stream`'s device (the source):
 * base/offsets/lengths/flags/counters (uint32[4], zeroed then summed) and
 * device_of (uint16[n], may be NULL) are device pointers on the source; key
 * and table stay host arrays (table_len <= 65536). On the source, one pass
 * hashes every frame's tuple (the flags rule above: option-less,
 * unfragmented IPv4/TCP, else table[0]) and orders the frames by device,
 * arrival order kept; the frames bound for each other device are gathered
 * into one packed run that device pulls over xGMI (hipMemcpyPeerAsync; the
 * HIP runtime stages it through host memory where the two devices have no
 * peer path). Each device validates its frames (the source's own in place)
 * and sends the flags home, where they are written in arrival order.
 * Ordered after the work queued on `stream`, which waits for all of it;
 * blocks once for the per-device frame counts (one small D2H). Not
 * capturable. tulips_csum_mctx_shard_bounds then reports the prefix sums of
 * the per-device frame counts.
 */
int tulips_csum_mctx_validate_frames_rss_device(tulips_csum_mctx* ctx, const uint8_t* base,
                                                const uint64_t* offsets,
                                                const uint16_t* lengths, uint32_t n,
                                                const uint8_t* key, size_t key_len,
                                                uint32_t init, const uint16_t* table,
                                                uint32_t table_len, uint8_t* flags,
                                                uint32_t* counters, uint16_t* device_of,
                                                void* stream);
/* The shard bounds (ndevices + 1 entries) of the context's last call. */
int tulips_csum_mctx_shard_bounds(const tulips_csum_mctx* ctx, uint32_t* bounds);
/* How the device-resident calls move a piece to a device other than the
 * source: 0 = over xGMI (peer DMA) where hipDeviceCanAccessPeer allows it,
 * else staged through page-locked host memory (the default); 1 = always
 * staged through page-locked host memory. */
int tulips_csum_mctx_set_peer_mode(tulips_csum_mctx* ctx, int mode);

/* ---- Toeplitz RSS hash -------------------------------- */
/*
 * tulips::stack::utils::toeplitz (include/tulips/stack/Utils.h:25-28,
 * src/stack/Utils.cpp:86-133), whose C++ symbol the library also exports:
 * the 96-bit tuple saddr | daddr | htons(sport) | htons(dport) hashed with a
 * `key_len`-byte key (>= 4; host pointer) starting from `init`. Addresses
 * are ipv4::Address::m_data words (wire bytes as a native uint32).
 */
int tulips_rss_toeplitz_host(uint32_t saddr, uint32_t daddr, uint16_t sport,
                             uint16_t dport, const uint8_t* key,
                             size_t key_len, uint32_t init, uint32_t* out);

/* Batch: device arrays of n tuples (structure of arrays) -> out[i]. */
int tulips_rss_toeplitz_batch(const uint32_t* saddr, const uint32_t* daddr,
                              const uint16_t* sport, const uint16_t* dport,
                              uint32_t n, const uint8_t* key, size_t key_len,
                              uint32_t init, uint32_t* out, void* stream);

/* ---- receive-side frame validation ------------------ */
/*
 * Per-frame result of the checks the reference stack makes before a segment
 * reaches TCP — ethernet/Processor.cpp:69,91 (ethertype), ipv4/Processor.cpp:
 * 67-122 (vhl 0x45, no fragments, header checksum, protocol), tcpv4/
 * Processor.cpp:121-131 (pseudo-header checksum) — in the role of the NIC
 * offload bits that transport::Device::VALIDATE_IP_CSUM / VALIDATE_L4_CSUM
 * consult (include/tulips/transport/Device.h:29-30,
 * src/transport/ena/Device.cpp:318-340).
 *
 *   0                    not IPv4 (short frame, other ethertype, IP options)
 *   IPV4                 an option-less IPv4 header follows the Ethernet one
 *   IP_CSUM_OK           ... and its header checksum verifies
 *   TCP                  ... unfragmented, protocol 6
 *   L4_CSUM_OK           ... and the TCP checksum over ntohs(len) - 20 bytes
 *                        verifies (never set with TRUNCATED)
 *   TRUNCATED            the frame ends before the IPv4 header (alone) or
 *                        before the TCP segment the IP length announces
 */
#define TULIPS_FRAME_IPV4 0x01u
#define TULIPS_FRAME_IP_CSUM_OK 0x02u
#define TULIPS_FRAME_TCP 0x04u
#define TULIPS_FRAME_L4_CSUM_OK 0x08u
#define TULIPS_FRAME_TRUNCATED 0x10u

/*
 * Frame i is base[offsets[i] .. offsets[i] + lengths[i]) (device pointers;
 * a frame is read only within its length). Writes flags[i] (uint8, may be
 * NULL) and, when `counters` (device uint32[4], may be NULL) is given,
 * overwrites it with this call's counts { IPv4 frames, bad IP checksums, TCP
 * frames, TCP frames without L4_CSUM_OK } (zeros for n == 0). At least one of
 * flags / counters is required for n > 0. Counting uses the per-stream state
 * below (a call captured in a graph gets counter shards the graph owns).
 */
int tulips_csum_validate_frames(const uint8_t* base, const uint64_t* offsets,
                                const uint16_t* lengths, uint32_t n,
                                uint8_t* flags, uint32_t* counters,
                                void* stream);

/* ---- send-side checksum generation --------------------- */
/*
 * Writes, in place, the IPv4 header checksum of every option-less IPv4 frame
 * (`ipchksum = ~ipv4::checksum(header)`, src/stack/ipv4/Producer.cpp:79-82)
 * and the TCP checksum of every unfragmented TCP frame over ntohs(len) - 20
 * segment bytes (`chksum = ~tcpv4 checksum`, src/stack/tcpv4/Send.cpp:
 * 441-449) — what the reference leaves to the NIC under
 * TULIPS_HAS_HW_CHECKSUM. The current field contents are ignored (as if
 * zeroed). Frames must not overlap. flags[i] (may be NULL) reports what was
 * written with the TULIPS_FRAME_* bits: IP_CSUM_OK = IP checksum written,
 * L4_CSUM_OK = TCP checksum written (TRUNCATED: the segment did not fit).
 */
int tulips_csum_generate_frames(uint8_t* base, const uint64_t* offsets,
                                const uint16_t* lengths, uint32_t n,
                                uint8_t* flags, void* stream);

/*
 * Compact-field generation: the two values tulips_csum_generate_frames would
 * write, returned instead of patched into the frames (which are only read):
 * fields[i] = IPv4 header checksum field (low 16 bits) | TCP checksum field
 * (high 16 bits), each as the uint16 a little-endian load of the header word
 * gives (so `*(uint16_t*)(frame + 24) = fields[i] & 0xffff` stores it), 0
 * where flags[i] (may be NULL; bits as for generate) reports nothing
 * written. For callers that patch headers when they post the TX descriptor
 * (src/stack/ipv4/Producer.cpp:79-82, src/stack/tcpv4/Send.cpp:441-449): 4
 * bytes written per frame instead of one partial 64-byte line. `fields` is
 * a device array of n uint32.
 */
int tulips_csum_generate_fields(const uint8_t* base, const uint64_t* offsets,
                                const uint16_t* lengths, uint32_t n, uint32_t* fields,
                                uint8_t* flags, void* stream);

/*
 * Segmentation offload (what src/transport/ofed/Device.cpp:688-772 asks of
 * the NIC with IBV_WR_TSO; header length per stack::utils::headerLength,
 * src/stack/Utils.cpp:67-84). Frame i = in_base[in_offsets[i]..][..
 * in_lengths[i]]. An option-less IPv4 / unfragmented TCP super-frame whose
 * payload P = ntohs(len) - 20 - doff*4 exceeds `mss` becomes ceil(P / mss)
 * frames, segment k carrying payload [k*mss, min(P, (k+1)*mss)) behind the
 * super-frame's header with: IPv4 total length and id + k, TCP seq +
 * k*mss, FIN/PSH kept on the last segment only, CWR on the first only, and
 * both checksums generated. Any other frame is copied whole with checksum
 * generation as tulips_csum_generate_frames does.
 *
 * out_first (n + 1 entries, device) receives the exclusive prefix sum of
 * the per-frame segment counts: frame i's segments are j = out_first[i] ..
 * out_first[i+1] - 1, out_first[n] is the total. Segment j is written to
 * out_base + j * out_stride (out_base 16-byte aligned, out_stride a multiple
 * of 16) with its length in out_lengths[j]; a segment longer than out_stride
 * is not written (length 0), nor is any j >= out_capacity. With
 * out_capacity == 0 only out_first is computed (to size the output).
 * n <= 2^24, 1 <= mss <= 65535. Input frames are not modified.
 *
 * The library keeps a device workspace per (device, stream), made or grown
 * on a call that needs more room; calls on one stream run in order, calls
 * on different streams may overlap. The calls a stream capture records on a
 * stream share a workspace made for that capture and owned by the graph (see
 * "per-stream state" below), so no warm-up call is needed, later direct
 * calls never free it under the graph, and a replay may overlap direct calls
 * on the capture stream.
 */
int tulips_csum_segment_frames(const uint8_t* in_base,
                               const uint64_t* in_offsets,
                               const uint16_t* in_lengths, uint32_t n,
                               uint32_t mss, uint8_t* out_base,
                               uint64_t out_stride, uint32_t out_capacity,
                               uint16_t* out_lengths, uint32_t* out_first,
                               void* stream);

/*
 * Segmentation with the caller's plan (the reference's split: the host knows
 * each super-frame's header length, stack::utils::headerLength,
 * src/stack/Utils.cpp:67-84, and the MSS it posts with the TSO request,
 * src/transport/ofed/Device.cpp:688-700). `first` (device, n + 1 entries)
 * is what tulips_csum_segment_frames would write to out_first: first[i] =
 * the segments of frames 0..i-1 (ceil(P / mss) for a super-frame as above,
 * 1 for any other frame; tulips_csum_segment_plan_host computes it from host
 * headers). The segment kernel then runs alone, with no counting prologue;
 * outputs, limits and semantics as tulips_csum_segment_frames (segments
 * j >= min(first[n], out_capacity) are not written). A segment whose frame's
 * header disagrees with the plan (more segments planned than its payload
 * makes, or a frame planned with none) gets length 0; reads never leave the
 * frames, writes never leave out_capacity slots. Needs no per-stream state
 * (capturable as is).
 */
int tulips_csum_segment_frames_planned(const uint8_t* in_base, const uint64_t* in_offsets,
                                       const uint16_t* in_lengths, uint32_t n, uint32_t mss,
                                       const uint32_t* first, uint8_t* out_base,
                                       uint64_t out_stride, uint32_t out_capacity,
                                       uint16_t* out_lengths, void* stream);

/*
 * The plan for tulips_csum_segment_frames_planned from host-resident frames
 * (each frame's first 48 bytes are read): first (host, n + 1 entries)
 * receives the exclusive prefix of the per-frame segment counts, first[n]
 * the total. The same rule as the device prologue.
 */
int tulips_csum_segment_plan_host(const uint8_t* base, const uint64_t* offsets,
                                  const uint16_t* lengths, uint32_t n, uint32_t mss,
                                  uint32_t* first);

/* Host-resident frames through a context's pinned pipeline; `flags` is a
 * host array of n bytes, `counters` (may be NULL) a host uint32[4]. */
int tulips_csum_validate_frames_host(tulips_csum_ctx* ctx, const uint8_t* base,
                                     const uint64_t* offsets,
                                     const uint16_t* lengths, uint32_t n,
                                     uint8_t* flags, uint32_t* counters);

/*
 * The same flags and counters for host-resident frames computed on the
 * calling thread with the host scalar drop-ins (tulips_csum_ipv4_host,
 * tulips_csum_tcp_host; no GPU involved), as the reference verifies each
 * frame in its poll loop (src/stack/ipv4/Processor.cpp:94-103,
 * src/stack/tcpv4/Processor.cpp:120-132). For poll bursts too small to pay
 * for a PCIe round trip: the gpucsum decorator takes it below its measured
 * crossover (a few dozen 1514 B frames). All arrays are host arrays.
 */
int tulips_csum_validate_frames_cpu(const uint8_t* base, const uint64_t* offsets,
                                    const uint16_t* lengths, uint32_t n,
                                    uint8_t* flags, uint32_t* counters);

/*
 * The CPU / GPU crossover for one receive poll burst, measured on MI355X
 * with frames a NIC has just written (outside the CPU caches; bench.py
 * extras.burst_latency_host.cold_ring): 1514 B frames cost the
 * host code ~0.13-0.16 us each, the zero-copy GPU path ~13 us + ~0.02 us
 * each (64 frames: 8.5 against 14.4 us; 256: 41.4 against 18.3), so they
 * cross near 96 frames; the host cost follows the bytes, so larger frames
 * cross sooner. Returns 1 when a burst of n frames and `bytes` bytes is
 * cheaper on the calling thread (tulips_csum_validate_frames_cpu): fewer
 * than TULIPS_CSUM_CPU_BELOW_FRAMES frames and fewer than
 * TULIPS_CSUM_CPU_BELOW_BYTES bytes. The gpucsum decorator's defaults.
 */
#define TULIPS_CSUM_CPU_BELOW_FRAMES 96u
#define TULIPS_CSUM_CPU_BELOW_BYTES (96u * 1514u)
int tulips_csum_burst_prefers_cpu(uint32_t n, uint64_t bytes);

/*
 * Low-latency (zero-copy) form of tulips_csum_validate_frames_host for poll
 * bursts (the reference is a latency stack: docs/topics/Test-and-
 * Performance.md:12-15, its OFED poll drains whatever CQ batch is ready,
 * src/transport/ofed/Device.cpp:505-545). Frames in page-locked memory (one
 * hipHostMalloc / hipHostRegister allocation, e.g. a transport's staging
 * arena) are read in place over PCIe by the kernel: no staging copy and no
 * DMA; the flags come back through a page-locked mailbox the calling thread
 * spins on. By default each call is one launch whose arguments carry the
 * burst's descriptors (up to 62 frames; larger bursts' descriptors go
 * through the mailbox, one workgroup per 64 frames). With
 * tulips_csum_ctx_set_lowlat(ctx, 1) eight workgroups stay resident on the
 * context's device instead and poll tagged doorbell words in the mailbox
 * (no launch per call; they leave the GPU after 100 ms without a burst, the
 * next call restarting them, and when the context is destroyed or switched
 * back). Frames in pageable memory are first packed into the context's
 * 2 MiB page-locked staging. Bursts of more than TULIPS_CSUM_ZC_MAX_FRAMES
 * frames, or pageable bursts past 2 MiB, take
 * tulips_csum_validate_frames_host. Same flags and counters.
 */
#define TULIPS_CSUM_ZC_MAX_FRAMES 1024u
int tulips_csum_validate_frames_zc(tulips_csum_ctx* ctx, const uint8_t* base,
                                   const uint64_t* offsets, const uint16_t* lengths,
                                   uint32_t n, uint8_t* flags, uint32_t* counters);
/* 0 = one launch per burst (default), 1 = resident server. */
int tulips_csum_ctx_set_lowlat(tulips_csum_ctx* ctx, int resident);

/* In-place checksum generation for host-resident frames (what a transport's
 * send path would offload, src/transport/ofed/Device.cpp:756): the frames
 * travel through the context's pinned pipeline, the GPU computes both fields
 * as tulips_csum_generate_frames does, and only the 4 field bytes per frame
 * are written back into `base`. `flags` (host, n bytes) may be NULL. */
int tulips_csum_generate_frames_host(tulips_csum_ctx* ctx, uint8_t* base,
                                     const uint64_t* offsets,
                                     const uint16_t* lengths, uint32_t n,
                                     uint8_t* flags);

/* Segmentation offload of host-resident super-frames (the TSO request of
 * src/transport/ofed/Device.cpp:688-772), semantics as
 * tulips_csum_segment_frames with host arrays: out_base (host) receives
 * segment j at out_base + j * out_stride for j < out_capacity, out_lengths
 * (host) its length, out_first (host, n + 1 entries) the exclusive prefix of
 * the per-frame segment counts. Blocks until the outputs are written. */
int tulips_csum_segment_frames_host(tulips_csum_ctx* ctx, const uint8_t* in_base,
                                    const uint64_t* in_offsets,
                                    const uint16_t* in_lengths, uint32_t n,
                                    uint32_t mss, uint8_t* out_base,
                                    uint64_t out_stride, uint32_t out_capacity,
                                    uint16_t* out_lengths, uint32_t* out_first);

/* ---- explicit kernel geometry -------------------------------------------- */
/*
 * The entry points above pick their kernel geometry themselves
 * (tulips_csum_default_tuning). These forms take it from the caller, for
 * geometry sweeps and the parity tests of every shipped geometry; results are
 * identical whatever the geometry.
 */
/* Kernel families (tulips_csum_tuning.kind). Kinds 2 and 4 (hybrid,
   workgroup-balanced) and the other span forms are measured variants kept
   outside the library (tools/sessions/variants/); the library rejects them. */
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

/* ---- per-stream state ---------------------------------------------------- */
/*
 * Counting calls (tulips_csum_verify, tulips_csum_validate_frames with
 * counters), the arena calls (tulips_csum_batch_arena, _verify_arena) and
 * tulips_csum_segment_frames keep a small device workspace per (device,
 * stream), on the stream's own device. A call holds the stream's lock from
 * its first launch to its last, so host threads sharing a stream (e.g. the
 * NULL stream) never interleave their launch sequences. The workspace is
 * allocated, freed and waited for in relaxed capture mode, so these calls
 * may run beside another thread's global-mode stream capture without
 * invalidating it.
 *
 * A call captured in a HIP graph (stream capture) runs on arrays made for
 * that capture, so no warm-up call is needed and replays never share arrays
 * with direct calls or with other graphs. The graph owns them, as the
 * reference's callers own their buffers (src/transport/list/Device.cpp:
 * 60-62): they are attached to the graph as a HIP user object
 * (hipGraphRetainUserObject), every executable instantiated from it holds a
 * reference, and once the graph and all its executables are destroyed the
 * arrays are freed by the library's next uncaptured call on any stream (or by
 * tulips_csum_release_stream). Graphs may be destroyed in any order and at
 * any time after their last replay completes.
 *
 * tulips_csum_release_stream waits for `stream` and frees the arrays the
 * library holds for that stream's direct calls, plus the arrays of graphs
 * destroyed so far. Call it before hipStreamDestroy; it must not race calls
 * on the same stream. Later calls on the stream start afresh; graphs
 * captured on it stay valid. tulips_csum_ctx_destroy releases the context's
 * own streams.
 */
int tulips_csum_release_stream(void* stream);

/* ---- misc ---------------------------------------------------------------- */

const char* tulips_csum_status_string(int status);
/* The HIP error behind the calling thread's last HardwareError /
 * NoMoreResources from a device entry point ("" if none). */
const char* tulips_csum_last_error(void);
const char* tulips_csum_version(void);

#ifdef __cplusplus
}
#endif

#endif /* TULIPS_CSUM_H */
