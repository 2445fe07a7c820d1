// csum_capi.hip — the C ABI of include/tulips_csum.h (batches, tuning
// forms, status strings), plus the host scalar drop-ins that keep the
// reference's C++ symbols (tulips::stack::utils::checksum & co.).
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/tulips_csum.h"
#include "csum_common.h"
#include "csum_launch.h"
#include "stream_state.h"

using namespace tulips_amd;

// ---------------------------------------------------------------------------
// Host scalar path. A 20-byte IPv4 header or an 8-byte ICMP header never goes
// to a GPU; these keep the reference's call sites compiling and linking
// unchanged. Exact by the closed form in csum_common.h: the data's
// little-endian dword sum (relative to `data`, i.e. an even "address"), folded,
// byte-swapped, then the seed added with end-around carry.
// ---------------------------------------------------------------------------
namespace {

inline uint32_t
host_le_partial(const uint8_t* data, uint32_t len)
{
  uint64_t acc = 0;
  uint32_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t w;
    memcpy(&w, data + i, 8);
    acc += (w & 0xffffffffu) + (w >> 32);
  }
  if (i < len) {
    uint8_t tail[8] = { 0, 0, 0, 0, 0, 0, 0, 0 };
    memcpy(tail, data + i, len - i);
    uint64_t w;
    memcpy(&w, tail, 8);
    acc += (w & 0xffffffffu) + (w >> 32);
  }
  return fold64(acc);
}

inline uint32_t
host_checksum(uint32_t seed, const uint8_t* data, uint32_t len)
{
  // `data` plays the role of an even start address: swap after the fold.
  const uint32_t r = bswap16(fold32(host_le_partial(data, len)));
  return add_seed(r, seed);
}

} // namespace

// The reference's C++ symbols (include/tulips/stack/Utils.h:10-11,
// include/tulips/stack/IPv4.h:90-92, include/tulips/stack/ICMPv4.h:37).
namespace tulips::stack::utils {
__attribute__((visibility("default"))) uint16_t
checksum(const uint16_t seed, const uint8_t* const data, const uint16_t len)
{
  return uint16_t(host_checksum(seed, data, len));
}
}
namespace tulips::stack::ipv4 {
__attribute__((visibility("default"))) uint16_t
checksum(const uint8_t* const data)
{
  return uint16_t(inet_post(host_checksum(0, data, 20)));
}
}
namespace tulips::stack::icmpv4 {
__attribute__((visibility("default"))) uint16_t
checksum(const uint8_t* const data)
{
  return uint16_t(inet_post(host_checksum(0, data, 8)));
}
}

// tulips::stack::tcpv4::Processor::checksum (private static,
// include/tulips/stack/tcpv4/Processor.h:142-145, src/stack/tcpv4/
// Processor.cpp:337-357). Exported under its mangled name so a stack linked
// against this library before its own objects resolves the verify
// (Processor.cpp:121) and generate (Send.cpp:448) sites here without a
// source change. The ipv4::Address arguments arrive by const reference, i.e.
// as pointers to the 4-byte m_data word (include/tulips/stack/IPv4.h:55).
extern "C" __attribute__((visibility("default"))) uint16_t
tulips_tcpv4_processor_checksum(const uint32_t* src, const uint32_t* dst,
                                const uint16_t len, const uint8_t* const data)
  __asm__("_ZN6tulips5stack5tcpv49Processor8checksumERKNS0_4ipv47AddressES6_tPKh");

uint16_t
tulips_tcpv4_processor_checksum(const uint32_t* src, const uint32_t* dst,
                                const uint16_t len, const uint8_t* const data)
{
  // the reference returns the uncomplemented sum in network order, 0 -> 0xffff
  return uint16_t(inet_post(host_checksum(tcp_seed(*src, *dst, len), data, len)));
}

extern "C" {

uint16_t
tulips_csum_host(uint16_t seed, const uint8_t* data, uint16_t len)
{
  return uint16_t(host_checksum(seed, data, len));
}

uint16_t
tulips_csum_ipv4_host(const uint8_t* header20)
{
  return uint16_t(inet_post(host_checksum(0, header20, 20)));
}

uint16_t
tulips_csum_icmpv4_host(const uint8_t* header8)
{
  return uint16_t(inet_post(host_checksum(0, header8, 8)));
}

uint16_t
tulips_csum_tcp_host(uint32_t src, uint32_t dst, uint16_t len,
                     const uint8_t* segment)
{
  return uint16_t(
    inet_post(host_checksum(tcp_seed(src, dst, len), segment, len)));
}

// Receive validation of host-resident frames on the calling thread: the
// flags and counters of tulips_csum_validate_frames, computed with the host
// scalar drop-ins above (ipv4::checksum over bytes 14..33, the tcpv4
// pseudo-header checksum over the segment), i.e. the reference's per-frame
// checks (ipv4/Processor.cpp:67-122, tcpv4/Processor.cpp:120-132). Header
// rules as frame_common.h parse_header.
int
tulips_csum_burst_prefers_cpu(uint32_t n, uint64_t bytes)
{
  return n < TULIPS_CSUM_CPU_BELOW_FRAMES && bytes < TULIPS_CSUM_CPU_BELOW_BYTES ? 1 : 0;
}

int
tulips_csum_validate_frames_cpu(const uint8_t* base, const uint64_t* offsets,
                                const uint16_t* lengths, uint32_t n, uint8_t* flags,
                                uint32_t* counters)
{
  if (counters) {
    memset(counters, 0, 4 * sizeof(uint32_t));
  }
  if (n == 0) {
    return TULIPS_STATUS_OK;
  }
  if (!base || !offsets || !lengths || (!flags && !counters)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  uint32_t cnt[4] = { 0, 0, 0, 0 };
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t* f = base + offsets[i];
    const uint32_t flen = lengths[i];
    auto byte = [&](uint32_t k) -> uint32_t { return k < flen ? f[k] : 0u; };
    const uint32_t type = (byte(12) << 8) | byte(13);
    const uint32_t total = (byte(16) << 8) | byte(17);
    const bool eth_ip = flen >= 14 && type == 0x0800u;
    const bool runt = eth_ip && flen < 34;
    const bool ipv4 = eth_ip && !runt && byte(14) == 0x45u;
    const bool tcp = ipv4 && (byte(20) & 0x3fu) == 0 && byte(21) == 0 && byte(23) == 6u;
    const uint32_t tcplen = (total - 20u) & 0xffffu;
    const bool trunc = tcp && (total < 20u || 34u + tcplen > flen);
    uint32_t fl = 0;
    if (runt) {
      fl = TULIPS_FRAME_TRUNCATED;
    } else if (ipv4) {
      const bool ip_ok = tulips_csum_ipv4_host(f + 14) == 0xffffu;
      bool l4_ok = false;
      if (tcp && !trunc) {
        uint32_t src, dst;
        memcpy(&src, f + 26, 4);
        memcpy(&dst, f + 30, 4);
        l4_ok = tulips_csum_tcp_host(src, dst, uint16_t(tcplen), f + 34) == 0xffffu;
      }
      fl = TULIPS_FRAME_IPV4 | (ip_ok ? TULIPS_FRAME_IP_CSUM_OK : 0u) |
           (tcp ? TULIPS_FRAME_TCP : 0u) | (trunc ? TULIPS_FRAME_TRUNCATED : 0u) |
           (l4_ok ? TULIPS_FRAME_L4_CSUM_OK : 0u);
      cnt[0] += 1;
      cnt[1] += ip_ok ? 0u : 1u;
      cnt[2] += tcp ? 1u : 0u;
      cnt[3] += (tcp && !l4_ok) ? 1u : 0u;
    }
    if (flags) {
      flags[i] = uint8_t(fl);
    }
  }
  if (counters) {
    memcpy(counters, cnt, sizeof(cnt));
  }
  return TULIPS_STATUS_OK;
}

} // extern "C"

// ---------------------------------------------------------------------------
// Device batches.
// ---------------------------------------------------------------------------
namespace {


thread_local char last_error[160] = "";

inline int
status_of(hipError_t e)
{
  if (e != hipSuccess) {
    snprintf(last_error, sizeof(last_error), "%s (%d): %s", hipGetErrorName(e),
             int(e), hipGetErrorString(e));
  }
  switch (e) {
    case hipSuccess:
      return TULIPS_STATUS_OK;
    case hipErrorOutOfMemory:
      return TULIPS_STATUS_NO_MORE_RESOURCES;
    case hipErrorInvalidValue:
      return TULIPS_STATUS_INVALID_ARGUMENT;
    default:
      return TULIPS_STATUS_HARDWARE_ERROR;
  }
}

inline bool
mode_ok(uint32_t mode, const uint32_t* src, const uint32_t* dst)
{
  if ((mode & ~(TULIPS_CSUM_MODE_MASK | TULIPS_CSUM_COMPLEMENT)) != 0) {
    return false;
  }
  const uint32_t m = mode & TULIPS_CSUM_MODE_MASK;
  if (m > TULIPS_CSUM_TCP) {
    return false;
  }
  return m != TULIPS_CSUM_TCP || (src && dst);
}

// The instantiated kernel geometries (csum_kernels.hip dispatch tables).
inline bool
geometry_ok(int kind, int group, int unroll, int spw, bool variable)
{
  switch (kind) {
    case TULIPS_CSUM_KIND_SUBGROUP:
      return spw == 1 && (((group == 16 || group == 32) &&
                           (unroll == 2 || unroll == 4 || unroll == 8)) ||
                          (group == 32 && unroll == 3) ||
                          (group == 64 && (unroll == 4 || unroll == 8 || unroll == 9 ||
                                           unroll == 10 || unroll == 12)));
    case TULIPS_CSUM_KIND_PACKED:
      // double-buffered windows only (sps 2)
      return variable && spw == 2 && (group == 8 || group == 16) &&
             (unroll == 2 || unroll == 4);
    default:
      return false;
  }
}

// Default geometry (measured on MI355X by tools/sessions/probes/sweep.py,
// profiles/sweep_r01.json): nt loads everywhere; the subgroup is sized so a
// lane holds about one batch of chunks.
tulips_csum_tuning
default_tuning(uint32_t len, bool variable)
{
  tulips_csum_tuning t;
  t.kind = TULIPS_CSUM_KIND_SUBGROUP;
  t.nontemporal = 1;
  t.max_blocks = 0;
  t.block = 256;
  t.sps = 1;
  if (variable) {
    // one wave per 8 segments, chunks packed end to end, 4 windows in
    // flight, double-buffered (tools/sessions/probes/probe_packed.py,
    // profiles/probe_packed_r01.json: ZIPF 14.8 us vs 16.8 single-buffered
    // and 18.7 hybrid; 1500 B through offsets 19.1 vs 34.2 hybrid).
    // 256-thread blocks: 1024-thread blocks are 0.6 us faster alone but
    // cannot share CUs with a concurrent launch (overlapped bursts: 21 us
    // per launch vs 10)
    t.kind = TULIPS_CSUM_KIND_PACKED;
    t.group = 8;
    t.unroll = 4;
    t.sps = 2;
    return t;
  }
  const uint32_t nch = len / 16 + 2;
  if (nch > 512) {        // > ~8 KiB (F9000): whole wave, 12 chunks per lane,
    t.group = 64;         // a 9000 B segment in one batch (tools/sessions/probes/probe_fixed.py:
    t.unroll = 12;        // 82.3 vs 84.0 us for 64 x 8)
  } else if (nch > 256) { // > ~4 KiB: whole wave, 8 chunks in flight per lane
    t.group = 64;
    t.unroll = 8;
  } else if (nch > 96) {  // ~1.5-4 KiB: 32 lanes x 4
    t.group = 32;
    t.unroll = 4;
  } else if (nch > 64) {  // ~1-1.5 KiB (F1500): 32 lanes x 3, the 96 chunks a
    t.group = 32;         // 1500 B segment touches at any alignment in one batch
    t.unroll = 3;         // with no redundant loads (tools/sessions/probes/probe_fixed.py,
                          // profiles/probe_fixed_r05.txt: 15.73 vs 15.95 us)
  } else {
    t.group = 16;
    t.unroll = 4;
  }
  return t;
}

inline void
apply_tuning(LaunchArgs& a, const tulips_csum_tuning& d,
             const tulips_csum_tuning* t)
{
  // an explicit kind takes its group/unroll from the caller (0 = default)
  const bool own = t && t->kind != TULIPS_CSUM_KIND_DEFAULT;
  a.kind = own ? t->kind : d.kind;
  a.group = (t && t->group) ? t->group : (own && t->kind != d.kind ? 0 : d.group);
  a.unroll = (t && t->unroll) ? t->unroll : (own && t->kind != d.kind ? 4 : d.unroll);
  const int32_t nt = (t && t->nontemporal >= 0) ? t->nontemporal : d.nontemporal;
  a.nontemporal = (nt & 1) != 0;
  a.nt_store = (nt & 2) != 0;
  a.max_blocks = (t && t->max_blocks) ? t->max_blocks : d.max_blocks;
  a.block = (t && t->block) ? t->block : d.block;
  a.spw = (t && t->sps) ? t->sps : (own && t->kind != d.kind ? 1 : d.sps);
}

inline bool
block_ok(int block)
{
  return block == 256 || block == 512 || block == 1024;
}

// fixed-length segments (one subgroup per segment, no per-workgroup state)
// also take 64- and 128-thread workgroups
inline bool
fixed_block_ok(int block)
{
  return block == 64 || block == 128 || block_ok(block);
}

int
batch_fixed(const uint8_t* base, uint64_t stride, uint32_t length,
            const uint16_t* seeds, const uint32_t* src, const uint32_t* dst,
            uint16_t* out, uint32_t* bad, uint32_t n, uint32_t mode,
            const tulips_csum_tuning* tuning, void* stream)
{
  if (n == 0) {
    return TULIPS_STATUS_OK;
  }
  if (!base || (!out && !bad) || length > TULIPS_CSUM_MAX_SEGMENT ||
      !mode_ok(mode, src, dst)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  LaunchArgs a{};
  a.seeds = seeds;
  a.src = src;
  a.dst = dst;
  a.out = out;
  a.bad = bad;
  a.n = n;
  a.mode = mode;
  apply_tuning(a, default_tuning(length, false), tuning);
  if (!geometry_ok(a.kind, a.group, a.unroll, a.spw, false) ||
      !fixed_block_ok(a.block)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return status_of(
    launch_fixed(base, stride, length, a, static_cast<hipStream_t>(stream)));
}

int
batch_var(const uint8_t* base, const uint64_t* offsets, const uint16_t* lengths,
          const uint16_t* seeds, const uint32_t* src, const uint32_t* dst,
          uint16_t* out, uint32_t* bad, uint32_t n, uint32_t mode,
          const tulips_csum_tuning* tuning, void* stream)
{
  if (n == 0) {
    return TULIPS_STATUS_OK;
  }
  if (!base || !offsets || !lengths || (!out && !bad) ||
      !mode_ok(mode, src, dst)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  LaunchArgs a{};
  a.seeds = seeds;
  a.src = src;
  a.dst = dst;
  a.out = out;
  a.bad = bad;
  a.n = n;
  a.mode = mode;
  apply_tuning(a, default_tuning(0, true), tuning);
  if (!geometry_ok(a.kind, a.group, a.unroll, a.spw, true) ||
      !block_ok(a.block)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return status_of(
    launch_var(base, offsets, lengths, a, static_cast<hipStream_t>(stream)));
}

// In-order arena batches (KIND_SPAN, csum_kernels.hip): the tuning's kind
// must be DEFAULT or SPAN; unroll = chunks per lane (4 KiB of arena per
// workgroup each), group 0 (or 7, the same form; include/tulips_csum.h).
int
batch_arena(const uint8_t* base, uint64_t arena, const uint64_t* offsets,
            const uint16_t* lengths, const uint16_t* seeds, const uint32_t* src,
            const uint32_t* dst, uint16_t* out, uint32_t* bad, uint32_t n, uint32_t mode,
            const tulips_csum_tuning* tuning, void* stream)
{
  if (n == 0) {
    return TULIPS_STATUS_OK;
  }
  if ((!base && arena) || !offsets || !lengths || (!out && !bad) ||
      !mode_ok(mode, src, dst)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (tuning && tuning->kind != TULIPS_CSUM_KIND_DEFAULT &&
      tuning->kind != TULIPS_CSUM_KIND_SPAN) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  LaunchArgs a{};
  a.seeds = seeds;
  a.src = src;
  a.dst = dst;
  a.out = out;
  a.bad = bad;
  a.n = n;
  a.mode = mode;
  a.kind = TULIPS_CSUM_KIND_SPAN;
  a.unroll = (tuning && tuning->unroll) ? tuning->unroll : SPAN_DEFAULT_UNROLL;
  a.group = (tuning && tuning->group) ? tuning->group : 0;
  if (!span_geometry_ok(a.unroll, a.group)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  a.spw = (tuning && a.group == 9) ? tuning->sps : 0; // tail-shaped: tail percent
  const int32_t nt = (tuning && tuning->nontemporal >= 0) ? tuning->nontemporal : 1;
  a.nontemporal = (nt & 1) != 0;
  a.nt_store = (nt & 2) != 0;
  return status_of(
    launch_span(base, arena, offsets, lengths, a, static_cast<hipStream_t>(stream)));
}

// A counting call: `launch(shards)` then the finalize into `count`, queued as
// one sequence under the stream's lock (stream_state.h).
template<class F>
int
counted(void* stream, uint32_t* count, const F& launch)
{
  hipStream_t st = static_cast<hipStream_t>(stream);
  std::shared_ptr<StreamState> ss;
  hipError_t e = stream_state(st, &ss);
  if (e != hipSuccess) {
    return status_of(e);
  }
  const bool capturing = stream_capturing(st);
  std::lock_guard<std::recursive_mutex> g(ss->call);
  uint32_t* shards = nullptr;
  if ((e = call_shards(*ss, capturing, &shards)) != hipSuccess) {
    return e == hipErrorStreamCaptureUnsupported ? TULIPS_STATUS_INVALID_ARGUMENT
                                                 : status_of(e);
  }
  int rc = launch(shards);
  if (rc == TULIPS_STATUS_OK) {
    // count = the shards' sum (0 for n == 0), shards zeroed again
    rc = status_of(launch_counters_finalize(shards, count, 1, st));
  }
  if (rc != TULIPS_STATUS_OK && !capturing) {
    drop_shards(*ss, shards);
  }
  return rc;
}

} // namespace

extern "C" {

int
tulips_csum_batch(const uint8_t* base, const uint64_t* offsets,
                  const uint16_t* lengths, const uint16_t* seeds,
                  const uint32_t* src, const uint32_t* dst, uint16_t* out,
                  uint32_t n, uint32_t mode, void* stream)
{
  if (n && !out) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return batch_var(base, offsets, lengths, seeds, src, dst, out, nullptr, n,
                   mode, nullptr, stream);
}

int
tulips_csum_batch_fixed(const uint8_t* base, uint64_t stride, uint32_t length,
                        const uint16_t* seeds, const uint32_t* src,
                        const uint32_t* dst, uint16_t* out, uint32_t n,
                        uint32_t mode, void* stream)
{
  if (n && !out) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return batch_fixed(base, stride, length, seeds, src, dst, out, nullptr, n,
                     mode, nullptr, stream);
}

int
tulips_csum_verify(const uint8_t* base, const uint64_t* offsets,
                   const uint16_t* lengths, const uint32_t* src,
                   const uint32_t* dst, uint16_t* out, uint32_t* bad_count,
                   uint32_t n, uint32_t mode, void* stream)
{
  const uint32_t m = mode & TULIPS_CSUM_MODE_MASK;
  if (!bad_count || (m != TULIPS_CSUM_INET && m != TULIPS_CSUM_TCP)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (n && (!base || !offsets || !lengths || !mode_ok(mode, src, dst))) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return counted(stream, bad_count, [&](uint32_t* shards) {
    return batch_var(base, offsets, lengths, nullptr, src, dst, out, shards, n, mode,
                     nullptr, stream);
  });
}

int
tulips_csum_batch_arena(const uint8_t* base, uint64_t arena_bytes,
                        const uint64_t* offsets, const uint16_t* lengths,
                        const uint16_t* seeds, const uint32_t* src, const uint32_t* dst,
                        uint16_t* out, uint32_t n, uint32_t mode, void* stream)
{
  if (n && !out) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return batch_arena(base, arena_bytes, offsets, lengths, seeds, src, dst, out, nullptr,
                     n, mode, nullptr, stream);
}

int
tulips_csum_verify_arena(const uint8_t* base, uint64_t arena_bytes,
                         const uint64_t* offsets, const uint16_t* lengths,
                         const uint32_t* src, const uint32_t* dst, uint16_t* out,
                         uint32_t* bad_count, uint32_t n, uint32_t mode, void* stream)
{
  const uint32_t m = mode & TULIPS_CSUM_MODE_MASK;
  if (!bad_count || (m != TULIPS_CSUM_INET && m != TULIPS_CSUM_TCP)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (n && ((!base && arena_bytes) || !offsets || !lengths || !mode_ok(mode, src, dst))) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return counted(stream, bad_count, [&](uint32_t* shards) {
    return batch_arena(base, arena_bytes, offsets, lengths, nullptr, src, dst, out,
                       shards, n, mode, nullptr, stream);
  });
}

int
tulips_csum_batch_arena_tuned(const uint8_t* base, uint64_t arena_bytes,
                              const uint64_t* offsets, const uint16_t* lengths,
                              const uint16_t* seeds, const uint32_t* src,
                              const uint32_t* dst, uint16_t* out, uint32_t n,
                              uint32_t mode, const tulips_csum_tuning* tuning,
                              void* stream)
{
  if (n && !out) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return batch_arena(base, arena_bytes, offsets, lengths, seeds, src, dst, out, nullptr,
                     n, mode, tuning, stream);
}

int
tulips_csum_default_tuning(uint32_t fixed_length, int variable,
                           tulips_csum_tuning* out)
{
  if (!out || fixed_length > TULIPS_CSUM_MAX_SEGMENT) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  *out = default_tuning(fixed_length, variable != 0);
  return TULIPS_STATUS_OK;
}

int
tulips_csum_batch_fixed_tuned(const uint8_t* base, uint64_t stride,
                              uint32_t length, const uint16_t* seeds,
                              const uint32_t* src, const uint32_t* dst,
                              uint16_t* out, uint32_t n, uint32_t mode,
                              const tulips_csum_tuning* tuning, void* stream)
{
  if (n && !out) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return batch_fixed(base, stride, length, seeds, src, dst, out, nullptr, n,
                     mode, tuning, stream);
}

int
tulips_csum_batch_tuned(const uint8_t* base, const uint64_t* offsets,
                        const uint16_t* lengths, const uint16_t* seeds,
                        const uint32_t* src, const uint32_t* dst,
                        uint16_t* out, uint32_t n, uint32_t mode,
                        const tulips_csum_tuning* tuning, void* stream)
{
  if (n && !out) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return batch_var(base, offsets, lengths, seeds, src, dst, out, nullptr, n,
                   mode, tuning, stream);
}

const char*
tulips_csum_status_string(int status)
{
  switch (status) {
    case TULIPS_STATUS_OK:
      return "Ok";
    case TULIPS_STATUS_INVALID_ARGUMENT:
      return "InvalidArgument";
    case TULIPS_STATUS_HARDWARE_ERROR:
      return "HardwareError";
    case TULIPS_STATUS_NO_MORE_RESOURCES:
      return "NoMoreResources";
    case TULIPS_STATUS_UNSUPPORTED_OPERATION:
      return "UnsupportedOperation";
    default:
      return "Unknown";
  }
}

const char*
tulips_csum_last_error(void)
{
  return last_error;
}

const char*
tulips_csum_version(void)
{
  return "tulips_amd-csum 0.1 gfx950";
}

} // extern "C"

