// zc_mailbox.h — the low-latency (zero-copy) receive-validation server's
// mailbox, shared by the host context (csum_host.hip) and the resident
// server kernel (frames.hip).
//
// A poll burst of a few frames costs the staged path (pinned staging copy,
// H2D, launch, D2H of the flags, event wait) ~28 us. Here the frames are read
// straight from the caller's page-locked arena over PCIe (no copies) by one
// workgroup, which writes the flags into this page-locked, host-coherent
// mailbox and publishes `done` (release, system scope) while the host spins
// on it. Either one launch per burst carries the request in its kernel
// arguments (ZcArgs), or one workgroup stays resident and polls the tagged
// doorbell words below (no launch at all).
// The server exits when `stop` is set or after ZC_IDLE_TICKS of silence
// (every wave reaches that exit: no kernel outlives an abandoned context);
// the host relaunches it on the next burst.
#pragma once

#include <stdint.h>

namespace tulips_amd {

constexpr uint32_t ZC_MAX_FRAMES = 1024;              // frames per request
constexpr uint64_t ZC_STAGING = 2ull << 20;           // packed bursts (pageable callers)
constexpr uint64_t ZC_IDLE_TICKS = 100ull * 100000;   // 100 ms of s_memrealtime (100 MHz)

// One launch per burst: the request itself rides in the kernel arguments
// (kernarg memory is device-resident), so a burst of up to ZC_ARG_FRAMES
// frames costs the frame reads and the flag writes over PCIe, nothing else.
constexpr uint32_t ZC_ARG_FRAMES = 62; // = ZC_REQ_FRAMES: the kernel builds the 64 doorbell words from them

struct ZcArgs
{
  uint64_t base;                 // frames arena (GPU address)
  uint64_t seq;                  // the request's 16-bit tag (published in `done`)
  uint32_t n;                    // frames
  uint32_t inline_n;             // n if <= ZC_ARG_FRAMES (descriptors below), else 0
                                 // (then ZcMailbox offs / lens, from `base`)
  uint32_t off[ZC_ARG_FRAMES];   // frame offsets from base (inline form)
  uint16_t len[ZC_ARG_FRAMES];
};

// Resident server doorbell: 64 tagged words, read by one wave load (a word
// per lane) on every poll. Each word carries the request's 16-bit tag in its
// top bits and is stored atomically by the host, so a poll that finds every
// word it needs carrying the new tag has a consistent request, and a poll
// that catches the host mid-write simply polls again: the request is known
// one PCIe round trip after the host posts it.
//   req[0] = tag << 48 | n             (n frames)
//   req[1] = tag << 48 | base          (GPU address of frame 0's arena, < 2^48)
//   req[2 + k] = tag << 48 | off << 16 | len   for k < n <= ZC_REQ_FRAMES
// Larger bursts put their descriptors in `offs` / `lens` (written before the
// tagged words; offsets there are from `base`).
constexpr uint32_t ZC_REQ_WORDS = 64, ZC_REQ_FRAMES = ZC_REQ_WORDS - 2;
static_assert(ZC_ARG_FRAMES == ZC_REQ_FRAMES, "one wave turns the arguments into the words");

__host__ __device__ inline uint64_t
zc_word(uint32_t tag, uint64_t payload)
{
  return (uint64_t(tag & 0xffffu) << 48) | (payload & 0xffffffffffffull);
}

// Workgroups serving one request: a resident server keeps ZC_RES_WG of them
// (each polls the doorbell, takes every ZC_RES_WG-th group of 64 frames and
// publishes its own completion word); one launch per burst uses one per 64
// frames, up to ZC_MAX_WG. More than one CU keeps more PCIe reads in flight
// than one CU can (a 64-frame burst read by one CU: ~7.5 GB/s).
constexpr uint32_t ZC_MAX_WG = 16, ZC_RES_WG = 8;

struct alignas(64) ZcMailbox
{
  alignas(64) uint64_t req[ZC_REQ_WORDS];
  // stop (host -> GPU)
  alignas(64) uint64_t stop;
  uint64_t pad2[7];
  // completion (GPU -> host), per workgroup: the tag of the last request
  // it finished and that request's counts {IPv4, bad IP csum, TCP, bad L4}
  alignas(64) uint64_t done[ZC_MAX_WG];
  uint32_t counters[ZC_MAX_WG][4];
  // diagnostics (workgroup 0)
  uint64_t beat;         // server heartbeat: polls / 1024
  uint64_t seen;         // last doorbell tag the server read
  uint64_t t_req;        // s_memrealtime when the request was picked up
  uint64_t t_done;       // ... and when its flags were out
  // per-frame arrays of bursts past ZC_REQ_FRAMES
  alignas(64) uint64_t offs[ZC_MAX_FRAMES];
  uint16_t lens[ZC_MAX_FRAMES];
  uint8_t flags[ZC_MAX_FRAMES];
};

} // namespace tulips_amd
