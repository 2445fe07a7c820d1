// zc_mailbox.h — the low-latency (zero-copy) receive-validation server's
// mailbox, shared by the host context (csum_host.hip) and the resident
// server kernel (frames.hip).
//
// A poll burst of a few frames costs the staged path (pinned staging copy,
// H2D, launch, D2H of the flags, event wait) ~28 us, more than the
// reference's CPU verify of one frame (~15 us). Here one workgroup stays
// resident and polls a doorbell in page-locked, host-coherent memory: the
// host copies the burst's offsets/lengths into the mailbox, bumps `seq`
// (release), and spins on `done`; the kernel reads the frames straight from
// the caller's page-locked arena over PCIe (no copies, no launch), writes
// the flags into the mailbox and publishes `done` (release, system scope).
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
constexpr uint32_t ZC_ARG_FRAMES = 64;

struct ZcArgs
{
  uint64_t base;                 // frames arena (GPU address)
  uint64_t seq;                  // the request being served
  uint32_t n;                    // frames
  uint32_t inline_n;             // n if <= ZC_ARG_FRAMES (descriptors below), else 0
  uint32_t off[ZC_ARG_FRAMES];   // frame offsets from base (inline form)
  uint16_t len[ZC_ARG_FRAMES];
};

struct alignas(64) ZcMailbox
{
  // request (host writes these, then `seq`)
  uint64_t base;        // frames arena, host address the GPU may read
  uint32_t n;           // frames
  uint32_t pad0;
  uint64_t pad1[6];
  // doorbell and stop (host -> GPU)
  alignas(64) uint64_t seq;
  uint64_t stop;
  uint64_t pad2[6];
  // completion (GPU -> host)
  alignas(64) uint64_t done;
  uint32_t counters[4];  // IPv4, bad IP csum, TCP, bad L4 csum of request `done`
  uint64_t beat;         // server heartbeat: polls / 1024 (diagnostics)
  uint64_t seen;         // last doorbell value the server read (diagnostics)
  uint64_t pad3[3];
  // per-frame arrays of the request
  alignas(64) uint64_t offs[ZC_MAX_FRAMES];
  uint16_t lens[ZC_MAX_FRAMES];
  uint8_t flags[ZC_MAX_FRAMES];
};

} // namespace tulips_amd
