#pragma once
/*
 * tulips::transport::gpucsum::Device — batched receive-side checksum
 * validation on an MI355X.
 *
 * A transport decorator in the pattern of the reference's check::Device
 * (include/tulips/transport/check/Device.h, src/transport/check/Device.cpp:
 * 14-36): it wraps any transport::Device, drains up to `burst` frames per
 * poll from it into a page-locked staging arena, validates the whole burst
 * in one GPU launch (tulips_csum_validate_frames_zc / _host: Ethernet ->
 * IPv4 header checksum -> TCP pseudo-header checksum, include/tulips_csum.h;
 * bursts below Config::cpu_below frames and Config::cpu_below_bytes bytes
 * on the polling thread with the library's host code, tulips_csum_validate_frames_cpu, as the reference
 * would per frame), and forwards to the stack only the frames that pass, in
 * arrival order.
 *
 * It realises the Device::VALIDATE_IP_CSUM / VALIDATE_L4_CSUM hints
 * (include/tulips/transport/Device.h:29-30) the way the ENA and OFED
 * transports do with NIC offload bits (src/transport/ena/Device.cpp:
 * 316-340, src/transport/ofed/Device.cpp:528-545): a frame whose IPv4
 * header checksum fails is dropped under VALIDATE_IP_CSUM; a TCP frame whose
 * checksum fails, or that is shorter than its IP length announces, is
 * dropped under VALIDATE_L4_CSUM; everything else is forwarded untouched.
 * api::Client/Server set both hints when the stack is built with
 * TULIPS_DISABLE_CHECKSUM_CHECK (src/api/Client.cpp:39-41,
 * src/api/Server.cpp:32-34); the `hints` constructor argument sets them up
 * front for stacks that do not.
 *
 * Ownership follows the reference: the inner device's buffer is borrowed
 * only for the process() call, so each frame is copied into the staging
 * arena there; forwarded frames point into the arena and are valid for the
 * duration of the downstream process() call.
 *
 * Transmit side (Config::tx) — what a stack built with
 * TULIPS_HAS_HW_CHECKSUM expects of the NIC (IBV_SEND_IP_CSUM,
 * src/transport/ofed/Device.cpp:756): committed frames are staged, and at a
 * burst boundary (tx_burst frames), at the next poll()/wait(), or on
 * flushTransmit(), their IPv4 and TCP checksums are generated on the GPU in
 * one batch (tulips_csum_generate_frames_host) and the frames are committed
 * to the inner device in order. With Config::tso the decorator also plays
 * the NIC's TSO (TULIPS_HAS_HW_TSO, src/transport/ofed/Device.cpp:688-772):
 * mss() advertises `tso`-byte send buffers, which prepare() hands out from
 * its own pool, and a committed frame longer than the inner device's buffer
 * is cut on the GPU (tulips_csum_segment_frames_host) into frames of the
 * commit's MSS (0 or too large: the largest that fits the inner buffer, as
 * the OFED device adjusts it) with both checksums generated; the pieces are
 * copied into inner buffers and committed in order. The stack's sent()
 * callback for such a frame comes once all its pieces are sent.
 */

#include <tulips/transport/Device.h>
#include <tulips_csum.h>
#include <cstdint>
#include <unordered_map>
#include <unordered_set>
#include <vector>

struct tulips_csum_ctx;

namespace tulips::transport::gpucsum {

class Device
  : public transport::Device
  , public Processor
{
public:
  struct Statistics
  {
    uint64_t frames = 0;     // received from the inner device
    uint64_t forwarded = 0;  // handed to the stack
    uint64_t bad_ip = 0;     // dropped: IPv4 header checksum
    uint64_t bad_l4 = 0;     // dropped: TCP checksum / truncation
    uint64_t batches = 0;    // GPU launches
    uint64_t cpu_batches = 0; // bursts below the crossover, validated on the host
    uint64_t tx_frames = 0;  // committed by the stack (tx)
    uint64_t tx_segments = 0; // frames committed to the inner device (tx)
    uint64_t tx_batches = 0; // GPU batches on the transmit side
  };

  static constexpr uint32_t DEFAULT_BURST = 1024;
  // bursts up to this size take the zero-copy path (on MI355X it beats the
  // staged one at every burst size up to its 1,024-frame limit: INTEGRATION.md
  // §3, the latency-per-burst table)
  static constexpr uint32_t DEFAULT_LOWLAT = 1024;
  // bursts of fewer frames (and bytes) are validated on the polling thread
  // by the library's host code (tulips_csum_validate_frames_cpu): below
  // this size a PCIe round trip to the GPU costs more than the per-frame
  // checks do on the CPU. The library's measured crossover
  // (tulips_csum_burst_prefers_cpu, include/tulips_csum.h): cold 1514 B
  // frames cost ~0.15 us each on the host against ~13 us + 0.02 us each on
  // the zero-copy path, crossing near 96 frames
  static constexpr uint32_t DEFAULT_CPU_BELOW = TULIPS_CSUM_CPU_BELOW_FRAMES;
  static constexpr uint64_t DEFAULT_CPU_BELOW_BYTES = TULIPS_CSUM_CPU_BELOW_BYTES;

  struct Config
  {
    int gpu = 0;
    uint32_t burst = DEFAULT_BURST; // receive: frames per GPU batch
    uint16_t hints = 0;             // VALIDATE_* set up front
    bool tx = false;                // transmit: checksums generated on the GPU
    uint32_t tx_burst = 64;         // transmit: frames per GPU batch
    uint32_t tso = 0;               // > 0: TSO with send buffers of this size
    // receive: bursts of at most this many frames go through the resident
    // low-latency server (tulips_csum_validate_frames_zc: frames read in
    // place from the pinned staging arena, no copies or launch); 0 = never
    uint32_t lowlat = DEFAULT_LOWLAT;
    // ... served by workgroups resident on the GPU (no launch per burst)
    bool lowlat_resident = false;
    // receive: bursts of fewer frames AND fewer bytes stay on the CPU;
    // cpu_below 0 = always the GPU
    uint32_t cpu_below = DEFAULT_CPU_BELOW;
    uint64_t cpu_below_bytes = DEFAULT_CPU_BELOW_BYTES;
  };

  static Ref allocate(system::Logger& log, transport::Device::Ref device,
                      const int gpu = 0, const uint32_t burst = DEFAULT_BURST,
                      const uint16_t hints = 0)
  {
    Config c;
    c.gpu = gpu;
    c.burst = burst;
    c.hints = hints;
    return std::make_unique<Device>(log, std::move(device), c);
  }

  static Ref allocate(system::Logger& log, transport::Device::Ref device,
                      Config const& config)
  {
    return std::make_unique<Device>(log, std::move(device), config);
  }

  /*
   * Throws std::runtime_error when the GPU context cannot be created (no
   * device, no libtulips_csum). Bursts below Config::cpu_below are a latency
   * choice made per burst, not a fallback: every larger burst goes to the
   * GPU, and a GPU failure is reported as HardwareError, never retried on
   * the CPU.
   */
  Device(system::Logger& log, transport::Device::Ref device, Config const& config);
  ~Device() override;

  /*
   * Device interface: everything but poll/wait passes through.
   */

  std::string_view name() const override { return m_device->name(); }

  stack::ethernet::Address const& address() const override
  {
    return m_device->address();
  }

  Status listen(const stack::ipv4::Protocol proto,
                stack::ipv4::Address const& laddr, const uint16_t lport,
                stack::ipv4::Address const& raddr,
                const uint16_t rport) override
  {
    return m_device->listen(proto, laddr, lport, raddr, rport);
  }

  void unlisten(const stack::ipv4::Protocol proto,
                stack::ipv4::Address const& laddr, const uint16_t lport,
                stack::ipv4::Address const& raddr,
                const uint16_t rport) override
  {
    m_device->unlisten(proto, laddr, lport, raddr, rport);
  }

  Status poll(Processor& proc) override;
  Status wait(Processor& proc, const uint64_t ns) override;

  uint32_t mtu() const override { return m_device->mtu(); }
  uint32_t mss() const override { return m_tso ? m_tso : m_device->mss(); }

  uint8_t receiveBufferLengthLog2() const override
  {
    return m_device->receiveBufferLengthLog2();
  }

  uint16_t receiveBuffersAvailable() const override
  {
    return m_device->receiveBuffersAvailable();
  }

  bool identify(const uint8_t* const buf) const override
  {
    return m_device->identify(buf);
  }

  Status prepare(uint8_t*& buf) override;
  Status commit(const uint16_t len, uint8_t* const buf,
                const uint16_t mss = 0) override;
  Status release(uint8_t* const buf) override;

  /*
   * Generate (and segment) the staged transmit burst on the GPU now and
   * commit it to the inner device. No-op without Config::tx.
   */
  Status flushTransmit();

  Statistics const& statistics() const { return m_stats; }

private:
  Status run() override { return Status::Ok; }
  Status process(const uint16_t len, const uint8_t* const data,
                 const Timestamp ts) override;
  Status sent(const uint16_t len, uint8_t* const buf) override;

  Status drain();
  Status flush();
  Status commitPiece(const uint8_t* data, uint16_t len, uint8_t* own, uint16_t mss);

  struct Pending
  {
    uint8_t* buf;
    uint16_t len;
    uint16_t mss;
  };

  transport::Device::Ref m_device;
  Processor* m_proc;
  tulips_csum_ctx* m_ctx;
  uint32_t m_burst;
  uint8_t* m_arena;
  size_t m_capacity;
  size_t m_used;
  std::vector<uint64_t> m_offsets;
  std::vector<uint16_t> m_lengths;
  std::vector<Timestamp> m_stamps;
  std::vector<uint8_t> m_flags;
  Status m_error;
  Statistics m_stats;
  // transmit
  bool m_tx;
  uint32_t m_tx_burst;
  uint32_t m_tso;
  uint32_t m_lowlat;
  uint32_t m_cpu_below;
  uint64_t m_cpu_below_bytes;
  std::vector<Pending> m_pending;
  std::unordered_set<uint8_t*> m_own;        // our TSO send buffers
  std::vector<uint8_t*> m_free;              // ... not handed out
  std::unordered_map<uint8_t*, uint8_t*> m_piece_of; // inner buf -> our buf
  std::unordered_map<uint8_t*, std::pair<uint32_t, uint16_t>> m_inflight;
  std::vector<uint64_t> m_tx_offsets;
  std::vector<uint16_t> m_tx_lengths;
  std::vector<uint8_t> m_tx_flags;
  std::vector<uint8_t> m_seg_out;
  std::vector<uint16_t> m_seg_lengths;
  std::vector<uint32_t> m_seg_first;
};

}
