// tulips::transport::gpucsum::Device — see the header for the contract.
// Host C++ over the C ABI of libtulips_csum (include/tulips_csum.h); no HIP
// or torch types cross into the reference's code.
#include <tulips/transport/gpucsum/Device.h>
#include <tulips_csum.h>
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>

namespace tulips::transport::gpucsum {

namespace {

constexpr size_t ALIGN = 16;

size_t
align_up(const size_t v)
{
  return (v + ALIGN - 1) & ~(ALIGN - 1);
}

}

Device::Device(system::Logger& log, transport::Device::Ref device,
               const int gpu, const uint32_t burst, const uint16_t hints)
  : transport::Device(log, "gpucsum")
  , m_device(std::move(device))
  , m_proc(nullptr)
  , m_ctx(nullptr)
  , m_burst(std::max<uint32_t>(burst, 1))
  , m_arena(nullptr)
  , m_capacity(0)
  , m_used(0)
  , m_offsets()
  , m_lengths()
  , m_stamps()
  , m_flags()
  , m_error(Status::Ok)
  , m_stats()
{
  m_hints |= hints;
  // Room for a whole burst of 2 KiB receive buffers (the OFED RX layout,
  // include/tulips/transport/ofed/Device.h:25) and always for one maximum
  // 64 KiB frame; a fuller arena is flushed early.
  m_capacity = std::max<size_t>(size_t(m_burst) * 2048, size_t(1) << 17);
  int rc = tulips_csum_ctx_create(gpu, m_capacity, &m_ctx);
  if (rc != TULIPS_STATUS_OK) {
    throw std::runtime_error(std::string("gpucsum: no GPU context: ") +
                             tulips_csum_status_string(rc) + " " +
                             tulips_csum_last_error());
  }
  void* p = nullptr;
  rc = tulips_csum_host_alloc(m_capacity, &p);
  if (rc != TULIPS_STATUS_OK) {
    tulips_csum_ctx_destroy(m_ctx);
    throw std::runtime_error("gpucsum: cannot allocate the staging arena");
  }
  m_arena = static_cast<uint8_t*>(p);
  m_offsets.reserve(m_burst);
  m_lengths.reserve(m_burst);
  m_stamps.reserve(m_burst);
  m_flags.resize(m_burst);
}

Device::~Device()
{
  tulips_csum_host_free(m_arena);
  tulips_csum_ctx_destroy(m_ctx);
}

Status
Device::process(const uint16_t len, const uint8_t* const data,
                const Timestamp ts)
{
  if (m_lengths.size() == m_burst || m_used + len > m_capacity) {
    const Status s = flush();
    if (s != Status::Ok && m_error == Status::Ok) {
      m_error = s;
    }
  }
  memcpy(m_arena + m_used, data, len);
  m_offsets.push_back(m_used);
  m_lengths.push_back(len);
  m_stamps.push_back(ts);
  m_used = align_up(m_used + len);
  m_stats.frames += 1;
  return Status::Ok;
}

Status
Device::sent(const uint16_t len, uint8_t* const buf)
{
  return m_proc->sent(len, buf);
}

/*
 * Pull frames from the inner device until it runs dry or a burst is staged.
 * Devices hand over one frame (list, npipe) or a completion batch (OFED,
 * ENA) per poll; the poll count is bounded by the burst either way.
 */
Status
Device::drain()
{
  for (uint32_t i = 0; i < m_burst && m_lengths.size() < m_burst; i += 1) {
    const Status s = m_device->poll(*this);
    if (s == Status::NoDataAvailable) {
      return Status::Ok;
    }
    if (s != Status::Ok) {
      return s;
    }
  }
  return Status::Ok;
}

/*
 * Validate the staged burst in one GPU batch and forward what passes.
 */
Status
Device::flush()
{
  const auto n = uint32_t(m_lengths.size());
  if (n == 0) {
    return Status::Ok;
  }
  const int rc = tulips_csum_validate_frames_host(
    m_ctx, m_arena, m_offsets.data(), m_lengths.data(), n, m_flags.data(),
    nullptr);
  m_stats.batches += 1;
  Status ret = Status::Ok;
  if (rc != TULIPS_STATUS_OK) {
    m_log.error("GPUCSUM", "batch validation failed: ",
                tulips_csum_status_string(rc), " ", tulips_csum_last_error());
    ret = rc == TULIPS_STATUS_NO_MORE_RESOURCES ? Status::NoMoreResources
                                                : Status::HardwareError;
  }
  for (uint32_t i = 0; ret == Status::Ok && i < n; i += 1) {
    const uint8_t fl = m_flags[i];
    if ((m_hints & VALIDATE_IP_CSUM) && (fl & TULIPS_FRAME_IPV4) &&
        !(fl & TULIPS_FRAME_IP_CSUM_OK)) {
      m_log.debug("GPUCSUM", "invalid IP checksum, dropping packet");
      m_stats.bad_ip += 1;
      continue;
    }
    if ((m_hints & VALIDATE_L4_CSUM) && (fl & TULIPS_FRAME_TCP) &&
        !(fl & TULIPS_FRAME_L4_CSUM_OK)) {
      m_log.debug("GPUCSUM", "invalid TCP checksum, dropping packet");
      m_stats.bad_l4 += 1;
      continue;
    }
    m_stats.forwarded += 1;
    const Status s =
      m_proc->process(m_lengths[i], m_arena + m_offsets[i], m_stamps[i]);
    if (s != Status::Ok && s != Status::UnsupportedProtocol &&
        m_error == Status::Ok) {
      m_log.error("GPUCSUM", "error processing buffer: ", toString(s));
      m_error = s;
    }
  }
  m_offsets.clear();
  m_lengths.clear();
  m_stamps.clear();
  m_used = 0;
  return ret;
}

Status
Device::poll(Processor& proc)
{
  m_proc = &proc;
  m_error = Status::Ok;
  const uint64_t before = m_stats.frames;
  const Status d = drain();
  const Status f = flush();
  if (d != Status::Ok) {
    return d;
  }
  if (f != Status::Ok) {
    return f;
  }
  if (m_error != Status::Ok) {
    return m_error;
  }
  return m_stats.frames == before ? Status::NoDataAvailable : Status::Ok;
}

Status
Device::wait(Processor& proc, const uint64_t ns)
{
  m_proc = &proc;
  m_error = Status::Ok;
  const uint64_t before = m_stats.frames;
  Status d = m_device->wait(*this, ns);
  if (d == Status::Ok) {
    d = drain();
  } else if (d == Status::NoDataAvailable) {
    d = Status::Ok;
  }
  const Status f = flush();
  if (d != Status::Ok) {
    return d;
  }
  if (f != Status::Ok) {
    return f;
  }
  if (m_error != Status::Ok) {
    return m_error;
  }
  return m_stats.frames == before ? Status::NoDataAvailable : Status::Ok;
}

}
