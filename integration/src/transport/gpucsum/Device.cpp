// tulips::transport::gpucsum::Device — see the header for the contract.
// Host C++ over the C ABI of libtulips_csum (include/tulips_csum.h); no HIP
// or torch types cross into the reference's code.
#include <tulips/transport/gpucsum/Device.h>
#include <tulips_csum.h>
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

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
               Config const& config)
  : transport::Device(log, "gpucsum")
  , m_device(std::move(device))
  , m_proc(nullptr)
  , m_ctx(nullptr)
  , m_burst(std::max<uint32_t>(config.burst, 1))
  , m_arena(nullptr)
  , m_capacity(0)
  , m_used(0)
  , m_offsets()
  , m_lengths()
  , m_stamps()
  , m_flags()
  , m_error(Status::Ok)
  , m_stats()
  , m_tx(config.tx || config.tso != 0)
  , m_tx_burst(std::max<uint32_t>(config.tx_burst, 1))
  , m_tso(config.tso ? std::max<uint32_t>(config.tso, m_device->mss()) : 0)
  , m_lowlat(config.lowlat)
  , m_cpu_below(config.cpu_below)
  , m_cpu_below_bytes(config.cpu_below_bytes)
{
  m_hints |= config.hints;
  // Room for a whole burst of 2 KiB receive buffers (the OFED RX layout,
  // include/tulips/transport/ofed/Device.h:25) and always for one maximum
  // 64 KiB frame; a fuller arena is flushed early.
  m_capacity = std::max<size_t>(size_t(m_burst) * 2048, size_t(1) << 17);
  int rc = tulips_csum_ctx_create(config.gpu, m_capacity, &m_ctx);
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
  if (config.lowlat_resident) {
    tulips_csum_ctx_set_lowlat(m_ctx, 1);
  }
  m_offsets.reserve(m_burst);
  m_lengths.reserve(m_burst);
  m_stamps.reserve(m_burst);
  m_flags.resize(m_burst);
  m_pending.reserve(m_tx_burst);
}

Device::~Device()
{
  for (uint8_t* b : m_own) {
    tulips_csum_host_free(b);
  }
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
  const auto it = m_piece_of.find(buf);
  if (it == m_piece_of.end()) {
    return m_proc->sent(len, buf);
  }
  // a piece we committed for one of our send buffers: give the inner buffer
  // back, and report the stack's buffer once all its pieces are out
  uint8_t* own = it->second;
  m_piece_of.erase(it);
  m_device->release(buf);
  auto f = m_inflight.find(own);
  if (f == m_inflight.end() || --f->second.first > 0) {
    return Status::Ok;
  }
  const uint16_t olen = f->second.second;
  m_inflight.erase(f);
  return m_proc->sent(olen, own);
}

// ---------------------------------------------------------------------------
// Transmit side.
// ---------------------------------------------------------------------------

Status
Device::prepare(uint8_t*& buf)
{
  if (!m_tso) {
    return m_device->prepare(buf);
  }
  if (m_free.empty()) {
    void* p = nullptr;
    if (tulips_csum_host_alloc(m_tso, &p) != TULIPS_STATUS_OK) {
      return Status::NoMoreResources;
    }
    m_own.insert(static_cast<uint8_t*>(p));
    m_free.push_back(static_cast<uint8_t*>(p));
  }
  buf = m_free.back();
  m_free.pop_back();
  return Status::Ok;
}

Status
Device::release(uint8_t* const buf)
{
  if (m_own.count(buf)) {
    m_free.push_back(buf);
    return Status::Ok;
  }
  return m_device->release(buf);
}

Status
Device::commit(const uint16_t len, uint8_t* const buf, const uint16_t mss)
{
  if (!m_tx) {
    return m_device->commit(len, buf, mss);
  }
  m_pending.push_back({ buf, len, mss });
  m_stats.tx_frames += 1;
  return m_pending.size() >= m_tx_burst ? flushTransmit() : Status::Ok;
}

// Copy `data` into a fresh inner buffer and commit it there, on behalf of our
// send buffer `own` (sent() reports `own` when its last piece is out).
Status
Device::commitPiece(const uint8_t* data, const uint16_t len, uint8_t* own,
                    const uint16_t mss)
{
  uint8_t* ib = nullptr;
  Status s = m_device->prepare(ib);
  if (s != Status::Ok) {
    return s;
  }
  memcpy(ib, data, len);
  m_piece_of[ib] = own;
  m_inflight[own].first += 1;
  m_stats.tx_segments += 1;
  return m_device->commit(len, ib, mss);
}

namespace {

// stack::utils::headerLength (src/stack/Utils.cpp:67-84): Ethernet + IPv4 +
// TCP header bytes of an option-less IPv4 / TCP frame, 0 otherwise.
uint32_t
tcp_header_length(const uint8_t* f, const uint32_t len)
{
  if (len < 54 || f[12] != 0x08 || f[13] != 0x00 || f[14] != 0x45 || f[23] != 6) {
    return 0;
  }
  return 34 + 4u * (f[46] >> 4);
}

}

Status
Device::flushTransmit()
{
  if (!m_tx || m_pending.empty()) {
    return Status::Ok;
  }
  std::vector<Pending> batch;
  batch.swap(m_pending);
  const uint32_t cap = m_device->mss(); // the inner device's send buffer
  // 1. checksum generation, in place, for every frame that fits the inner
  //    device as it is: one GPU batch
  uint8_t* base = nullptr;
  for (auto const& p : batch) {
    if (p.len <= cap && (!base || p.buf < base)) {
      base = p.buf;
    }
  }
  m_tx_offsets.clear();
  m_tx_lengths.clear();
  for (auto const& p : batch) {
    if (p.len <= cap) {
      m_tx_offsets.push_back(uint64_t(p.buf - base));
      m_tx_lengths.push_back(p.len);
    }
  }
  Status ret = Status::Ok;
  if (!m_tx_offsets.empty()) {
    m_tx_flags.resize(m_tx_offsets.size());
    const int rc = tulips_csum_generate_frames_host(
      m_ctx, base, m_tx_offsets.data(), m_tx_lengths.data(),
      uint32_t(m_tx_offsets.size()), m_tx_flags.data());
    m_stats.tx_batches += 1;
    if (rc != TULIPS_STATUS_OK) {
      m_log.error("GPUCSUM", "transmit generation failed: ",
                  tulips_csum_status_string(rc), " ", tulips_csum_last_error());
      return rc == TULIPS_STATUS_NO_MORE_RESOURCES ? Status::NoMoreResources
                                                   : Status::HardwareError;
    }
  }
  // 2. segmentation of the super-frames (our TSO buffers), one GPU batch per
  //    distinct MSS, pieces written to slots of the inner buffer's size
  const uint64_t stride = (uint64_t(cap) + 15) & ~uint64_t(15);
  std::vector<std::pair<uint32_t, uint32_t>> pieces(batch.size(), { 0, 0 });
  std::unordered_map<uint32_t, std::vector<uint32_t>> by_mss;
  for (uint32_t i = 0; i < batch.size(); ++i) {
    auto const& p = batch[i];
    if (p.len <= cap) {
      continue;
    }
    const uint32_t hl = tcp_header_length(p.buf, p.len);
    if (hl == 0 || hl >= cap) {
      m_log.error("GPUCSUM", "cannot segment a ", p.len, "B frame");
      ret = Status::IncompleteData;
      continue;
    }
    uint32_t lmss = p.mss;
    if (lmss == 0 || lmss > cap - hl) {
      lmss = cap - hl; // as the OFED device adjusts it
    }
    by_mss[lmss].push_back(i);
  }
  m_seg_out.clear();
  m_seg_lengths.clear();
  for (auto const& [lmss, idx] : by_mss) {
    uint8_t* sb = nullptr;
    uint64_t bound = 0;
    for (uint32_t i : idx) {
      sb = (!sb || batch[i].buf < sb) ? batch[i].buf : sb;
      bound += batch[i].len / lmss + 1;
    }
    m_tx_offsets.clear();
    m_tx_lengths.clear();
    for (uint32_t i : idx) {
      m_tx_offsets.push_back(uint64_t(batch[i].buf - sb));
      m_tx_lengths.push_back(batch[i].len);
    }
    const size_t at = m_seg_lengths.size();
    m_seg_out.resize(size_t((at + bound) * stride));
    m_seg_lengths.resize(size_t(at + bound));
    m_seg_first.resize(idx.size() + 1);
    const int rc = tulips_csum_segment_frames_host(
      m_ctx, sb, m_tx_offsets.data(), m_tx_lengths.data(), uint32_t(idx.size()), lmss,
      m_seg_out.data() + at * stride, stride, uint32_t(bound), m_seg_lengths.data() + at,
      m_seg_first.data());
    m_stats.tx_batches += 1;
    if (rc != TULIPS_STATUS_OK) {
      m_log.error("GPUCSUM", "transmit segmentation failed: ",
                  tulips_csum_status_string(rc), " ", tulips_csum_last_error());
      return rc == TULIPS_STATUS_NO_MORE_RESOURCES ? Status::NoMoreResources
                                                   : Status::HardwareError;
    }
    for (size_t k = 0; k < idx.size(); ++k) {
      pieces[idx[k]] = { uint32_t(at + m_seg_first[k]), m_seg_first[k + 1] - m_seg_first[k] };
    }
    m_seg_lengths.resize(at + m_seg_first[idx.size()]);
  }
  // 3. commit everything to the inner device in the stack's order
  for (uint32_t i = 0; i < batch.size(); ++i) {
    auto const& p = batch[i];
    Status s = Status::Ok;
    if (p.len <= cap) {
      s = m_own.count(p.buf) ? commitPiece(p.buf, p.len, p.buf, 0)
                             : (m_stats.tx_segments += 1, m_device->commit(p.len, p.buf, p.mss));
      if (m_own.count(p.buf) && s == Status::Ok) {
        m_inflight[p.buf].second = p.len;
      }
    } else {
      for (uint32_t k = 0; k < pieces[i].second && s == Status::Ok; ++k) {
        const uint32_t j = pieces[i].first + k;
        if (m_seg_lengths[j] == 0) {
          s = Status::IncompleteData; // did not fit a slot
          break;
        }
        s = commitPiece(m_seg_out.data() + uint64_t(j) * stride, m_seg_lengths[j], p.buf, 0);
      }
      if (s == Status::Ok && pieces[i].second) {
        m_inflight[p.buf].second = p.len;
      }
    }
    if (s != Status::Ok && ret == Status::Ok) {
      ret = s;
    }
  }
  return ret;
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
  // tiny bursts on this thread (cheaper than a PCIe round trip), small
  // ones read in place from the pinned arena by the zero-copy path, large
  // ones staged through the context's DMA pipeline
  int rc;
  uint64_t bytes = 0;
  if (n < m_cpu_below) {
    for (uint32_t i = 0; i < n; ++i) {
      bytes += m_lengths[i];
    }
  }
  if (n < m_cpu_below && bytes < m_cpu_below_bytes) {
    rc = tulips_csum_validate_frames_cpu(m_arena, m_offsets.data(), m_lengths.data(), n,
                                         m_flags.data(), nullptr);
    m_stats.cpu_batches += 1;
  } else {
    rc = n <= m_lowlat
           ? tulips_csum_validate_frames_zc(m_ctx, m_arena, m_offsets.data(),
                                            m_lengths.data(), n, m_flags.data(), nullptr)
           : tulips_csum_validate_frames_host(m_ctx, m_arena, m_offsets.data(),
                                              m_lengths.data(), n, m_flags.data(), nullptr);
    m_stats.batches += 1;
  }
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
  const Status t = flushTransmit();
  if (t != Status::Ok) {
    return t;
  }
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
  const Status t = flushTransmit();
  if (t != Status::Ok) {
    return t;
  }
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
