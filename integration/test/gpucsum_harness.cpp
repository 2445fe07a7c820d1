// TEST INFRASTRUCTURE — drives tulips::transport::gpucsum::Device the way
// the reference's stack does: frames committed on one reference
// list::Device (src/transport/list/Device.cpp) arrive on its peer, which is
// wrapped by the decorator; a recording Processor stands where the stack's
// ethernet::Processor would. Called from tests/test_gpucsum_device.py.
#include <tulips/stack/Ethernet.h>
#include <tulips/system/Logger.h>
#include <tulips/transport/gpucsum/Device.h>
#include <tulips/transport/list/Device.h>
#include <cstdio>
#include <cstring>
#include <exception>
#include <vector>

using namespace tulips;

namespace {

uint64_t
fnv1a(const uint8_t* p, size_t n)
{
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < n; ++i) {
    h = (h ^ p[i]) * 0x100000001b3ull;
  }
  return h;
}

struct Recorder : transport::Processor
{
  std::vector<std::pair<uint16_t, uint64_t>> got;
  uint64_t sent_count = 0;

  Status run() override { return Status::Ok; }

  Status process(const uint16_t len, const uint8_t* const data,
                 const Timestamp) override
  {
    got.emplace_back(len, fnv1a(data, len));
    return Status::Ok;
  }

  Status sent(const uint16_t, uint8_t* const) override
  {
    sent_count += 1;
    return Status::Ok;
  }
};

constexpr uint32_t LIST_MTU = 65536;

int run_cfg(const uint8_t* arena, const uint64_t* offs, const uint16_t* lens, uint32_t n,
            uint32_t burst, uint16_t hints, int use_wait, int64_t cpu_below,
            uint8_t* forwarded, uint64_t* stats);

}

extern "C" int
gpucsum_run(const uint8_t* arena, const uint64_t* offs, const uint16_t* lens,
            uint32_t n, uint32_t burst, uint16_t hints, int use_wait,
            uint8_t* forwarded, uint64_t* stats)
{
  return run_cfg(arena, offs, lens, n, burst, hints, use_wait, -1, forwarded, stats);
}

// gpucsum_run with Config::cpu_below set (-1: the decorator's default
// crossover, frames and bytes; otherwise that many frames and no bytes
// limit); stats[5] = cpu_batches.
extern "C" int
gpucsum_run_cpu_below(const uint8_t* arena, const uint64_t* offs, const uint16_t* lens,
                      uint32_t n, uint32_t burst, uint16_t hints, int64_t cpu_below,
                      uint8_t* forwarded, uint64_t* stats)
{
  stats[5] = 0;
  const int rc = run_cfg(arena, offs, lens, n, burst, hints, 0, cpu_below < 0 ? -2 : cpu_below,
                         forwarded, stats);
  return rc;
}

namespace {

int
run_cfg(const uint8_t* arena, const uint64_t* offs, const uint16_t* lens, uint32_t n,
        uint32_t burst, uint16_t hints, int use_wait, int64_t cpu_below,
        uint8_t* forwarded, uint64_t* stats)
{
  try {
    system::ConsoleLogger log(system::Logger::Level::Error);
    transport::list::Device::List a2b, b2a;
    stack::ethernet::Address mac(0x02, 0, 0, 0, 0, 1);
    auto peer = transport::list::Device::allocate(log, mac, LIST_MTU, b2a, a2b);
    auto rx = transport::list::Device::allocate(log, mac, LIST_MTU, a2b, b2a);
    for (uint32_t i = 0; i < n; ++i) {
      uint8_t* buf = nullptr;
      if (peer->prepare(buf) != Status::Ok) {
        return -3;
      }
      memcpy(buf, arena + offs[i], lens[i]);
      if (peer->commit(lens[i], buf, 0) != Status::Ok) {
        return -3;
      }
    }
    transport::gpucsum::Device::Config cfg;
    cfg.burst = burst;
    cfg.hints = hints;
    if (cpu_below >= 0) {
      cfg.cpu_below = uint32_t(cpu_below);
      cfg.cpu_below_bytes = UINT64_MAX;
    }
    transport::gpucsum::Device dev(log, std::move(rx), cfg);
    Recorder rec;
    Status s = Status::Ok;
    for (uint64_t it = 0; it <= uint64_t(n) + 2; ++it) {
      s = use_wait ? dev.wait(rec, 1000) : dev.poll(rec);
      if (s != Status::Ok) {
        break;
      }
    }
    if (s != Status::NoDataAvailable) {
      fprintf(stderr, "gpucsum_run: poll ended with %s\n", toString(s).c_str());
      return -4;
    }
    // Forwarded frames keep arrival order: match them to the inputs.
    memset(forwarded, 0, n);
    uint32_t j = 0;
    for (auto const& [len, h] : rec.got) {
      while (j < n && !(lens[j] == len && fnv1a(arena + offs[j], lens[j]) == h)) {
        ++j;
      }
      if (j == n) {
        return -2;
      }
      forwarded[j++] = 1;
    }
    auto const& st = dev.statistics();
    stats[0] = st.frames;
    stats[1] = st.forwarded;
    stats[2] = st.bad_ip;
    stats[3] = st.bad_l4;
    stats[4] = st.batches;
    if (cpu_below >= 0 || cpu_below == -2) { // -2: default crossover, stats[5] wanted
      stats[5] = st.cpu_batches;
    }
    return 0;
  } catch (std::exception const& e) {
    fprintf(stderr, "gpucsum_run: %s\n", e.what());
    return -1;
  }
}

}

// Transmit side: the stack's frames (arena/offs/lens, checksum fields as the
// sender left them) are prepared on and committed to a gpucsum::Device with
// Config::tx (and Config::tso = `tso` if non-zero) over a list::Device whose
// buffers hold `wire_mtu` bytes; `mss` is the commit's MSS. The frames that
// reach the wire (the peer's read list) are copied out back to back into
// `out` (capacity `out_cap` bytes) with their lengths in out_lens (at most
// `out_n`). stats = { tx_frames, tx_segments, tx_batches, sent callbacks for
// the stack's buffers, buffers released }. Returns the number of wire frames
// or < 0 on failure.
extern "C" int64_t
gpucsum_tx_run(const uint8_t* arena, const uint64_t* offs, const uint16_t* lens,
               uint32_t n, uint16_t mss, uint32_t tx_burst, uint32_t tso,
               uint32_t wire_mtu, uint8_t* out, uint64_t out_cap, uint16_t* out_lens,
               uint32_t out_n, uint64_t* stats)
{
  try {
    system::ConsoleLogger log(system::Logger::Level::Error);
    transport::list::Device::List a2b, b2a;
    stack::ethernet::Address mac(0x02, 0, 0, 0, 0, 1);
    auto inner = transport::list::Device::allocate(log, mac, wire_mtu, b2a, a2b);
    transport::gpucsum::Device::Config cfg;
    cfg.tx = true;
    cfg.tx_burst = tx_burst;
    cfg.tso = tso;
    transport::gpucsum::Device dev(log, std::move(inner), cfg);
    std::vector<uint8_t*> bufs;
    for (uint32_t i = 0; i < n; ++i) {
      uint8_t* buf = nullptr;
      if (dev.prepare(buf) != Status::Ok) {
        return -3;
      }
      memcpy(buf, arena + offs[i], lens[i]);
      bufs.push_back(buf);
      if (dev.commit(lens[i], buf, mss) != Status::Ok) {
        return -4;
      }
    }
    if (dev.flushTransmit() != Status::Ok) {
      return -5;
    }
    // the list device reports its committed buffers as sent on the next
    // poll; the stack (here: the recorder) then releases them
    Recorder rec;
    Status s = dev.poll(rec);
    if (s != Status::Ok && s != Status::NoDataAvailable) {
      return -6;
    }
    uint64_t released = 0;
    for (uint8_t* b : bufs) {
      if (dev.release(b) == Status::Ok) {
        released += 1;
      }
    }
    uint64_t at = 0;
    int64_t k = 0;
    for (auto* p : a2b) {
      if (uint32_t(k) >= out_n || at + p->len > out_cap) {
        return -7;
      }
      memcpy(out + at, p->data, p->len);
      out_lens[k++] = uint16_t(p->len);
      at += p->len;
    }
    for (auto* p : a2b) {
      transport::list::Device::Packet::release(p);
    }
    auto const& st = dev.statistics();
    stats[0] = st.tx_frames;
    stats[1] = st.tx_segments;
    stats[2] = st.tx_batches;
    stats[3] = rec.sent_count;
    stats[4] = released;
    return k;
  } catch (std::exception const& e) {
    fprintf(stderr, "gpucsum_tx_run: %s\n", e.what());
    return -1;
  }
}
