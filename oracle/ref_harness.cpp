// ref_harness.cpp — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
//
// A C-linkage harness around the reference's OWN checksum functions. It is
// linked (oracle/Makefile) with the reference's src/stack + src/system
// sources, compiled where they lie under /root/reference, into
// oracle/_ref/libtulips_ref.so. Nothing from the reference is copied here;
// this file only declares entry points and calls them.
//
//   ref_checksum        -> tulips::stack::utils::checksum   (src/stack/Utils.cpp:14-42)
//   ref_ipv4_checksum   -> tulips::stack::ipv4::checksum    (src/stack/IPv4.cpp:75-82)
//   ref_icmpv4_checksum -> tulips::stack::icmpv4::checksum  (src/stack/ICMPv4.cpp:10-15)
//   ref_tcp_checksum    -> tulips::stack::tcpv4::Processor::checksum
//                          (private static, src/stack/tcpv4/Processor.cpp:337-357),
//                          reached through its exported symbol.
//   ref_batch           -> the reference's per-segment call pattern (one a1/a2
//                          call per segment, as the stack does per frame,
//                          src/stack/tcpv4/Processor.cpp:121) over a batch, on
//                          N std::threads pinned to distinct cores: the CPU
//                          baseline bench.py reports ("kind": "reference").
#include <tulips/stack/ICMPv4.h>
#include <tulips/stack/IPv4.h>
#include <tulips/stack/Utils.h>
#include <arpa/inet.h>
#include <pthread.h>
#include <sched.h>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <chrono>
#include <thread>
#include <vector>

// tcpv4::Processor::checksum is a private static member: call its exported
// symbol directly. The ipv4::Address arguments are passed by const reference,
// i.e. as pointers to the 4-byte m_data word (include/tulips/stack/IPv4.h:55).
extern "C" uint16_t
_ZN6tulips5stack5tcpv49Processor8checksumERKNS0_4ipv47AddressES6_tPKh(
  const void* src, const void* dst, uint16_t len, const uint8_t* data);

namespace {

constexpr uint32_t MODE_RAW = 0, MODE_INET = 1, MODE_TCP = 2;
constexpr uint32_t MODE_MASK = 0xff, FLAG_COMPLEMENT = 0x100;

inline uint16_t
one(const uint8_t* seg, uint16_t len, uint16_t seed, uint32_t src,
    uint32_t dst, uint32_t mode)
{
  uint16_t v;
  switch (mode & MODE_MASK) {
    case MODE_TCP:
      v = _ZN6tulips5stack5tcpv49Processor8checksumERKNS0_4ipv47AddressES6_tPKh(
        &src, &dst, len, seg);
      break;
    case MODE_INET: {
      uint16_t s = tulips::stack::utils::checksum(seed, seg, len);
      v = s == 0 ? 0xffff : htons(s);
      break;
    }
    default:
      v = tulips::stack::utils::checksum(seed, seg, len);
      break;
  }
  return (mode & FLAG_COMPLEMENT) ? uint16_t(~v) : v;
}

}

extern "C" {

uint16_t
ref_checksum(uint16_t seed, const uint8_t* data, uint16_t len)
{
  return tulips::stack::utils::checksum(seed, data, len);
}

uint16_t
ref_ipv4_checksum(const uint8_t* hdr)
{
  return tulips::stack::ipv4::checksum(hdr);
}

uint16_t
ref_icmpv4_checksum(const uint8_t* hdr)
{
  return tulips::stack::icmpv4::checksum(hdr);
}

uint16_t
ref_tcp_checksum(uint32_t src, uint32_t dst, uint16_t len, const uint8_t* data)
{
  return _ZN6tulips5stack5tcpv49Processor8checksumERKNS0_4ipv47AddressES6_tPKh(
    &src, &dst, len, data);
}

// Same argument convention as orc_batch (oracle/csum_oracle.c).
int
ref_batch(const uint8_t* base, const uint64_t* offsets, const uint16_t* lengths,
          uint64_t stride, uint32_t fixed_len, const uint16_t* seeds,
          const uint32_t* src, const uint32_t* dst, uint16_t* out, uint64_t n,
          uint32_t mode, int nthreads)
{
  if (fixed_len > 0xffff || (n && (!base || !out)) ||
      (mode & MODE_MASK) > MODE_TCP) {
    return -1;
  }
  if (nthreads < 1) {
    nthreads = 1;
  }
  if (uint64_t(nthreads) > n) {
    nthreads = n ? int(n) : 1;
  }
  auto work = [=](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; ++i) {
      uint64_t off = offsets ? offsets[i] : i * stride;
      uint16_t len = lengths ? lengths[i] : uint16_t(fixed_len);
      out[i] = one(base + off, len, seeds ? seeds[i] : 0, src ? src[i] : 0,
                   dst ? dst[i] : 0, mode);
    }
  };
  if (nthreads == 1) {
    work(0, n);
    return 0;
  }
  // Pin thread t to the t-th CPU of the process's allowed set.
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  std::vector<int> cpus;
  if (sched_getaffinity(0, sizeof(allowed), &allowed) == 0) {
    for (int c = 0; c < CPU_SETSIZE; ++c) {
      if (CPU_ISSET(c, &allowed)) {
        cpus.push_back(c);
      }
    }
  }
  std::vector<std::thread> ts;
  ts.reserve(nthreads);
  for (int t = 0; t < nthreads; ++t) {
    uint64_t lo = n * uint64_t(t) / uint64_t(nthreads);
    uint64_t hi = n * uint64_t(t + 1) / uint64_t(nthreads);
    int cpu = cpus.empty() ? -1 : cpus[size_t(t) % cpus.size()];
    ts.emplace_back([=] {
      if (cpu >= 0) {
        cpu_set_t one_cpu;
        CPU_ZERO(&one_cpu);
        CPU_SET(cpu, &one_cpu);
        pthread_setaffinity_np(pthread_self(), sizeof(one_cpu), &one_cpu);
      }
      work(lo, hi);
    });
  }
  for (auto& t : ts) {
    t.join();
  }
  return 0;
}

}

// The reference's receive-side verification of one poll burst, timed in C
// (bench.py cpu_baseline.burst_latency): for each frame, as the stack does
// on arrival, ipv4::checksum of its 20-byte header (src/stack/ipv4/
// Processor.cpp:94-103) and the tcpv4 checksum of its segment
// (src/stack/tcpv4/Processor.cpp:121-131). `reps` bursts back to back on
// one thread; out = median, p99, min, mean microseconds per burst; returns
// the number of frames of the last burst that verified.
extern "C" uint32_t
ref_time_verify_burst(const uint8_t* base, const uint64_t* offsets, const uint16_t* lengths,
                      uint32_t n, uint32_t reps, double* out)
{
  std::vector<double> t(reps ? reps : 1);
  uint32_t good = 0;
  for (uint32_t r = 0; r < reps; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    good = 0;
    for (uint32_t i = 0; i < n; ++i) {
      const uint8_t* f = base + offsets[i];
      const uint16_t ip = tulips::stack::ipv4::checksum(f + 14);
      uint32_t src, dst;
      memcpy(&src, f + 26, 4);
      memcpy(&dst, f + 30, 4);
      const uint16_t tl = uint16_t(((f[16] << 8) | f[17]) - 20);
      const uint16_t tc =
        _ZN6tulips5stack5tcpv49Processor8checksumERKNS0_4ipv47AddressES6_tPKh(&src, &dst, tl,
                                                                            f + 34);
      good += (ip == 0xffff && tc == 0xffff) ? 1u : 0u;
    }
    t[r] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
             .count();
  }
  std::vector<double> s = t;
  std::sort(s.begin(), s.end());
  double mean = 0;
  for (double x : t) {
    mean += x / double(t.size());
  }
  out[0] = s[s.size() / 2];
  out[1] = s[std::min<size_t>(s.size() - 1, size_t(double(s.size()) * 0.99))];
  out[2] = s[0];
  out[3] = mean;
  return good;
}

extern "C" uint32_t
ref_toeplitz(uint32_t saddr, uint32_t daddr, uint16_t sport, uint16_t dport,
             size_t len, const uint8_t* key, uint32_t init)
{
  // ipv4::Address is a packed wrapper of the 4 wire bytes
  // (include/tulips/stack/IPv4.h:13-62); build it from them.
  uint8_t s[4], d[4];
  memcpy(s, &saddr, 4);
  memcpy(d, &daddr, 4);
  const tulips::stack::ipv4::Address sa(s[0], s[1], s[2], s[3]);
  const tulips::stack::ipv4::Address da(d[0], d[1], d[2], d[3]);
  return tulips::stack::utils::toeplitz(sa, da, sport, dport, len, key, init);
}
