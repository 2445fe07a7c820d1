// bench_host.cpp — the host-side measurement entry points of
// include/tulips_csum_bench.h: C-timed receive-validation latency through the
// product's public C ABI, and the crash backtrace hook.
#include <execinfo.h>
#include <signal.h>
#include <stdint.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "../../include/tulips_csum_bench.h"

extern "C" int
tulips_csum_time_validate(tulips_csum_ctx* ctx, int path, const uint8_t* base,
                          const uint64_t* offsets, const uint16_t* lengths, uint32_t n,
                          uint32_t reps, uint8_t* flags, double* out)
{
  return tulips_csum_time_validate_ring(ctx, path, base, 0, 1, offsets, lengths, n, reps,
                                        flags, out);
}

extern "C" int
tulips_csum_time_validate_ring(tulips_csum_ctx* ctx, int path, const uint8_t* ring,
                               uint64_t burst_stride, uint32_t nbursts,
                               const uint64_t* offsets, const uint16_t* lengths, uint32_t n,
                               uint32_t reps, uint8_t* flags, double* out)
{
  if (!ctx || !out || reps == 0 || path < 0 || path > 3 || nbursts == 0) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  std::vector<double> t(reps);
  for (uint32_t r = 0; r < reps; ++r) {
    const uint8_t* base = ring + uint64_t(r % nbursts) * burst_stride;
    const auto t0 = std::chrono::steady_clock::now();
    int use = path;
    if (use == 3) { // the decorator's default choice, made inside the timed call
      uint64_t bytes = 0;
      for (uint32_t k = 0; k < n; ++k) {
        bytes += lengths[k];
      }
      use = tulips_csum_burst_prefers_cpu(n, bytes) ? 2 : 1;
    }
    const int rc =
      use == 2   ? tulips_csum_validate_frames_cpu(base, offsets, lengths, n, flags, nullptr)
      : use == 1 ? tulips_csum_validate_frames_zc(ctx, base, offsets, lengths, n, flags, nullptr)
                  : tulips_csum_validate_frames_host(ctx, base, offsets, lengths, n, flags,
                                                     nullptr);
    t[r] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
             .count();
    if (rc != TULIPS_STATUS_OK) {
      return rc;
    }
  }
  std::vector<double> s = t;
  std::sort(s.begin(), s.end());
  double mean = 0;
  for (double x : t) {
    mean += x / reps;
  }
  out[0] = s[reps / 2];
  out[1] = s[std::min<size_t>(reps - 1, size_t(double(reps) * 0.99))];
  out[2] = s[0];
  out[3] = mean;
  return TULIPS_STATUS_OK;
}

namespace {

constexpr int CRASH_SIGNALS[] = { SIGSEGV, SIGBUS, SIGILL, SIGFPE, SIGABRT };
struct sigaction g_crash_prev[sizeof(CRASH_SIGNALS) / sizeof(int)];
bool g_crash_on = false;

// async-signal-safe: write(2) of a decimal / hex number
void
crash_write(const char* s)
{
  (void)!write(2, s, strlen(s));
}

void
crash_hex(uintptr_t v)
{
  char b[19] = "0x";
  for (int i = 0; i < 16; ++i) {
    const unsigned d = unsigned(v >> (60 - 4 * i)) & 15u;
    b[2 + i] = char(d < 10 ? '0' + d : 'a' + d - 10);
  }
  b[18] = 0;
  crash_write(b);
}

void
crash_handler(int sig, siginfo_t* si, void* uc)
{
  crash_write("\ntulips_csum: fatal signal ");
  char num[4] = { char('0' + (sig / 10) % 10), char('0' + sig % 10), 0, 0 };
  crash_write(num);
  crash_write(" (");
  crash_write(sig == SIGSEGV ? "SIGSEGV" : sig == SIGBUS ? "SIGBUS" : sig == SIGILL ? "SIGILL"
              : sig == SIGFPE ? "SIGFPE" : "SIGABRT");
  crash_write(") at address ");
  crash_hex(si ? reinterpret_cast<uintptr_t>(si->si_addr) : 0);
  crash_write("; native stack:\n");
  void* frames[64];
  const int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  // the earlier handler takes it from here: restored, then the signal is
  // delivered again (a faulting instruction re-executes on return; abort()
  // raises SIGABRT a second time once its handler returns)
  for (size_t k = 0; k < sizeof(CRASH_SIGNALS) / sizeof(int); ++k) {
    if (CRASH_SIGNALS[k] == sig) {
      (void)sigaction(sig, &g_crash_prev[k], nullptr);
    }
  }
  if (si && si->si_code <= 0) {
    (void)raise(sig); // sent by kill/raise: nothing re-executes
  }
  (void)uc;
}

} // namespace

extern "C" int
tulips_csum_debug_crash_backtrace(int enable)
{
  if (enable != 0 && enable != 1) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (enable && !g_crash_on) {
    void* warm[2];
    (void)backtrace(warm, 2); // loads the unwinder now, not inside the handler
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = crash_handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    for (size_t k = 0; k < sizeof(CRASH_SIGNALS) / sizeof(int); ++k) {
      if (sigaction(CRASH_SIGNALS[k], &sa, &g_crash_prev[k]) != 0) {
        return TULIPS_STATUS_HARDWARE_ERROR;
      }
    }
    g_crash_on = true;
  } else if (!enable && g_crash_on) {
    for (size_t k = 0; k < sizeof(CRASH_SIGNALS) / sizeof(int); ++k) {
      (void)sigaction(CRASH_SIGNALS[k], &g_crash_prev[k], nullptr);
    }
    g_crash_on = false;
  }
  return TULIPS_STATUS_OK;
}
