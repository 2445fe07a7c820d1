// runtime_check.cpp — the product library driven through its C ABI from a
// plain C++ process: no torch, no Python, linked against the ROCm runtime an
// integrator links (/opt/rocm, libamdhip64.so.7 by the library's RUNPATH).
// Test infrastructure (tests/test_native_runtime.py runs it on the GPU box).
//
//   runtime_check runtime
//       which libamdhip64 the process mapped (dl_iterate_phdr) and the HIP
//       runtime/driver versions, as one JSON line.
//   runtime_check zipf-lengths
//       (no GPU) the FNV-1a-64 digest and total of the §8c Zipf lengths.
//   runtime_check parity NAME=FNV ...
//       the SURVEY.md §8c golden batches F1500, F1500-tcp, F9000, F9000-tcp,
//       ZIPF, ZIPF-tcp (and ZIPF_LENGTHS, the Zipf length sequence itself):
//       SplitMix64 arena made on the host, copied to HBM, checksummed by
//       tulips_csum_batch_fixed / tulips_csum_batch_arena / tulips_csum_batch,
//       FNV-1a-64 of the outputs compared with the expected digests (the
//       driving test passes tests/golden/digests.json's). Semantics:
//       /root/reference/src/stack/Utils.cpp:14-42 and
//       src/stack/tcpv4/Processor.cpp:337-357.
//   runtime_check user-object
//       the HIP user-object contract the library's graph ownership relies on
//       (stream_state.h): a user object moved to a capture's graph survives
//       the graph's destruction while an executable instantiated from it
//       lives, and its destructor runs once the last of them is gone.
//   runtime_check graph-cycles N
//       N single-stream cycles of capture (counting verify, arena batch,
//       segmentation), instantiate, destroy the template, replay twice,
//       destroy the executable: every replay's outputs equal the direct
//       calls', and device memory (hipMemGetInfo, after 5 warm-up cycles)
//       ends within 1 MiB of where it started (also reported half-way).
//   runtime_check graph-churn-stateful SECONDS SEED
//       graph ownership under churn: multi-branch graphs of counting, arena,
//       segmentation and fixed calls captured, replayed (checked) and
//       destroyed; device memory flat at the end.
//   runtime_check serial-rate L NBATCH FNV
//       the fixed-stride kernel's one-launch-at-a-time rate on this runtime
//       (NBATCH rotated batches of 65,536 x L bytes, a captured chain of 256
//       launches, HIP events, median of 5), batch 0 checked against FNV.
//   runtime_check fixtures DIR
//       the §8f kernels on this runtime against fixtures the driving test
//       writes to DIR as raw little-endian arrays (test infrastructure):
//       frame validation flags == the reference-computed flags of
//       tests/golden/frames.npz; in-place generation restores the checksum
//       fields of every frame the reference found valid, after they were
//       zeroed, and touches no other byte; compact fields equal the stored
//       fields of those frames; Toeplitz RSS == tests/golden/rss.npz (10
//       keys x 2 inits); segmentation == the oracle's segments (LSO fix-ups
//       parity-unpinned); and the host-memory forms of
//       validation (staged, host code, zero-copy per burst and resident),
//       generation and segmentation through a host context.
//   runtime_check thread-churn SECONDS THREADS
//       graph ownership across host threads: each thread on its own stream
//       captures (thread-local mode), instantiates, replays (checked) and
//       destroys graphs of counting, arena and segmentation calls, with
//       direct calls between; device memory back within 32 MiB at the end
//       (a leak of the graphs' arrays would be >= 4 KiB x every graph).
//   runtime_check capture-neutral F1500=FNV ZIPF=FNV ZIPF-tcp=FNV
//       the library beside another thread's global-mode capture: thread A
//       captures a fixed-stride F1500 call (hipStreamCaptureModeGlobal);
//       while the capture is open thread B makes first calls on a fresh
//       stream (counting verify_arena and batch_arena over ZIPF, which
//       allocate that stream's state and synchronise it) and creates, uses
//       and destroys a host context and a two-entry multi-device context over
//       F1500 host bytes. A's capture must survive and replay to F1500's
//       digest; every B result must equal its digest.
//   runtime_check graph-churn SECONDS SEED
//       the multi-branch capture/replay/destroy churn that faults inside
//       the runtime torch bundles, on this runtime, with
//       library calls as the graphs' kernels and every replay checked
//       (diagnostics: CHURN_PRESYNC=1 completes the poison before each
//       launch, CHURN_DEVSYNC=1 waits for the device instead of the replay
//       stream, CHURN_KERNEL_POISON=1 poisons with a kernel instead of
//       hipMemsetAsync, CHURN_NODROP=1 never destroys a graph (8 are made),
//       CHURN_ONE_ROOT=1 gives every graph a single root node;
//       each mismatch is printed).
// Exit status 0 = all checks passed; every result is printed as JSON.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <link.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tulips_csum.h"

namespace {

#define HIP_OK(x)                                                                    \
  do {                                                                               \
    const hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(3);                                                                       \
    }                                                                                \
  } while (0)

#define CS_OK(x)                                                                     \
  do {                                                                               \
    const int rc_ = (x);                                                             \
    if (rc_ != TULIPS_STATUS_OK) {                                                   \
      fprintf(stderr, "%s:%d %s: status %d (%s)\n", __FILE__, __LINE__, #x, rc_,     \
              tulips_csum_last_error());                                             \
      exit(4);                                                                       \
    }                                                                                \
  } while (0)

// ---- SURVEY.md §8c golden spec ----------------------------------------------
constexpr uint64_t ARENA_SEED = 0x54554C495053ull;
constexpr uint64_t ZIPF_SEED = 0x5A495046ull;
constexpr uint32_t ZIPF_RMAX = 8937;
constexpr uint32_t NSEG = 65536;

uint64_t
splitmix_next(uint64_t& s)
{
  s += 0x9E3779B97F4A7C15ull;
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// the arena byte stream: 8 little-endian bytes per draw, continuous
void
splitmix_fill(uint8_t* dst, uint64_t nbytes)
{
  uint64_t s = ARENA_SEED;
  uint64_t i = 0;
  for (; i + 8 <= nbytes; i += 8) {
    const uint64_t z = splitmix_next(s);
    memcpy(dst + i, &z, 8);
  }
  if (i < nbytes) {
    const uint64_t z = splitmix_next(s);
    memcpy(dst + i, &z, nbytes - i);
  }
}

// Zipf lengths: u = (next >> 11) * 2^-53, r = first index with
// C[r] >= u * C[rmax], C[r] = sum_{k<=r} k^-1.1 summed in order; L = 63 + r
std::vector<uint16_t>
zipf_lengths(uint32_t n)
{
  std::vector<double> c(ZIPF_RMAX);
  double acc = 0;
  for (uint32_t k = 1; k <= ZIPF_RMAX; ++k) {
    acc += std::pow(double(k), -1.1);
    c[k - 1] = acc;
  }
  std::vector<uint16_t> out(n);
  uint64_t s = ZIPF_SEED;
  for (uint32_t i = 0; i < n; ++i) {
    const double u = double(splitmix_next(s) >> 11) * 0x1p-53;
    const double t = u * c.back();
    const uint32_t r = uint32_t(std::lower_bound(c.begin(), c.end(), t) - c.begin()) + 1;
    out[i] = uint16_t(63 + r);
  }
  return out;
}

uint64_t
fnv1a_u16(const std::vector<uint16_t>& v)
{
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint16_t x : v) {
    h = (h ^ (x & 0xff)) * 0x100000001b3ull;
    h = (h ^ (x >> 8)) * 0x100000001b3ull;
  }
  return h;
}

uint32_t
ip4(uint8_t a, uint8_t b, uint8_t c, uint8_t d)
{
  return uint32_t(a) | uint32_t(b) << 8 | uint32_t(c) << 16 | uint32_t(d) << 24;
}

template<class T>
T*
to_device(const std::vector<T>& v)
{
  void* p = nullptr;
  HIP_OK(hipMalloc(&p, std::max<size_t>(1, v.size()) * sizeof(T)));
  if (!v.empty()) {
    HIP_OK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  }
  return static_cast<T*>(p);
}

template<class T>
std::vector<T>
to_host(const T* p, size_t n)
{
  std::vector<T> v(n);
  HIP_OK(hipMemcpy(v.data(), p, n * sizeof(T), hipMemcpyDeviceToHost));
  return v;
}

std::string
hex64(uint64_t v)
{
  char b[17];
  snprintf(b, sizeof(b), "%016llx", static_cast<unsigned long long>(v));
  return b;
}

// ---- runtime --------------------------------------------------------------------
int
find_hip(struct dl_phdr_info* info, size_t, void* data)
{
  if (info->dlpi_name && strstr(info->dlpi_name, "libamdhip64")) {
    static_cast<std::vector<std::string>*>(data)->push_back(info->dlpi_name);
  }
  return 0;
}

std::string
runtime_json()
{
  std::vector<std::string> libs;
  dl_iterate_phdr(find_hip, &libs);
  int rt = 0, drv = 0;
  (void)hipRuntimeGetVersion(&rt);
  (void)hipDriverGetVersion(&drv);
  std::string s = "{\"hip_runtime_libs\": [";
  for (size_t i = 0; i < libs.size(); ++i) {
    s += (i ? ", \"" : "\"") + libs[i] + "\"";
  }
  s += "], \"hip_runtime_version\": " + std::to_string(rt) +
       ", \"hip_driver_version\": " + std::to_string(drv) + ", \"library\": \"" +
       tulips_csum_version() + "\"}";
  return s;
}

// ---- parity ---------------------------------------------------------------------
int
cmd_parity(int argc, char** argv)
{
  std::map<std::string, std::string> want;
  for (int i = 0; i < argc; ++i) {
    const char* eq = strchr(argv[i], '=');
    if (!eq) {
      fprintf(stderr, "expected NAME=FNV, got %s\n", argv[i]);
      return 2;
    }
    want[std::string(argv[i], size_t(eq - argv[i]))] = eq + 1;
  }
  const std::vector<uint16_t> zl = zipf_lengths(NSEG);
  uint64_t ztotal = 0;
  std::vector<uint64_t> zoffs(NSEG);
  for (uint32_t i = 0; i < NSEG; ++i) {
    zoffs[i] = ztotal;
    ztotal += zl[i];
  }
  // one arena for all batches: the largest is F9000 (NSEG * 9000 bytes)
  const uint64_t nbytes = uint64_t(NSEG) * 9000;
  std::vector<uint8_t> host(nbytes + 64, 0);
  splitmix_fill(host.data(), nbytes);
  uint8_t* arena = to_device(host);
  host.clear();
  host.shrink_to_fit();
  uint16_t* out = nullptr;
  HIP_OK(hipMalloc(reinterpret_cast<void**>(&out), NSEG * 2));
  uint32_t* src = to_device(std::vector<uint32_t>(NSEG, ip4(10, 1, 0, 1)));
  uint32_t* dst = to_device(std::vector<uint32_t>(NSEG, ip4(10, 1, 0, 2)));
  uint64_t* d_zoffs = to_device(zoffs);
  uint16_t* d_zlens = to_device(zl);
  hipStream_t st = nullptr;
  HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));

  std::map<std::string, std::string> got;
  auto digest = [&]() {
    HIP_OK(hipStreamSynchronize(st));
    return hex64(fnv1a_u16(to_host(out, NSEG)));
  };
  got["ZIPF_LENGTHS"] = hex64(fnv1a_u16(zl));
  for (uint32_t L : { 1500u, 9000u }) {
    const std::string name = "F" + std::to_string(L);
    CS_OK(tulips_csum_batch_fixed(arena, L, L, nullptr, nullptr, nullptr, out, NSEG,
                                  TULIPS_CSUM_RAW, st));
    got[name] = digest();
    CS_OK(tulips_csum_batch_fixed(arena, L, L, nullptr, src, dst, out, NSEG, TULIPS_CSUM_TCP,
                                  st));
    got[name + "-tcp"] = digest();
  }
  CS_OK(tulips_csum_batch_arena(arena, ztotal, d_zoffs, d_zlens, nullptr, nullptr, nullptr, out,
                                NSEG, TULIPS_CSUM_RAW, st));
  got["ZIPF"] = digest();
  CS_OK(tulips_csum_batch_arena(arena, ztotal, d_zoffs, d_zlens, nullptr, src, dst, out, NSEG,
                                TULIPS_CSUM_TCP, st));
  got["ZIPF-tcp"] = digest();
  // the any-layout entry point over the same Zipf segments
  CS_OK(tulips_csum_batch(arena, d_zoffs, d_zlens, nullptr, nullptr, nullptr, out, NSEG,
                          TULIPS_CSUM_RAW, st));
  got["ZIPF-any"] = digest();
  if (want.count("ZIPF")) {
    want["ZIPF-any"] = want["ZIPF"];
  }

  int bad = 0;
  std::string s = "{\"parity\": {";
  bool first = true;
  for (auto& kv : got) {
    const auto w = want.find(kv.first);
    const bool ok = w != want.end() && w->second == kv.second;
    bad += ok ? 0 : 1;
    s += std::string(first ? "" : ", ") + "\"" + kv.first + "\": {\"fnv1a64\": \"" + kv.second +
         "\", \"expect\": \"" + (w == want.end() ? "" : w->second) + "\", \"ok\": " +
         (ok ? "true" : "false") + "}";
    first = false;
  }
  s += "}, \"runtime\": " + runtime_json() + "}";
  printf("%s\n", s.c_str());
  HIP_OK(hipStreamDestroy(st));
  (void)hipFree(arena);
  (void)hipFree(out);
  (void)hipFree(src);
  (void)hipFree(dst);
  (void)hipFree(d_zoffs);
  (void)hipFree(d_zlens);
  return bad ? 1 : 0;
}

// ---- §8f kernels against fixtures -----------------------------------------------------
template<class T>
std::vector<T>
read_raw(const std::string& path)
{
  std::vector<T> v;
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", path.c_str());
    exit(2);
  }
  fseek(f, 0, SEEK_END);
  const long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  v.resize(size_t(n) / sizeof(T));
  if (!v.empty() && fread(v.data(), sizeof(T), v.size(), f) != v.size()) {
    fprintf(stderr, "short read %s\n", path.c_str());
    exit(2);
  }
  fclose(f);
  return v;
}

// progress of `fixtures` on stderr (the driving test shows it when a run
// fails or stalls)
void
phase(const char* what)
{
  static const auto t0 = std::chrono::steady_clock::now();
  const double t =
    std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  fprintf(stderr, "[fixtures %.3f s] %s\n", t, what);
  fflush(stderr);
}

int
cmd_fixtures(const std::string& dir)
{
  hipStream_t st = nullptr;
  HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::string out = "{\"fixtures\": {";
  int bad = 0;
  auto report = [&](const char* name, bool ok, const std::string& detail) {
    bad += ok ? 0 : 1;
    out += std::string(out.back() == '{' ? "" : ", ") + "\"" + name + "\": {\"ok\": " +
           (ok ? "true" : "false") + detail + "}";
  };

  // frames: validation, in-place generation, compact fields
  phase("frames");
  {
    const auto arena = read_raw<uint8_t>(dir + "/frames.arena.bin");
    const auto offs = read_raw<uint64_t>(dir + "/frames.offsets.bin");
    const auto lens = read_raw<uint16_t>(dir + "/frames.lengths.bin");
    const auto expect = read_raw<uint8_t>(dir + "/frames.expect.bin");
    const uint32_t n = uint32_t(offs.size());
    uint8_t* d_arena = to_device(arena);
    uint64_t* d_offs = to_device(offs);
    uint16_t* d_lens = to_device(lens);
    uint8_t* d_flags = to_device(std::vector<uint8_t>(n, 0xA5));
    uint32_t* d_cnt = to_device(std::vector<uint32_t>(4, 0xA5A5A5A5u));
    CS_OK(tulips_csum_validate_frames(d_arena, d_offs, d_lens, n, d_flags, d_cnt, st));
    HIP_OK(hipStreamSynchronize(st));
    const auto flags = to_host(d_flags, n);
    const auto cnt = to_host(d_cnt, 4);
    uint32_t want_cnt[4] = { 0, 0, 0, 0 };
    uint32_t mism = 0, valid = 0;
    for (uint32_t i = 0; i < n; ++i) {
      mism += flags[i] != expect[i];
      const uint8_t e = expect[i];
      want_cnt[0] += (e & TULIPS_FRAME_IPV4) != 0;
      want_cnt[1] += (e & TULIPS_FRAME_IPV4) && !(e & TULIPS_FRAME_IP_CSUM_OK);
      want_cnt[2] += (e & TULIPS_FRAME_TCP) != 0;
      want_cnt[3] += (e & TULIPS_FRAME_TCP) && !(e & TULIPS_FRAME_L4_CSUM_OK);
      valid += e == 0x0F;
    }
    const bool cnt_ok = std::equal(cnt.begin(), cnt.end(), want_cnt);
    report("frames_validate", mism == 0 && cnt_ok,
           ", \"frames\": " + std::to_string(n) + ", \"flag_mismatches\": " +
             std::to_string(mism) + ", \"counters_ok\": " + (cnt_ok ? "true" : "false"));

    // compact fields of the frames the reference found valid: their stored words
    uint32_t* d_fields = to_device(std::vector<uint32_t>(n, 0xA5A5A5A5u));
    CS_OK(tulips_csum_generate_fields(d_arena, d_offs, d_lens, n, d_fields, nullptr, st));
    HIP_OK(hipStreamSynchronize(st));
    const auto fields = to_host(d_fields, n);
    uint32_t fmism = 0;
    auto word = [&](const std::vector<uint8_t>& a, uint64_t at) {
      return uint32_t(a[at]) | uint32_t(a[at + 1]) << 8;
    };
    for (uint32_t i = 0; i < n; ++i) {
      if (expect[i] == 0x0F) {
        const uint32_t w = word(arena, offs[i] + 24) | word(arena, offs[i] + 50) << 16;
        fmism += fields[i] != w;
      }
    }
    report("frames_generate_fields", fmism == 0 && valid > 0,
           ", \"valid_frames\": " + std::to_string(valid) + ", \"mismatches\": " +
             std::to_string(fmism));

    // in place: zero the fields of the valid frames, regenerate every frame
    std::vector<uint8_t> zeroed = arena;
    std::vector<uint8_t> field_byte(arena.size(), 0);
    for (uint32_t i = 0; i < n; ++i) {
      for (uint64_t at : { offs[i] + 24, offs[i] + 25, offs[i] + 50, offs[i] + 51 }) {
        if (at < arena.size()) {
          field_byte[at] = 1;
          if (expect[i] == 0x0F) {
            zeroed[at] = 0;
          }
        }
      }
    }
    HIP_OK(hipMemcpy(d_arena, zeroed.data(), zeroed.size(), hipMemcpyHostToDevice));
    CS_OK(tulips_csum_generate_frames(d_arena, d_offs, d_lens, n, nullptr, st));
    HIP_OK(hipStreamSynchronize(st));
    const auto gen = to_host(d_arena, arena.size());
    uint64_t restored_bad = 0, other_bad = 0;
    for (uint32_t i = 0; i < n; ++i) {
      if (expect[i] == 0x0F) {
        for (uint64_t at : { offs[i] + 24, offs[i] + 25, offs[i] + 50, offs[i] + 51 }) {
          restored_bad += gen[at] != arena[at];
        }
      }
    }
    for (size_t b = 0; b < arena.size(); ++b) {
      other_bad += !field_byte[b] && gen[b] != zeroed[b];
    }
    report("frames_generate_in_place", restored_bad == 0 && other_bad == 0,
           ", \"field_bytes_wrong\": " + std::to_string(restored_bad) +
             ", \"other_bytes_changed\": " + std::to_string(other_bad));
    for (void* q : { static_cast<void*>(d_arena), static_cast<void*>(d_offs),
                     static_cast<void*>(d_lens), static_cast<void*>(d_flags),
                     static_cast<void*>(d_cnt), static_cast<void*>(d_fields) }) {
      (void)hipFree(q);
    }
  }

  // Toeplitz RSS
  phase("rss");
  {
    const auto sa = read_raw<uint32_t>(dir + "/rss.saddr.bin");
    const auto da = read_raw<uint32_t>(dir + "/rss.daddr.bin");
    const auto sp = read_raw<uint16_t>(dir + "/rss.sport.bin");
    const auto dp = read_raw<uint16_t>(dir + "/rss.dport.bin");
    const uint32_t n = uint32_t(sa.size());
    uint32_t* d_sa = to_device(sa);
    uint32_t* d_da = to_device(da);
    uint16_t* d_sp = to_device(sp);
    uint16_t* d_dp = to_device(dp);
    uint32_t* d_h = to_device(std::vector<uint32_t>(n, 0));
    uint32_t keys = 0, mism = 0;
    for (int k = 0;; ++k) {
      const std::string kp = dir + "/rss.key_" + std::to_string(k) + ".bin";
      FILE* f = fopen(kp.c_str(), "rb");
      if (!f) {
        break;
      }
      fclose(f);
      const auto key = read_raw<uint8_t>(kp);
      for (const char* tag : { "init0", "initff" }) {
        const uint32_t init = strcmp(tag, "init0") == 0 ? 0u : 0xFFFFFFFFu;
        const auto want = read_raw<uint32_t>(dir + "/rss.expect_" + std::to_string(k) + "_" +
                                             tag + ".bin");
        HIP_OK(hipMemsetAsync(d_h, 0xA5, n * 4, st));
        CS_OK(tulips_rss_toeplitz_batch(d_sa, d_da, d_sp, d_dp, n, key.data(), key.size(), init,
                                        d_h, st));
        HIP_OK(hipStreamSynchronize(st));
        const auto got = to_host(d_h, n);
        for (uint32_t i = 0; i < n; ++i) {
          mism += got[i] != want[i];
        }
      }
      ++keys;
    }
    report("rss_toeplitz", mism == 0 && keys > 0,
           ", \"tuples\": " + std::to_string(n) + ", \"keys\": " + std::to_string(keys) +
             ", \"mismatches\": " + std::to_string(mism));
    for (void* q : { static_cast<void*>(d_sa), static_cast<void*>(d_da), static_cast<void*>(d_sp),
                     static_cast<void*>(d_dp), static_cast<void*>(d_h) }) {
      (void)hipFree(q);
    }
  }

  // segmentation against the oracle's segments
  phase("segmentation");
  {
    const auto arena = read_raw<uint8_t>(dir + "/seg.arena.bin");
    const auto offs = read_raw<uint64_t>(dir + "/seg.offsets.bin");
    const auto lens = read_raw<uint16_t>(dir + "/seg.lengths.bin");
    const auto params = read_raw<uint32_t>(dir + "/seg.params.bin"); // mss, stride
    const auto efirst = read_raw<uint32_t>(dir + "/seg.first.bin");
    const auto eout = read_raw<uint8_t>(dir + "/seg.out.bin");
    const auto elens = read_raw<uint16_t>(dir + "/seg.out_lengths.bin");
    const uint32_t n = uint32_t(offs.size()), mss = params[0], stride = params[1];
    const uint32_t total = efirst[n];
    uint8_t* d_in = to_device(arena);
    uint64_t* d_offs = to_device(offs);
    uint16_t* d_lens = to_device(lens);
    uint8_t* d_out = to_device(std::vector<uint8_t>(size_t(total) * stride, 0x5B));
    uint16_t* d_olens = to_device(std::vector<uint16_t>(total, 0xA5A5));
    uint32_t* d_first = to_device(std::vector<uint32_t>(n + 1, 0xA5A5A5A5u));
    CS_OK(tulips_csum_segment_frames(d_in, d_offs, d_lens, n, mss, d_out, stride, total, d_olens,
                                     d_first, st));
    HIP_OK(hipStreamSynchronize(st));
    const auto first = to_host(d_first, n + 1);
    const auto olens = to_host(d_olens, total);
    const auto sout = to_host(d_out, size_t(total) * stride);
    uint64_t bytes_bad = 0;
    const bool plan_ok = first == efirst && olens == elens;
    if (plan_ok) {
      for (uint32_t j = 0; j < total; ++j) {
        for (uint32_t b = 0; b < elens[j]; ++b) {
          bytes_bad += sout[size_t(j) * stride + b] != eout[size_t(j) * stride + b];
        }
      }
    }
    report("segment_frames", plan_ok && bytes_bad == 0,
           ", \"super_frames\": " + std::to_string(n) + ", \"segments\": " +
             std::to_string(total) + ", \"plan_ok\": " + (plan_ok ? "true" : "false") +
             ", \"bytes_wrong\": " + std::to_string(bytes_bad));
    for (void* q : { static_cast<void*>(d_in), static_cast<void*>(d_offs),
                     static_cast<void*>(d_lens), static_cast<void*>(d_out),
                     static_cast<void*>(d_olens), static_cast<void*>(d_first) }) {
      (void)hipFree(q);
    }
  }
  // the host-memory forms: the same fixtures through a host context
  phase("host context");
  {
    const auto arena = read_raw<uint8_t>(dir + "/frames.arena.bin");
    const auto offs = read_raw<uint64_t>(dir + "/frames.offsets.bin");
    const auto lens = read_raw<uint16_t>(dir + "/frames.lengths.bin");
    const auto expect = read_raw<uint8_t>(dir + "/frames.expect.bin");
    const uint32_t n = uint32_t(offs.size());
    tulips_csum_ctx* ctx = nullptr;
    CS_OK(tulips_csum_ctx_create(0, 0, &ctx));
    auto flags_ok = [&](const std::vector<uint8_t>& f) {
      return std::equal(f.begin(), f.end(), expect.begin());
    };
    std::vector<uint8_t> f(n, 0xA5);
    phase("ctx validate_frames_host");
    CS_OK(tulips_csum_validate_frames_host(ctx, arena.data(), offs.data(), lens.data(), n,
                                           f.data(), nullptr));
    const bool host_ok = flags_ok(f);
    std::fill(f.begin(), f.end(), 0xA5);
    phase("validate_frames_cpu");
    CS_OK(tulips_csum_validate_frames_cpu(arena.data(), offs.data(), lens.data(), n, f.data(),
                                          nullptr));
    const bool cpu_ok = flags_ok(f);
    // zero-copy bursts of at most TULIPS_CSUM_ZC_MAX_FRAMES from page-locked
    // memory, one launch per burst and then the resident server
    void* pinned = nullptr;
    CS_OK(tulips_csum_host_alloc(arena.size(), &pinned));
    memcpy(pinned, arena.data(), arena.size());
    bool zc_ok[2] = { false, false };
    phase("zc");
    for (int resident = 0; resident < 2; ++resident) {
      phase(resident ? "zc resident" : "zc launch per burst");
      CS_OK(tulips_csum_ctx_set_lowlat(ctx, resident));
      std::fill(f.begin(), f.end(), 0xA5);
      for (uint32_t i = 0; i < n; i += TULIPS_CSUM_ZC_MAX_FRAMES) {
        const uint32_t m = std::min<uint32_t>(TULIPS_CSUM_ZC_MAX_FRAMES, n - i);
        CS_OK(tulips_csum_validate_frames_zc(ctx, static_cast<const uint8_t*>(pinned),
                                             offs.data() + i, lens.data() + i, m, f.data() + i,
                                             nullptr));
      }
      zc_ok[resident] = flags_ok(f);
    }
    phase("zc back to launch per burst");
    CS_OK(tulips_csum_ctx_set_lowlat(ctx, 0));
    CS_OK(tulips_csum_host_free(pinned));
    report("ctx_validate_frames", host_ok && cpu_ok && zc_ok[0] && zc_ok[1],
           std::string(", \"host\": ") + (host_ok ? "true" : "false") + ", \"cpu\": " +
             (cpu_ok ? "true" : "false") + ", \"zc\": " + (zc_ok[0] ? "true" : "false") +
             ", \"zc_resident\": " + (zc_ok[1] ? "true" : "false"));
    // in-place generation of host frames: the valid frames' fields zeroed
    std::vector<uint8_t> zeroed = arena;
    std::vector<uint8_t> field_byte(arena.size(), 0);
    for (uint32_t i = 0; i < n; ++i) {
      for (uint64_t at : { offs[i] + 24, offs[i] + 25, offs[i] + 50, offs[i] + 51 }) {
        if (at < arena.size()) {
          field_byte[at] = 1;
          if (expect[i] == 0x0F) {
            zeroed[at] = 0;
          }
        }
      }
    }
    std::vector<uint8_t> gen = zeroed;
    phase("ctx generate_frames_host");
    CS_OK(tulips_csum_generate_frames_host(ctx, gen.data(), offs.data(), lens.data(), n,
                                           nullptr));
    uint64_t restored_bad = 0, other_bad = 0;
    for (uint32_t i = 0; i < n; ++i) {
      if (expect[i] == 0x0F) {
        for (uint64_t at : { offs[i] + 24, offs[i] + 25, offs[i] + 50, offs[i] + 51 }) {
          restored_bad += gen[at] != arena[at];
        }
      }
    }
    for (size_t b = 0; b < arena.size(); ++b) {
      other_bad += !field_byte[b] && gen[b] != zeroed[b];
    }
    report("ctx_generate_frames", restored_bad == 0 && other_bad == 0,
           ", \"field_bytes_wrong\": " + std::to_string(restored_bad) +
             ", \"other_bytes_changed\": " + std::to_string(other_bad));
    // segmentation of host super-frames
    const auto sarena = read_raw<uint8_t>(dir + "/seg.arena.bin");
    const auto soffs = read_raw<uint64_t>(dir + "/seg.offsets.bin");
    const auto slens = read_raw<uint16_t>(dir + "/seg.lengths.bin");
    const auto params = read_raw<uint32_t>(dir + "/seg.params.bin");
    const auto efirst = read_raw<uint32_t>(dir + "/seg.first.bin");
    const auto eout = read_raw<uint8_t>(dir + "/seg.out.bin");
    const auto elens = read_raw<uint16_t>(dir + "/seg.out_lengths.bin");
    const uint32_t sn = uint32_t(soffs.size()), mss = params[0], stride = params[1];
    const uint32_t total = efirst[sn];
    std::vector<uint8_t> sout(size_t(total) * stride, 0x5B);
    std::vector<uint16_t> solens(total, 0xA5A5);
    std::vector<uint32_t> sfirst(sn + 1, 0xA5A5A5A5u);
    phase("ctx segment_frames_host");
    CS_OK(tulips_csum_segment_frames_host(ctx, sarena.data(), soffs.data(), slens.data(), sn, mss,
                                          sout.data(), stride, total, solens.data(),
                                          sfirst.data()));
    uint64_t bytes_bad = 0;
    const bool plan_ok = sfirst == efirst && solens == elens;
    if (plan_ok) {
      for (uint32_t j = 0; j < total; ++j) {
        for (uint32_t b = 0; b < elens[j]; ++b) {
          bytes_bad += sout[size_t(j) * stride + b] != eout[size_t(j) * stride + b];
        }
      }
    }
    report("ctx_segment_frames", plan_ok && bytes_bad == 0,
           std::string(", \"plan_ok\": ") + (plan_ok ? "true" : "false") +
             ", \"bytes_wrong\": " + std::to_string(bytes_bad));
    phase("ctx destroy");
    tulips_csum_ctx_destroy(ctx);
  }
  phase("release");
  CS_OK(tulips_csum_release_stream(st));
  HIP_OK(hipStreamDestroy(st));
  phase("done");
  out += "}, \"runtime\": " + runtime_json() + "}";
  printf("%s\n", out.c_str());
  return bad ? 1 : 0;
}

// ---- capture-mode neutrality -------------------------------------------------------
int
cmd_capture_neutral(int argc, char** argv)
{
  std::map<std::string, std::string> want;
  for (int i = 0; i < argc; ++i) {
    const char* eq = strchr(argv[i], '=');
    if (!eq) {
      fprintf(stderr, "expected NAME=FNV, got %s\n", argv[i]);
      return 2;
    }
    want[std::string(argv[i], size_t(eq - argv[i]))] = eq + 1;
  }
  const std::vector<uint16_t> zl = zipf_lengths(NSEG);
  uint64_t ztotal = 0;
  std::vector<uint64_t> zoffs(NSEG);
  for (uint32_t i = 0; i < NSEG; ++i) {
    zoffs[i] = ztotal;
    ztotal += zl[i];
  }
  const uint64_t nbytes = uint64_t(NSEG) * 1500;
  std::vector<uint8_t> host(std::max<uint64_t>(nbytes, ztotal) + 64, 0);
  splitmix_fill(host.data(), host.size() - 64);
  uint8_t* arena = to_device(host);
  const std::vector<uint32_t> hsrc(NSEG, ip4(10, 1, 0, 1)), hdst(NSEG, ip4(10, 1, 0, 2));
  uint32_t* src = to_device(hsrc);
  uint32_t* dst = to_device(hdst);
  uint64_t* d_zoffs = to_device(zoffs);
  uint16_t* d_zlens = to_device(zl);
  std::vector<uint64_t> foffs(NSEG);
  for (uint32_t i = 0; i < NSEG; ++i) {
    foffs[i] = uint64_t(i) * 1500;
  }
  const std::vector<uint16_t> flens(NSEG, 1500);
  uint16_t *out_a = nullptr, *out_v = nullptr, *out_z = nullptr;
  uint32_t* bad = nullptr;
  HIP_OK(hipMalloc(reinterpret_cast<void**>(&out_a), NSEG * 2));
  HIP_OK(hipMalloc(reinterpret_cast<void**>(&out_v), NSEG * 2));
  HIP_OK(hipMalloc(reinterpret_cast<void**>(&out_z), NSEG * 2));
  HIP_OK(hipMalloc(reinterpret_cast<void**>(&bad), 16));
  hipStream_t sa = nullptr, sb = nullptr;
  HIP_OK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  HIP_OK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  HIP_OK(hipDeviceSynchronize());

  std::atomic<int> stage{ 0 };
  int rc_v = -1, rc_z = -1, rc_ctx = -1, rc_mctx = -1;
  std::vector<uint16_t> h_ctx(NSEG, 0xA5A5), h_mctx(NSEG, 0xA5A5);
  std::thread tb([&] {
    while (stage.load() < 1) {
      std::this_thread::yield();
    }
    rc_v = tulips_csum_verify_arena(arena, ztotal, d_zoffs, d_zlens, src, dst, out_v, bad, NSEG,
                                    TULIPS_CSUM_TCP, sb);
    rc_z = tulips_csum_batch_arena(arena, ztotal, d_zoffs, d_zlens, nullptr, nullptr, nullptr,
                                   out_z, NSEG, TULIPS_CSUM_RAW, sb);
    tulips_csum_ctx* ctx = nullptr;
    rc_ctx = tulips_csum_ctx_create(0, 0, &ctx);
    if (rc_ctx == TULIPS_STATUS_OK) {
      rc_ctx = tulips_csum_batch_host(ctx, host.data(), foffs.data(), flens.data(), nullptr,
                                      nullptr, nullptr, h_ctx.data(), NSEG, TULIPS_CSUM_RAW);
      tulips_csum_ctx_destroy(ctx);
    }
    const int devs[2] = { 0, 0 };
    tulips_csum_mctx* m = nullptr;
    rc_mctx = tulips_csum_mctx_create(devs, 2, 0, &m);
    if (rc_mctx == TULIPS_STATUS_OK) {
      rc_mctx = tulips_csum_mctx_batch_host(m, host.data(), foffs.data(), flens.data(), nullptr,
                                            nullptr, nullptr, h_mctx.data(), NSEG,
                                            TULIPS_CSUM_RAW);
      tulips_csum_mctx_destroy(m);
    }
    stage.store(2);
  });
  HIP_OK(hipStreamBeginCapture(sa, hipStreamCaptureModeGlobal));
  const int rc_a = tulips_csum_batch_fixed(arena, 1500, 1500, nullptr, nullptr, nullptr, out_a,
                                           NSEG, TULIPS_CSUM_RAW, sa);
  stage.store(1);
  while (stage.load() < 2) {
    std::this_thread::yield();
  }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(sa, &cs);
  hipGraph_t g = nullptr;
  const hipError_t e_end = hipStreamEndCapture(sa, &g);
  tb.join();
  (void)hipGetLastError();
  bool replay_ok = false;
  std::string d_a;
  if (e_end == hipSuccess && g) {
    hipGraphExec_t x = nullptr;
    HIP_OK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    HIP_OK(hipMemsetAsync(out_a, 0xA5, NSEG * 2, sa));
    HIP_OK(hipGraphLaunch(x, sa));
    HIP_OK(hipStreamSynchronize(sa));
    d_a = hex64(fnv1a_u16(to_host(out_a, NSEG)));
    replay_ok = d_a == want["F1500"];
    HIP_OK(hipGraphExecDestroy(x));
    HIP_OK(hipGraphDestroy(g));
  }
  HIP_OK(hipStreamSynchronize(sb));
  const std::string d_v = hex64(fnv1a_u16(to_host(out_v, NSEG)));
  const std::string d_z = hex64(fnv1a_u16(to_host(out_z, NSEG)));
  const std::string d_ctx = hex64(fnv1a_u16(h_ctx)), d_mctx = hex64(fnv1a_u16(h_mctx));
  const bool ok = rc_a == 0 && cs == hipStreamCaptureStatusActive && e_end == hipSuccess &&
                  replay_ok && rc_v == 0 && rc_z == 0 && rc_ctx == 0 && rc_mctx == 0 &&
                  d_v == want["ZIPF-tcp"] && d_z == want["ZIPF"] && d_ctx == want["F1500"] &&
                  d_mctx == want["F1500"];
  printf("{\"capture_neutral\": {\"capture_status_after_b\": %d, \"end_capture\": %d, "
         "\"replay_F1500\": \"%s\", \"b_rc\": [%d, %d, %d, %d], \"b_verify_arena_tcp\": \"%s\", "
         "\"b_batch_arena\": \"%s\", \"b_ctx_host\": \"%s\", \"b_mctx_host\": \"%s\", "
         "\"ok\": %s}, \"runtime\": %s}\n",
         int(cs), int(e_end), d_a.c_str(), rc_v, rc_z, rc_ctx, rc_mctx, d_v.c_str(), d_z.c_str(),
         d_ctx.c_str(), d_mctx.c_str(), ok ? "true" : "false", runtime_json().c_str());
  CS_OK(tulips_csum_release_stream(sa));
  CS_OK(tulips_csum_release_stream(sb));
  HIP_OK(hipStreamDestroy(sa));
  HIP_OK(hipStreamDestroy(sb));
  for (void* q : { static_cast<void*>(arena), static_cast<void*>(src), static_cast<void*>(dst),
                   static_cast<void*>(d_zoffs), static_cast<void*>(d_zlens),
                   static_cast<void*>(out_a), static_cast<void*>(out_v),
                   static_cast<void*>(out_z), static_cast<void*>(bad) }) {
    (void)hipFree(q);
  }
  return ok ? 0 : 1;
}

// ---- user objects ---------------------------------------------------------------
std::atomic<int> g_fired{ 0 };
std::atomic<bool> g_same_thread{ false };
std::thread::id g_main;

void
on_destroy(void*)
{
  g_same_thread = std::this_thread::get_id() == g_main;
  g_fired.fetch_add(1);
}

int
fired_after_settle()
{
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  return g_fired.load();
}

int
cmd_user_object()
{
  g_main = std::this_thread::get_id();
  hipStream_t s = nullptr;
  HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void* d = nullptr;
  HIP_OK(hipMalloc(&d, 4096));
  struct Order
  {
    const char* name;
    bool exec_first;
  };
  std::string js = "{\"user_object\": [";
  int bad = 0;
  for (const Order o : { Order{ "template_destroyed_first", false },
                         Order{ "exec_destroyed_first", true } }) {
    g_fired = 0;
    HIP_OK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    HIP_OK(hipMemsetAsync(d, 1, 4096, s));
    hipStreamCaptureStatus cs;
    unsigned long long id = 0;
    hipGraph_t cg = nullptr;
    HIP_OK(hipStreamGetCaptureInfo_v2(s, &cs, &id, &cg, nullptr, nullptr));
    hipUserObject_t obj = nullptr;
    HIP_OK(hipUserObjectCreate(&obj, nullptr, on_destroy, 1, hipUserObjectNoDestructorSync));
    HIP_OK(hipGraphRetainUserObject(cg, obj, 1, hipGraphUserObjectMove));
    HIP_OK(hipMemsetAsync(d, 2, 4096, s));
    hipGraph_t g = nullptr;
    HIP_OK(hipStreamEndCapture(s, &g));
    const bool same_graph = g == cg;
    hipGraphExec_t x = nullptr;
    HIP_OK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    int after_first = 0, after_launch = 0, after_second = 0;
    if (o.exec_first) {
      HIP_OK(hipGraphLaunch(x, s));
      HIP_OK(hipStreamSynchronize(s));
      after_launch = fired_after_settle();
      HIP_OK(hipGraphExecDestroy(x));
      after_first = fired_after_settle();
      HIP_OK(hipGraphDestroy(g));
      after_second = fired_after_settle();
    } else {
      HIP_OK(hipGraphDestroy(g));
      after_first = fired_after_settle();
      HIP_OK(hipGraphLaunch(x, s));
      HIP_OK(hipStreamSynchronize(s));
      after_launch = fired_after_settle();
      HIP_OK(hipGraphExecDestroy(x));
      after_second = fired_after_settle();
    }
    const bool ok = same_graph && after_first == 0 && after_launch == 0 && after_second == 1;
    bad += ok ? 0 : 1;
    char b[400];
    snprintf(b, sizeof(b),
             "%s{\"order\": \"%s\", \"capture_graph_is_result\": %s, \"fired_after_first_destroy\": "
             "%d, \"fired_after_launch\": %d, \"fired_after_last_destroy\": %d, "
             "\"destructor_on_calling_thread\": %s, \"ok\": %s}",
             o.exec_first ? ", " : "", o.name, same_graph ? "true" : "false", after_first,
             after_launch, after_second, g_same_thread ? "true" : "false", ok ? "true" : "false");
    js += b;
  }
  js += "], \"runtime\": " + runtime_json() + "}";
  printf("%s\n", js.c_str());
  (void)hipFree(d);
  HIP_OK(hipStreamDestroy(s));
  return bad ? 1 : 0;
}

// ---- graph cycles ---------------------------------------------------------------
struct Rng
{
  uint64_t s;
  uint32_t next() { return uint32_t(splitmix_next(s) >> 32); }
};

void
put16(uint8_t* p, uint16_t v)
{
  p[0] = uint8_t(v >> 8);
  p[1] = uint8_t(v);
}

// an Ethernet / option-less IPv4 / TCP frame with `payload` bytes
std::vector<uint8_t>
tcp_frame(Rng& r, uint32_t payload)
{
  std::vector<uint8_t> f(14 + 20 + 20 + payload);
  for (auto& b : f) {
    b = uint8_t(r.next());
  }
  put16(&f[12], 0x0800);
  uint8_t* ip = &f[14];
  ip[0] = 0x45;
  ip[1] = 0;
  put16(ip + 2, uint16_t(40 + payload));
  put16(ip + 6, 0x4000); // DF
  ip[8] = 64;
  ip[9] = 6;
  uint8_t* tcp = ip + 20;
  tcp[12] = 5 << 4;
  tcp[13] = 0x18; // PSH | ACK
  return f;
}

int
cmd_graph_cycles(uint32_t cycles)
{
  Rng r{ 0x6c69666574696d65ull };
  // counting + arena batch: 4,096 segments of 40-9000 bytes, packed in order
  const uint32_t n = 4096;
  std::vector<uint16_t> lens(n);
  std::vector<uint64_t> offs(n);
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i) {
    lens[i] = uint16_t(40 + r.next() % 8960);
    offs[i] = total;
    total += lens[i];
  }
  std::vector<uint8_t> bytes(total + 64);
  for (auto& b : bytes) {
    b = uint8_t(r.next());
  }
  uint8_t* d_arena = to_device(bytes);
  uint64_t* d_offs = to_device(offs);
  uint16_t* d_lens = to_device(lens);
  uint32_t* src = to_device(std::vector<uint32_t>(n, ip4(10, 1, 0, 1)));
  uint32_t* dst = to_device(std::vector<uint32_t>(n, ip4(10, 1, 0, 2)));
  // segmentation: 24 super-frames of 1-60 KB payload, 2 KiB-aligned in
  std::vector<uint8_t> frames;
  std::vector<uint64_t> foffs;
  std::vector<uint16_t> flens;
  for (int k = 0; k < 24; ++k) {
    const std::vector<uint8_t> f = tcp_frame(r, 1000 + r.next() % 59000);
    foffs.push_back(frames.size());
    flens.push_back(uint16_t(f.size()));
    frames.insert(frames.end(), f.begin(), f.end());
    frames.resize((frames.size() + 2047) & ~size_t(2047));
  }
  const uint32_t nf = uint32_t(foffs.size()), mss = 1460, ostride = 2048, cap = 1024;
  uint8_t* d_frames = to_device(frames);
  uint64_t* d_foffs = to_device(foffs);
  uint16_t* d_flens = to_device(flens);

  struct Outs
  {
    uint16_t* csum;
    uint32_t* bad;
    uint16_t* arena;
    uint8_t* seg;
    uint16_t* seg_lens;
    uint32_t* first;
  };
  auto make_outs = [&]() {
    Outs o{};
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&o.csum), n * 2));
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&o.bad), 4));
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&o.arena), n * 2));
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&o.seg), size_t(cap) * ostride));
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&o.seg_lens), cap * 2));
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&o.first), (nf + 1) * 4));
    return o;
  };
  auto clear = [&](const Outs& o, hipStream_t s) {
    HIP_OK(hipMemsetAsync(o.csum, 0xA5, n * 2, s));
    HIP_OK(hipMemsetAsync(o.bad, 0xA5, 4, s));
    HIP_OK(hipMemsetAsync(o.arena, 0xA5, n * 2, s));
    HIP_OK(hipMemsetAsync(o.seg, 0xA5, size_t(cap) * ostride, s));
    HIP_OK(hipMemsetAsync(o.seg_lens, 0xA5, cap * 2, s));
    HIP_OK(hipMemsetAsync(o.first, 0xA5, (nf + 1) * 4, s));
  };
  auto calls = [&](const Outs& o, hipStream_t s) {
    CS_OK(tulips_csum_verify(d_arena, d_offs, d_lens, src, dst, o.csum, o.bad, n,
                             TULIPS_CSUM_TCP, s));
    CS_OK(tulips_csum_batch_arena(d_arena, total, d_offs, d_lens, nullptr, nullptr, nullptr,
                                  o.arena, n, TULIPS_CSUM_INET, s));
    CS_OK(tulips_csum_segment_frames(d_frames, d_foffs, d_flens, nf, mss, o.seg, ostride, cap,
                                     o.seg_lens, o.first, s));
  };
  struct Snap
  {
    std::vector<uint16_t> csum, arena, seg_lens;
    std::vector<uint32_t> bad, first;
    std::vector<uint8_t> seg;
    bool operator==(const Snap& b) const
    {
      return csum == b.csum && arena == b.arena && seg_lens == b.seg_lens && bad == b.bad &&
             first == b.first && seg == b.seg;
    }
  };
  auto snap = [&](const Outs& o) {
    Snap x;
    x.csum = to_host(o.csum, n);
    x.bad = to_host(o.bad, 1);
    x.arena = to_host(o.arena, n);
    x.first = to_host(o.first, nf + 1);
    x.seg_lens = to_host(o.seg_lens, cap);
    x.seg = to_host(o.seg, size_t(cap) * ostride);
    return x;
  };

  hipStream_t s = nullptr, other = nullptr;
  HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  HIP_OK(hipStreamCreateWithFlags(&other, hipStreamNonBlocking));
  const Outs direct = make_outs(), replay = make_outs();
  clear(direct, s);
  calls(direct, s);
  HIP_OK(hipStreamSynchronize(s));
  const Snap want = snap(direct);
  const uint32_t segs = want.first[nf];
  uint32_t mismatches = 0;
  auto cycle = [&](uint32_t c, bool check_all) {
    hipGraph_t g = nullptr;
    HIP_OK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    calls(replay, s);
    HIP_OK(hipStreamEndCapture(s, &g));
    hipGraphExec_t x = nullptr;
    HIP_OK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    HIP_OK(hipGraphDestroy(g)); // as torch.cuda.CUDAGraph does
    for (int rep = 0; rep < 2; ++rep) {
      hipStream_t on = rep ? other : s;
      clear(replay, on);
      HIP_OK(hipGraphLaunch(x, on));
      HIP_OK(hipStreamSynchronize(on));
      // a direct call on the capture stream between replays
      if (rep == 0) {
        calls(direct, s);
      }
      if (check_all || c % 25 == 0) {
        mismatches += snap(replay) == want ? 0 : 1;
      } else {
        mismatches += to_host(replay.bad, 1) == want.bad && to_host(replay.arena, n) == want.arena
                        ? 0
                        : 1;
      }
    }
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipGraphExecDestroy(x));
  };
  // the library's next uncaptured call frees what the destroyed graphs held
  auto free_now = [&]() {
    calls(direct, s);
    HIP_OK(hipDeviceSynchronize());
    size_t f = 0, t = 0;
    HIP_OK(hipMemGetInfo(&f, &t));
    return f;
  };
  // warm-up: the runtime's own first-use pools (graph instantiation, kernel
  // arguments) are made here, before the measured cycles
  for (uint32_t c = 0; c < 5; ++c) {
    cycle(c, true);
  }
  const size_t free0 = free_now();
  size_t free_half = 0;
  for (uint32_t c = 0; c < cycles; ++c) {
    cycle(c, c + 1 == cycles);
    if (c + 1 == cycles / 2) {
      free_half = free_now();
    }
  }
  const size_t free1 = free_now();
  mismatches += snap(direct) == want ? 0 : 1;
  const long long grew = (long long)free0 - (long long)free1;
  const bool ok = mismatches == 0 && grew < (1ll << 20);
  printf("{\"graph_cycles\": %u, \"segments\": %u, \"mismatches\": %u, \"free_before\": %zu, "
         "\"free_half\": %zu, \"free_after\": %zu, \"device_memory_growth\": %lld, "
         "\"ok\": %s, \"runtime\": %s}\n",
         cycles, segs, mismatches, free0, free_half, free1, grew, ok ? "true" : "false",
         runtime_json().c_str());
  CS_OK(tulips_csum_release_stream(s));
  CS_OK(tulips_csum_release_stream(other));
  HIP_OK(hipStreamDestroy(s));
  HIP_OK(hipStreamDestroy(other));
  return ok ? 0 : 1;
}

// ---- graph ownership across threads --------------------------------------------
// THREADS host threads, each on its own stream, capture (thread-local mode)
// counting verify + arena batch + segmentation, instantiate, destroy the
// template, replay, check, destroy the executable - so user-object
// destructors fire on every thread and several threads reclaim at once -
// with direct calls between, for SECONDS. Every replay's outputs equal the
// direct calls' made before the threads start; at the end (streams released)
// device memory is back within 32 MiB of where it was after a warm-up (the
// runtime keeps per-thread pools, 4 MiB measured; the graphs' own arrays,
// leaked, would be at least 4 KiB each, hundreds of MiB).
int
cmd_thread_churn(double seconds, uint32_t nthreads)
{
  Rng r{ 0x7468726561647321ull };
  const uint32_t n = 4096;
  std::vector<uint16_t> lens(n);
  std::vector<uint64_t> offs(n);
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i) {
    lens[i] = uint16_t(40 + r.next() % 8960);
    offs[i] = total;
    total += lens[i];
  }
  std::vector<uint8_t> bytes(total + 64);
  for (auto& b : bytes) {
    b = uint8_t(r.next());
  }
  uint8_t* d_arena = to_device(bytes);
  uint64_t* d_offs = to_device(offs);
  uint16_t* d_lens = to_device(lens);
  uint32_t* src = to_device(std::vector<uint32_t>(n, ip4(10, 1, 0, 1)));
  uint32_t* dst = to_device(std::vector<uint32_t>(n, ip4(10, 1, 0, 2)));
  std::vector<uint8_t> frames;
  std::vector<uint64_t> foffs;
  std::vector<uint16_t> flens;
  for (int k = 0; k < 16; ++k) {
    const std::vector<uint8_t> f = tcp_frame(r, 1000 + r.next() % 59000);
    foffs.push_back(frames.size());
    flens.push_back(uint16_t(f.size()));
    frames.insert(frames.end(), f.begin(), f.end());
    frames.resize((frames.size() + 2047) & ~size_t(2047));
  }
  const uint32_t nf = uint32_t(foffs.size()), mss = 1460, ostride = 2048, cap = 1024;
  uint8_t* d_frames = to_device(frames);
  uint64_t* d_foffs = to_device(foffs);
  uint16_t* d_flens = to_device(flens);

  struct Outs
  {
    uint16_t* csum = nullptr;
    uint32_t* bad = nullptr;
    uint16_t* arena = nullptr;
    uint8_t* seg = nullptr;
    uint16_t* seg_lens = nullptr;
    uint32_t* first = nullptr;
  };
  auto make_outs = [&]() {
    Outs o;
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&o.csum), n * 2));
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&o.bad), 4));
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&o.arena), n * 2));
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&o.seg), size_t(cap) * ostride));
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&o.seg_lens), cap * 2));
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&o.first), (nf + 1) * 4));
    return o;
  };
  auto free_outs = [](const Outs& o) {
    for (void* q : { static_cast<void*>(o.csum), static_cast<void*>(o.bad),
                     static_cast<void*>(o.arena), static_cast<void*>(o.seg),
                     static_cast<void*>(o.seg_lens), static_cast<void*>(o.first) }) {
      (void)hipFree(q);
    }
  };
  auto clear = [&](const Outs& o, hipStream_t s) {
    HIP_OK(hipMemsetAsync(o.csum, 0xA5, n * 2, s));
    HIP_OK(hipMemsetAsync(o.bad, 0xA5, 4, s));
    HIP_OK(hipMemsetAsync(o.arena, 0xA5, n * 2, s));
    HIP_OK(hipMemsetAsync(o.seg, 0xA5, size_t(cap) * ostride, s));
    HIP_OK(hipMemsetAsync(o.seg_lens, 0xA5, cap * 2, s));
    HIP_OK(hipMemsetAsync(o.first, 0xA5, (nf + 1) * 4, s));
  };
  auto calls = [&](const Outs& o, hipStream_t s) {
    CS_OK(tulips_csum_verify(d_arena, d_offs, d_lens, src, dst, o.csum, o.bad, n,
                             TULIPS_CSUM_TCP, s));
    CS_OK(tulips_csum_batch_arena(d_arena, total, d_offs, d_lens, nullptr, nullptr, nullptr,
                                  o.arena, n, TULIPS_CSUM_INET, s));
    CS_OK(tulips_csum_segment_frames(d_frames, d_foffs, d_flens, nf, mss, o.seg, ostride, cap,
                                     o.seg_lens, o.first, s));
  };
  // outputs copied back on the thread's own stream
  auto back = [](const void* p, size_t bytes, hipStream_t s) {
    std::vector<uint8_t> v(bytes);
    HIP_OK(hipMemcpyAsync(v.data(), p, bytes, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return v;
  };
  struct Snap
  {
    std::vector<uint8_t> csum, bad, arena, seg, seg_lens, first;
    bool operator==(const Snap& b) const
    {
      return csum == b.csum && bad == b.bad && arena == b.arena && seg == b.seg &&
             seg_lens == b.seg_lens && first == b.first;
    }
  };
  auto snap = [&](const Outs& o, hipStream_t s) {
    Snap x;
    x.csum = back(o.csum, n * 2, s);
    x.bad = back(o.bad, 4, s);
    x.arena = back(o.arena, n * 2, s);
    x.seg = back(o.seg, size_t(cap) * ostride, s);
    x.seg_lens = back(o.seg_lens, cap * 2, s);
    x.first = back(o.first, (nf + 1) * 4, s);
    return x;
  };

  // reference outputs, and a single-thread warm-up of the same cycle
  hipStream_t s0 = nullptr;
  HIP_OK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  const Outs o0 = make_outs();
  clear(o0, s0);
  calls(o0, s0);
  HIP_OK(hipStreamSynchronize(s0));
  const Snap want = snap(o0, s0);
  auto cycle = [&](hipStream_t s, const Outs& o, bool full) {
    hipGraph_t g = nullptr;
    HIP_OK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    calls(o, s);
    HIP_OK(hipStreamEndCapture(s, &g));
    hipGraphExec_t x = nullptr;
    HIP_OK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    HIP_OK(hipGraphDestroy(g));
    clear(o, s);
    HIP_OK(hipStreamSynchronize(s)); // the launch stream idle
    HIP_OK(hipGraphLaunch(x, s));
    HIP_OK(hipStreamSynchronize(s));
    bool ok;
    if (full) {
      ok = snap(o, s) == want;
    } else {
      ok = back(o.bad, 4, s) == want.bad && back(o.arena, n * 2, s) == want.arena &&
           back(o.first, (nf + 1) * 4, s) == want.first;
    }
    HIP_OK(hipGraphExecDestroy(x));
    return ok;
  };
  for (int c = 0; c < 5; ++c) {
    if (!cycle(s0, o0, true)) {
      fprintf(stderr, "warm-up cycle %d mismatched\n", c);
      return 1;
    }
  }
  calls(o0, s0); // reclaims the warm-up graphs' arrays
  HIP_OK(hipDeviceSynchronize());
  size_t free0 = 0, tot = 0;
  HIP_OK(hipMemGetInfo(&free0, &tot));

  std::atomic<uint64_t> cycles{ 0 }, mism{ 0 }, directs{ 0 };
  const auto t_end =
    std::chrono::steady_clock::now() + std::chrono::milliseconds(int64_t(seconds * 1000));
  std::vector<std::thread> ts;
  for (uint32_t t = 0; t < nthreads; ++t) {
    ts.emplace_back([&, t] {
      hipStream_t s = nullptr;
      HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      const Outs o = make_outs(), od = make_outs();
      uint64_t c = 0;
      while (std::chrono::steady_clock::now() < t_end) {
        mism += cycle(s, o, c % 10 == t % 10) ? 0 : 1;
        ++c;
        if (c % 4 == 0) { // a direct call on the stream between graphs
          clear(od, s);
          calls(od, s);
          HIP_OK(hipStreamSynchronize(s));
          mism += back(od.arena, n * 2, s) == want.arena ? 0 : 1;
          ++directs;
        }
      }
      cycles += c;
      CS_OK(tulips_csum_release_stream(s));
      HIP_OK(hipStreamDestroy(s));
      free_outs(o);
      free_outs(od);
    });
  }
  for (auto& th : ts) {
    th.join();
  }
  calls(o0, s0); // frees what the last destroyed graphs held
  HIP_OK(hipDeviceSynchronize());
  mism += snap(o0, s0) == want ? 0 : 1;
  size_t free1 = 0;
  HIP_OK(hipMemGetInfo(&free1, &tot));
  const long long grew = (long long)free0 - (long long)free1;
  const bool ok = mism.load() == 0 && cycles.load() > 0 && grew < (32ll << 20);
  printf("{\"thread_churn\": {\"threads\": %u, \"seconds\": %.1f, \"graphs\": %llu, "
         "\"direct_calls\": %llu, \"mismatches\": %llu, \"device_memory_growth\": %lld, "
         "\"ok\": %s}, \"runtime\": %s}\n",
         nthreads, seconds, (unsigned long long)cycles.load(),
         (unsigned long long)directs.load(), (unsigned long long)mism.load(), grew,
         ok ? "true" : "false", runtime_json().c_str());
  CS_OK(tulips_csum_release_stream(s0));
  HIP_OK(hipStreamDestroy(s0));
  free_outs(o0);
  for (void* q : { static_cast<void*>(d_arena), static_cast<void*>(d_offs),
                   static_cast<void*>(d_lens), static_cast<void*>(src), static_cast<void*>(dst),
                   static_cast<void*>(d_frames), static_cast<void*>(d_foffs),
                   static_cast<void*>(d_flens) }) {
    (void)hipFree(q);
  }
  return ok ? 0 : 1;
}

// ---- multi-branch graph churn ---------------------------------------------------
// The capture/replay/destroy churn that faults inside hipGraphLaunch on the
// runtime torch bundles (profiles/graph_crash_r05.txt), run here
// on /opt/rocm's runtime with library calls as the graph's kernels: graphs of
// 1-6 tulips_csum_batch_fixed calls round-robin over 1-4 side streams forked
// from and joined to the capture stream, at most 8 live (a new capture
// destroys a random one), replays on a pool of other streams with every
// output checked, direct calls between, random drops. Prints one progress
// line a second; a fault ends the process.
int
cmd_graph_churn(double seconds, uint64_t seed)
{
  Rng r{ seed * 0x9E3779B97F4A7C15ull + 1 };
  const uint32_t n = 4096, L = 1500;
  std::vector<uint8_t> bytes(size_t(n) * L + 64);
  for (auto& b : bytes) {
    b = uint8_t(r.next());
  }
  uint8_t* arena = to_device(bytes);
  uint16_t* ref = nullptr;
  HIP_OK(hipMalloc(reinterpret_cast<void**>(&ref), n * 2));
  CS_OK(tulips_csum_batch_fixed(arena, L, L, nullptr, nullptr, nullptr, ref, n,
                                TULIPS_CSUM_RAW, nullptr));
  HIP_OK(hipDeviceSynchronize());
  const std::vector<uint16_t> want = to_host(ref, n);
  struct Live
  {
    hipGraphExec_t x;
    std::vector<uint16_t*> outs;
    uint32_t nside;
  };
  const bool presync = getenv("CHURN_PRESYNC") != nullptr;
  const bool devsync = getenv("CHURN_DEVSYNC") != nullptr;
  // diagnostic: poison with a kernel (the library's checksum of an all-zero
  // arena: 0x0000 words) instead of hipMemsetAsync
  const bool kpoison = getenv("CHURN_KERNEL_POISON") != nullptr;
  // diagnostic: never destroy a graph (at most 8 are made, then only replays)
  const bool nodrop = getenv("CHURN_NODROP") != nullptr;
  // diagnostic: give every graph one root node (a 4-byte memset on the
  // capture stream before the fork), so every branch depends on it
  const bool one_root = getenv("CHURN_ONE_ROOT") != nullptr;
  uint32_t* scratch = nullptr;
  HIP_OK(hipMalloc(reinterpret_cast<void**>(&scratch), 64));
  uint8_t* zeros = nullptr;
  HIP_OK(hipMalloc(reinterpret_cast<void**>(&zeros), size_t(n) * L + 64));
  HIP_OK(hipMemset(zeros, 0, size_t(n) * L + 64));
  HIP_OK(hipDeviceSynchronize());
  const uint16_t poison_word = kpoison ? 0x0000 : 0xA5A5;
  std::vector<Live> live;
  auto drop = [&](size_t k) {
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipGraphExecDestroy(live[k].x));
    for (uint16_t* o : live[k].outs) {
      HIP_OK(hipFree(o));
    }
    live.erase(live.begin() + long(k));
  };
  std::vector<hipStream_t> pool(4);
  for (auto& p : pool) {
    HIP_OK(hipStreamCreateWithFlags(&p, hipStreamNonBlocking));
  }
  uint64_t steps = 0, captures = 0, replays = 0, destroyed = 0, bad = 0;
  const auto t0 = std::chrono::steady_clock::now();
  auto last = t0;
  for (;;) {
    const auto now = std::chrono::steady_clock::now();
    const double el = std::chrono::duration<double>(now - t0).count();
    if (el >= seconds) {
      break;
    }
    if (std::chrono::duration<double>(now - last).count() >= 1.0) {
      last = now;
      printf("{\"progress_s\": %.0f, \"steps\": %llu}\n", el, (unsigned long long)steps);
      fflush(stdout);
    }
    uint32_t op = r.next() % 100;
    if (nodrop && live.size() >= 8 && (op < 30 || op >= 95)) {
      op = 50; // a replay instead of a capture or a drop
    }
    if (op < 30 || live.empty()) {
      const uint32_t ncalls = 1 + r.next() % 6, nside = 1 + r.next() % 4;
      hipStream_t cap = nullptr;
      std::vector<hipStream_t> side(nside);
      HIP_OK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
      for (auto& sd : side) {
        HIP_OK(hipStreamCreateWithFlags(&sd, hipStreamNonBlocking));
      }
      Live g{};
      g.nside = nside;
      for (uint32_t c = 0; c < ncalls; ++c) {
        uint16_t* o = nullptr;
        HIP_OK(hipMalloc(reinterpret_cast<void**>(&o), n * 2));
        g.outs.push_back(o);
      }
      hipEvent_t fork = nullptr;
      std::vector<hipEvent_t> joins(nside);
      HIP_OK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
      for (auto& e : joins) {
        HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      }
      HIP_OK(hipStreamBeginCapture(cap, hipStreamCaptureModeGlobal));
      if (one_root) {
        HIP_OK(hipMemsetAsync(scratch, 0, 4, cap));
      }
      HIP_OK(hipEventRecord(fork, cap));
      for (auto& sd : side) {
        HIP_OK(hipStreamWaitEvent(sd, fork, 0));
      }
      for (uint32_t c = 0; c < ncalls; ++c) {
        CS_OK(tulips_csum_batch_fixed(arena, L, L, nullptr, nullptr, nullptr, g.outs[c], n,
                                      TULIPS_CSUM_RAW, side[c % nside]));
      }
      for (uint32_t k = 0; k < nside; ++k) {
        HIP_OK(hipEventRecord(joins[k], side[k]));
        HIP_OK(hipStreamWaitEvent(cap, joins[k], 0));
      }
      hipGraph_t graph = nullptr;
      HIP_OK(hipStreamEndCapture(cap, &graph));
      HIP_OK(hipGraphInstantiate(&g.x, graph, nullptr, nullptr, 0));
      HIP_OK(hipGraphDestroy(graph));
      HIP_OK(hipEventDestroy(fork));
      for (auto& e : joins) {
        HIP_OK(hipEventDestroy(e));
      }
      for (auto& sd : side) {
        HIP_OK(hipStreamDestroy(sd));
      }
      HIP_OK(hipStreamDestroy(cap));
      live.push_back(g);
      ++captures;
      if (live.size() > 8) {
        drop(r.next() % live.size());
        ++destroyed;
      }
    } else if (op < 75) {
      Live& g = live[r.next() % live.size()];
      hipStream_t on = pool[r.next() % pool.size()];
      // poisoned in the replay stream's order (a plain hipMemset is not
      // ordered with non-blocking streams)
      for (uint16_t* o : g.outs) {
        if (kpoison) {
          CS_OK(tulips_csum_batch_fixed(zeros, L, L, nullptr, nullptr, nullptr, o, n,
                                        TULIPS_CSUM_RAW, on));
        } else {
          HIP_OK(hipMemsetAsync(o, 0xA5, n * 2, on));
        }
      }
      if (presync) { // diagnostic: the poison complete before the launch
        HIP_OK(hipStreamSynchronize(on));
      }
      HIP_OK(hipGraphLaunch(g.x, on));
      if (devsync) { // diagnostic: wait for the whole device, not the stream
        HIP_OK(hipDeviceSynchronize());
      } else {
        HIP_OK(hipStreamSynchronize(on));
      }
      for (size_t c = 0; c < g.outs.size(); ++c) {
        const std::vector<uint16_t> got = to_host(g.outs[c], n);
        if (got != want) {
          ++bad;
          uint32_t poison = 0, wrong = 0, first = n;
          for (uint32_t k = 0; k < n; ++k) {
            if (got[k] != want[k]) {
              poison += got[k] == poison_word ? 1 : 0;
              wrong += got[k] != poison_word ? 1 : 0;
              first = std::min(first, k);
            }
          }
          // read again after the whole device has idled: right now (the
          // graph's kernel finished after the replay stream's sync: the end
          // of the replay unordered) or still poisoned (the kernel ran
          // before the poison: the start unordered)
          std::this_thread::sleep_for(std::chrono::milliseconds(2));
          HIP_OK(hipDeviceSynchronize());
          const bool late_ok = to_host(g.outs[c], n) == want;
          if (bad <= 12) {
            printf("{\"mismatch\": \"replay\", \"step\": %llu, \"call\": %zu, \"calls\": %zu, "
                   "\"branches\": %u, \"poison_words\": %u, \"wrong_words\": %u, "
                   "\"first\": %u, \"right_after_idle\": %s}\n",
                   (unsigned long long)steps, c, g.outs.size(), g.nside, poison, wrong, first,
                   late_ok ? "true" : "false");
            fflush(stdout);
          }
        }
      }
      ++replays;
    } else if (op < 95) {
      hipStream_t on = pool[r.next() % pool.size()];
      HIP_OK(hipMemsetAsync(ref, 0xA5, n * 2, on));
      CS_OK(tulips_csum_batch_fixed(arena, L, L, nullptr, nullptr, nullptr, ref, n,
                                    TULIPS_CSUM_RAW, on));
      HIP_OK(hipStreamSynchronize(on));
      if (to_host(ref, n) != want) {
        ++bad;
        if (bad <= 12) {
          printf("{\"mismatch\": \"direct\", \"step\": %llu}\n", (unsigned long long)steps);
          fflush(stdout);
        }
      }
    } else {
      drop(r.next() % live.size());
      ++destroyed;
    }
    ++steps;
  }
  while (!live.empty()) {
    drop(0);
  }
  printf("{\"graph_churn_s\": %.1f, \"steps\": %llu, \"captures\": %llu, \"replays\": %llu, "
         "\"destroyed\": %llu, \"mismatches\": %llu, \"ok\": %s, \"runtime\": %s}\n",
         seconds, (unsigned long long)steps, (unsigned long long)captures,
         (unsigned long long)replays, (unsigned long long)destroyed, (unsigned long long)bad,
         bad ? "false" : "true", runtime_json().c_str());
  for (auto& p : pool) {
    HIP_OK(hipStreamDestroy(p));
  }
  (void)hipFree(arena);
  (void)hipFree(ref);
  (void)hipFree(zeros);
  (void)hipFree(scratch);
  return bad ? 1 : 0;
}

// ---- serial rate ------------------------------------------------------------------
// The headline kernel's one-launch-at-a-time rate on this runtime: NB batches
// of 65,536 segments of L bytes (the §8c arena, rotated so every launch
// streams from HBM), a chain of 256 tulips_csum_batch_fixed launches captured
// in one single-stream graph, timed with HIP events over 5 replays (median),
// every batch's digest checked against `want` (the §8c FNV of batch 0).
int
cmd_serial_rate(uint32_t L, uint32_t nb, const char* want0)
{
  const uint64_t bb = uint64_t(NSEG) * L;
  std::vector<uint8_t> host(nb * bb + 64, 0);
  splitmix_fill(host.data(), nb * bb);
  uint8_t* arena = to_device(host);
  host.clear();
  host.shrink_to_fit();
  uint16_t* out = nullptr;
  HIP_OK(hipMalloc(reinterpret_cast<void**>(&out), size_t(nb) * NSEG * 2));
  hipStream_t s = nullptr;
  HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  constexpr int CHAIN = 256;
  auto launch = [&](int i) {
    const uint32_t b = uint32_t(i) % nb;
    CS_OK(tulips_csum_batch_fixed(arena + b * bb, L, L, nullptr, nullptr, nullptr,
                                  out + size_t(b) * NSEG, NSEG, TULIPS_CSUM_RAW, s));
  };
  for (uint32_t i = 0; i < nb; ++i) {
    launch(int(i));
  }
  HIP_OK(hipStreamSynchronize(s));
  hipGraph_t g = nullptr;
  HIP_OK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < CHAIN; ++i) {
    launch(i);
  }
  HIP_OK(hipStreamEndCapture(s, &g));
  hipGraphExec_t x = nullptr;
  HIP_OK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  HIP_OK(hipGraphDestroy(g));
  HIP_OK(hipGraphLaunch(x, s)); // warm
  HIP_OK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  std::vector<double> us;
  for (int rep = 0; rep < 5; ++rep) {
    HIP_OK(hipMemsetAsync(out, 0xA5, size_t(nb) * NSEG * 2, s));
    HIP_OK(hipEventRecord(e0, s));
    HIP_OK(hipGraphLaunch(x, s));
    HIP_OK(hipEventRecord(e1, s));
    HIP_OK(hipEventSynchronize(e1));
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    us.push_back(double(ms) * 1e3 / CHAIN);
  }
  std::sort(us.begin(), us.end());
  const double med = us[us.size() / 2];
  const std::vector<uint16_t> b0 = to_host(out, NSEG);
  const std::string d0 = hex64(fnv1a_u16(b0));
  const bool ok = d0 == want0;
  const double frac = double(bb) / (med * 1e-6) / 8e12;
  printf("{\"serial_rate\": {\"length\": %u, \"batches\": %u, \"chain\": %d, \"us_per_launch\": %.3f, "
         "\"frac_of_8TBps\": %.4f, \"GiBps\": %.1f, \"batch0_fnv1a64\": \"%s\", \"parity\": \"%s\"}, "
         "\"runtime\": %s}\n",
         L, nb, CHAIN, med, frac, double(bb) / (med * 1e-6) / 1073741824.0, d0.c_str(),
         ok ? "ok" : "MISMATCH", runtime_json().c_str());
  HIP_OK(hipGraphExecDestroy(x));
  HIP_OK(hipStreamDestroy(s));
  (void)hipFree(arena);
  (void)hipFree(out);
  return ok ? 0 : 1;
}

// ---- stateful multi-branch churn --------------------------------------------------
// Graph ownership under churn (stream_state.h): graphs of 1-6 library calls of
// every stateful kind — counting verify (counter shards), arena batch (span
// words), segmentation (workspace) — and the stateless fixed batch,
// round-robin over 1-4 side streams forked from and joined to the capture
// stream (each side stream's state attaches its own user object to the
// graph), at most 8 live, a new capture destroying a random one; replays on
// a pool of other streams with every output checked against the direct
// calls'; random drops. The launch stream is idle before each replay (the
// /opt/rocm runtime can start a multi-branch graph before the launch
// stream's pending work). At the end every graph is destroyed,
// one direct call reclaims their arrays, and device memory must be back
// within 4 MiB of where it stood after the warm-up.
int
cmd_graph_churn_stateful(double seconds, uint64_t seed)
{
  Rng r{ seed * 0x9E3779B97F4A7C15ull + 7 };
  const uint32_t n = 2048, L = 1500;
  std::vector<uint8_t> bytes(size_t(n) * 9000 + 64);
  for (auto& b : bytes) {
    b = uint8_t(r.next());
  }
  std::vector<uint16_t> lens(n);
  std::vector<uint64_t> offs(n);
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i) {
    lens[i] = uint16_t(40 + r.next() % 8960);
    offs[i] = total;
    total += lens[i];
  }
  uint8_t* d_bytes = to_device(bytes);
  uint64_t* d_offs = to_device(offs);
  uint16_t* d_lens = to_device(lens);
  uint32_t* src = to_device(std::vector<uint32_t>(n, ip4(10, 1, 0, 1)));
  uint32_t* dst = to_device(std::vector<uint32_t>(n, ip4(10, 1, 0, 2)));
  std::vector<uint8_t> frames;
  std::vector<uint64_t> foffs;
  std::vector<uint16_t> flens;
  for (int k = 0; k < 16; ++k) {
    const std::vector<uint8_t> f = tcp_frame(r, 1000 + r.next() % 30000);
    foffs.push_back(frames.size());
    flens.push_back(uint16_t(f.size()));
    frames.insert(frames.end(), f.begin(), f.end());
    frames.resize((frames.size() + 2047) & ~size_t(2047));
  }
  const uint32_t nf = uint32_t(foffs.size()), mss = 1460, ostride = 2048, cap_seg = 512;
  uint8_t* d_frames = to_device(frames);
  uint64_t* d_foffs = to_device(foffs);
  uint16_t* d_flens = to_device(flens);
  // a call's output buffers, by kind: 0 fixed, 1 verify, 2 arena, 3 segmentation
  struct Out
  {
    int kind;
    std::vector<void*> bufs;
    std::vector<size_t> sizes;
  };
  auto make_out = [&](int kind) {
    Out o{ kind, {}, {} };
    std::vector<size_t> sz;
    switch (kind) {
      case 0: sz = { n * 2 }; break;
      case 1: sz = { n * 2, 4 }; break;
      case 2: sz = { n * 2 }; break;
      default: sz = { size_t(cap_seg) * ostride, cap_seg * 2, (nf + 1) * 4 }; break;
    }
    for (size_t b : sz) {
      void* p = nullptr;
      HIP_OK(hipMalloc(&p, b));
      o.bufs.push_back(p);
      o.sizes.push_back(b);
    }
    return o;
  };
  auto call = [&](const Out& o, hipStream_t st) {
    switch (o.kind) {
      case 0:
        CS_OK(tulips_csum_batch_fixed(d_bytes, L, L, nullptr, nullptr, nullptr,
                                      static_cast<uint16_t*>(o.bufs[0]), n, TULIPS_CSUM_RAW, st));
        break;
      case 1:
        CS_OK(tulips_csum_verify(d_bytes, d_offs, d_lens, src, dst,
                                 static_cast<uint16_t*>(o.bufs[0]),
                                 static_cast<uint32_t*>(o.bufs[1]), n, TULIPS_CSUM_TCP, st));
        break;
      case 2:
        CS_OK(tulips_csum_batch_arena(d_bytes, total, d_offs, d_lens, nullptr, nullptr, nullptr,
                                      static_cast<uint16_t*>(o.bufs[0]), n, TULIPS_CSUM_INET,
                                      st));
        break;
      default:
        CS_OK(tulips_csum_segment_frames(d_frames, d_foffs, d_flens, nf, mss,
                                         static_cast<uint8_t*>(o.bufs[0]), ostride, cap_seg,
                                         static_cast<uint16_t*>(o.bufs[1]),
                                         static_cast<uint32_t*>(o.bufs[2]), st));
        break;
    }
  };
  auto poison = [&](const Out& o, hipStream_t st) {
    for (size_t b = 0; b < o.bufs.size(); ++b) {
      HIP_OK(hipMemsetAsync(o.bufs[b], 0xA5, o.sizes[b], st));
    }
  };
  auto snap = [&](const Out& o) {
    std::vector<std::vector<uint8_t>> v;
    for (size_t b = 0; b < o.bufs.size(); ++b) {
      v.push_back(to_host(static_cast<const uint8_t*>(o.bufs[b]), o.sizes[b]));
    }
    if (o.kind == 3) { // segment slots past each segment's length are not written
      const uint16_t* ol = reinterpret_cast<const uint16_t*>(v[1].data());
      const uint32_t segs =
        std::min<uint32_t>(reinterpret_cast<const uint32_t*>(v[2].data())[nf], cap_seg);
      for (uint32_t j = 0; j < cap_seg; ++j) {
        const uint32_t keep = j < segs ? ol[j] : 0;
        std::fill(v[0].begin() + size_t(j) * ostride + keep,
                  v[0].begin() + size_t(j + 1) * ostride, uint8_t(0));
      }
    }
    return v;
  };
  hipStream_t ds = nullptr;
  HIP_OK(hipStreamCreateWithFlags(&ds, hipStreamNonBlocking));
  std::vector<std::vector<std::vector<uint8_t>>> want(4);
  std::vector<Out> ref;
  for (int k = 0; k < 4; ++k) {
    ref.push_back(make_out(k));
    poison(ref[k], ds);
    call(ref[k], ds);
    HIP_OK(hipStreamSynchronize(ds));
    want[k] = snap(ref[k]);
  }
  struct Live
  {
    hipGraphExec_t x;
    std::vector<Out> outs;
  };
  std::vector<Live> live;
  auto free_out = [&](Out& o) {
    for (void* p : o.bufs) {
      HIP_OK(hipFree(p));
    }
  };
  auto drop = [&](size_t k) {
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipGraphExecDestroy(live[k].x));
    for (Out& o : live[k].outs) {
      free_out(o);
    }
    live.erase(live.begin() + long(k));
  };
  std::vector<hipStream_t> pool(4);
  for (auto& p : pool) {
    HIP_OK(hipStreamCreateWithFlags(&p, hipStreamNonBlocking));
  }
  auto free_now = [&]() {
    for (int k = 0; k < 4; ++k) { // direct calls of every kind reclaim
      call(ref[k], ds);
    }
    HIP_OK(hipDeviceSynchronize());
    size_t f = 0, t = 0;
    HIP_OK(hipMemGetInfo(&f, &t));
    return f;
  };
  uint64_t steps = 0, captures = 0, replays = 0, destroyed = 0, bad = 0;
  size_t free0 = 0, free_half = 0;
  const auto t0 = std::chrono::steady_clock::now();
  auto last = t0;
  for (;;) {
    const auto now = std::chrono::steady_clock::now();
    const double el = std::chrono::duration<double>(now - t0).count();
    if (el >= seconds) {
      break;
    }
    if (std::chrono::duration<double>(now - last).count() >= 1.0) {
      last = now;
      printf("{\"progress_s\": %.0f, \"steps\": %llu}\n", el, (unsigned long long)steps);
      fflush(stdout);
    }
    if (steps == 40 || (!free_half && free0 && el >= seconds / 2)) {
      // after a warm-up of captures, replays and drops, and half-way: every
      // graph destroyed, their arrays reclaimed
      while (!live.empty()) {
        drop(0);
        ++destroyed;
      }
      (free0 ? free_half : free0) = free_now();
    }
    const uint32_t op = r.next() % 100;
    if (op < 30 || live.empty()) {
      const uint32_t ncalls = 1 + r.next() % 6, nside = 1 + r.next() % 4;
      hipStream_t cap = nullptr;
      std::vector<hipStream_t> side(nside);
      HIP_OK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
      for (auto& sd : side) {
        HIP_OK(hipStreamCreateWithFlags(&sd, hipStreamNonBlocking));
      }
      Live g{};
      for (uint32_t c = 0; c < ncalls; ++c) {
        g.outs.push_back(make_out(int(r.next() % 4)));
      }
      hipEvent_t fork = nullptr;
      std::vector<hipEvent_t> joins(nside);
      HIP_OK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
      for (auto& e : joins) {
        HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      }
      HIP_OK(hipStreamBeginCapture(cap, hipStreamCaptureModeGlobal));
      HIP_OK(hipEventRecord(fork, cap));
      for (auto& sd : side) {
        HIP_OK(hipStreamWaitEvent(sd, fork, 0));
      }
      for (uint32_t c = 0; c < ncalls; ++c) {
        call(g.outs[c], side[c % nside]);
      }
      for (uint32_t k = 0; k < nside; ++k) {
        HIP_OK(hipEventRecord(joins[k], side[k]));
        HIP_OK(hipStreamWaitEvent(cap, joins[k], 0));
      }
      hipGraph_t graph = nullptr;
      HIP_OK(hipStreamEndCapture(cap, &graph));
      HIP_OK(hipGraphInstantiate(&g.x, graph, nullptr, nullptr, 0));
      HIP_OK(hipGraphDestroy(graph));
      HIP_OK(hipEventDestroy(fork));
      for (auto& e : joins) {
        HIP_OK(hipEventDestroy(e));
      }
      // the library's state of these streams goes with them; the arrays the
      // capture took stay with the graph
      CS_OK(tulips_csum_release_stream(cap));
      for (auto& sd : side) {
        CS_OK(tulips_csum_release_stream(sd));
        HIP_OK(hipStreamDestroy(sd));
      }
      HIP_OK(hipStreamDestroy(cap));
      live.push_back(std::move(g));
      ++captures;
      if (live.size() > 8) {
        drop(r.next() % live.size());
        ++destroyed;
      }
    } else if (op < 75) {
      Live& g = live[r.next() % live.size()];
      hipStream_t on = pool[r.next() % pool.size()];
      for (const Out& o : g.outs) {
        poison(o, on);
      }
      HIP_OK(hipStreamSynchronize(on)); // idle before a multi-branch launch
      HIP_OK(hipGraphLaunch(g.x, on));
      HIP_OK(hipStreamSynchronize(on));
      for (size_t c = 0; c < g.outs.size(); ++c) {
        if (snap(g.outs[c]) != want[g.outs[c].kind]) {
          ++bad;
          if (bad <= 12) {
            printf("{\"mismatch\": \"replay\", \"step\": %llu, \"kind\": %d}\n",
                   (unsigned long long)steps, g.outs[c].kind);
            fflush(stdout);
          }
        }
      }
      ++replays;
    } else if (op < 95) {
      const int k = int(r.next() % 4);
      hipStream_t on = pool[r.next() % pool.size()];
      poison(ref[k], on);
      call(ref[k], on);
      HIP_OK(hipStreamSynchronize(on));
      if (snap(ref[k]) != want[k]) {
        ++bad;
        if (bad <= 12) {
          printf("{\"mismatch\": \"direct\", \"step\": %llu, \"kind\": %d}\n",
                 (unsigned long long)steps, k);
          fflush(stdout);
        }
      }
    } else {
      drop(r.next() % live.size());
      ++destroyed;
    }
    ++steps;
  }
  while (!live.empty()) {
    drop(0);
    ++destroyed;
  }
  const size_t free1 = free_now();
  // the second half's captures (about as many as the first's) must leave
  // nothing behind; the first half's growth (runtime pools of the streams and
  // graphs it made) is reported
  const long long grew_first = free_half ? (long long)free0 - (long long)free_half : 0;
  const long long grew_second = free_half ? (long long)free_half - (long long)free1 : 0;
  const bool ok = bad == 0 && free_half != 0 && grew_second < (4ll << 20);
  printf("{\"graph_churn_stateful_s\": %.1f, \"steps\": %llu, \"captures\": %llu, "
         "\"replays\": %llu, \"destroyed\": %llu, \"mismatches\": %llu, \"free_after_warmup\": %zu, "
         "\"free_half\": %zu, \"free_after\": %zu, \"growth_first_half\": %lld, "
         "\"growth_second_half\": %lld, \"ok\": %s, \"runtime\": %s}\n",
         seconds, (unsigned long long)steps, (unsigned long long)captures,
         (unsigned long long)replays, (unsigned long long)destroyed, (unsigned long long)bad,
         free0, free_half, free1, grew_first, grew_second, ok ? "true" : "false",
         runtime_json().c_str());
  for (auto& p : pool) {
    CS_OK(tulips_csum_release_stream(p));
    HIP_OK(hipStreamDestroy(p));
  }
  CS_OK(tulips_csum_release_stream(ds));
  HIP_OK(hipStreamDestroy(ds));
  return ok ? 0 : 1;
}

} // namespace

int
main(int argc, char** argv)
{
  if (argc < 2) {
    fprintf(stderr,
            "usage: %s runtime | zipf-lengths | parity NAME=FNV... | user-object | "
            "graph-cycles N | graph-churn[-stateful] SECONDS SEED | serial-rate L NBATCH FNV\n",
            argv[0]);
    return 2;
  }
  const std::string cmd = argv[1];
  if (cmd == "runtime") {
    printf("%s\n", runtime_json().c_str());
    return 0;
  }
  if (cmd == "zipf-lengths") { // no GPU: the §8c length sequence's digest and total
    const std::vector<uint16_t> zl = zipf_lengths(NSEG);
    uint64_t total = 0;
    for (uint16_t l : zl) {
      total += l;
    }
    printf("{\"fnv1a64\": \"%s\", \"total\": %llu}\n", hex64(fnv1a_u16(zl)).c_str(),
           static_cast<unsigned long long>(total));
    return 0;
  }
  if (cmd == "parity") {
    return cmd_parity(argc - 2, argv + 2);
  }
  if (cmd == "thread-churn" && argc == 4) {
    return cmd_thread_churn(atof(argv[2]), uint32_t(atoi(argv[3])));
  }
  if (cmd == "fixtures" && argc == 3) {
    return cmd_fixtures(argv[2]);
  }
  if (cmd == "capture-neutral") {
    return cmd_capture_neutral(argc - 2, argv + 2);
  }
  if (cmd == "user-object") {
    return cmd_user_object();
  }
  if (cmd == "serial-rate" && argc == 5) {
    return cmd_serial_rate(uint32_t(strtoul(argv[2], nullptr, 10)),
                           uint32_t(strtoul(argv[3], nullptr, 10)), argv[4]);
  }
  if (cmd == "graph-churn-stateful" && argc == 4) {
    return cmd_graph_churn_stateful(strtod(argv[2], nullptr), strtoull(argv[3], nullptr, 10));
  }
  if (cmd == "graph-churn" && argc == 4) {
    return cmd_graph_churn(strtod(argv[2], nullptr), strtoull(argv[3], nullptr, 10));
  }
  if (cmd == "graph-cycles" && argc == 3) {
    return cmd_graph_cycles(uint32_t(strtoul(argv[2], nullptr, 10)));
  }
  fprintf(stderr, "unknown command %s\n", cmd.c_str());
  return 2;
}
