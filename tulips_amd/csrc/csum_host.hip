// csum_host.hip — end-to-end path for host-resident segments
// (tulips_csum_ctx_* / tulips_csum_batch_host in include/tulips_csum.h).
//
// The reference's segments live in host memory delivered by src/transport
// (one mmap of nbuf x 2048 B for OFED RX, src/transport/ofed/Utils.cpp:241;
// a reused read buffer for npipe, include/tulips/transport/npipe/Device.h:103)
// and are checksummed per frame on the CPU. Here a batch is cut into chunks
// of <= chunk_bytes; each chunk goes host -> pinned staging -> HBM -> kernel
// -> results back, on NSLOTS pipeline slots with their own streams so that
// packing the next chunks on the CPU (a pool of up to MAX_PACK_THREADS
// threads owned by the context) overlaps the copies and kernels of the
// previous ones.
//
// When the caller's arena is already pinned (hipHostMalloc/hipHostRegister,
// as a registered NIC ring would be) and a chunk's segments lie in a compact
// span inside ONE page-locked allocation, the span is DMA'd straight from the
// caller's memory (no CPU copy); any other span is packed.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/tulips_csum.h"
#include "csum_common.h"
#include "csum_launch.h"
#include "zc_mailbox.h"

#include <chrono>

using namespace tulips_amd;

namespace {

// 16 MiB chunks on 3 slots: the first chunk's pack and the last chunk's
// kernel + D2H are the only unoverlapped steps
constexpr uint64_t DEFAULT_CHUNK = 16ull << 20;
constexpr uint32_t MAX_SEGS_PER_CHUNK = 1u << 20;
constexpr int NSLOTS = 3;
// Staging-copy threads: the CPUs this process may run on, at most 16 (a GPU's
// share of a host; 16 threads took pageable F1500 from 37 to 44 GiB/s over 8
// on the MI355X box, alternating builds).
constexpr int MAX_PACK_THREADS = 16;

} // namespace

namespace tulips_amd {
int
pack_threads()
{
  cpu_set_t set;
  CPU_ZERO(&set);
  int n = 0;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) {
    n = CPU_COUNT(&set);
  }
  if (n <= 0) {
    n = int(std::thread::hardware_concurrency());
  }
  return n < 1 ? 1 : (n > MAX_PACK_THREADS ? MAX_PACK_THREADS : n);
}
} // namespace tulips_amd

namespace {
using tulips_amd::pack_threads;

// Persistent workers for the staging copy (a thread per pack would cost
// tens of microseconds per chunk to create). run(f) calls f(0..size()-1)
// once each, part 0 on the calling thread, and returns when all are done.
class PackPool
{
public:
  explicit PackPool(int n) : n_(n < 1 ? 1 : n)
  {
    for (int t = 1; t < n_; ++t) {
      threads_.emplace_back([this, t] { worker(t); });
    }
  }
  int size() const { return n_; }
  ~PackPool()
  {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) {
      t.join();
    }
  }
  void run(const std::function<void(int)>& f)
  {
    {
      std::lock_guard<std::mutex> g(m_);
      work_ = &f;
      pending_ = n_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return pending_ == 0; });
    work_ = nullptr;
  }

private:
  void worker(int id)
  {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* f;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) {
          return;
        }
        seen = gen_;
        f = work_;
      }
      (*f)(id);
      {
        std::lock_guard<std::mutex> g(m_);
        if (--pending_ == 0) {
          done_.notify_one();
        }
      }
    }
  }
  const int n_;
  std::vector<std::thread> threads_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* work_ = nullptr;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
};

struct Slot
{
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  uint8_t* h_bytes = nullptr;
  uint64_t* h_offs = nullptr;
  uint16_t* h_lens = nullptr;
  uint16_t* h_seeds = nullptr;
  uint32_t* h_src = nullptr;
  uint32_t* h_dst = nullptr;
  uint16_t* h_out = nullptr;
  uint32_t* h_cnt = nullptr;
  uint32_t* h_fields = nullptr;
  uint8_t* d_bytes = nullptr;
  uint64_t* d_offs = nullptr;
  uint16_t* d_lens = nullptr;
  uint16_t* d_seeds = nullptr;
  uint32_t* d_src = nullptr;
  uint32_t* d_dst = nullptr;
  uint16_t* d_out = nullptr;
  uint32_t* d_cnt = nullptr;
  uint32_t* d_fields = nullptr;
  bool busy = false;
  uint32_t i0 = 0, i1 = 0;
};

int
status_of(hipError_t e)
{
  if (e == hipSuccess) {
    return TULIPS_STATUS_OK;
  }
  return e == hipErrorOutOfMemory ? TULIPS_STATUS_NO_MORE_RESOURCES
                                  : TULIPS_STATUS_HARDWARE_ERROR;
}

// The page-locked allocation holding `p`, as [lo, hi) (empty when `p` is not
// in page-locked host memory): a span may be DMA'd straight from the
// caller only when it lies inside one such allocation.
struct PinnedRange
{
  uintptr_t lo = 0, hi = 0;
  bool holds(uintptr_t a, uintptr_t b) const { return lo <= a && a <= b && b <= hi; }
};

PinnedRange
pinned_range(const void* p)
{
  PinnedRange r;
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess || attr.type != hipMemoryTypeHost) {
    (void)hipGetLastError();
    return r;
  }
  void* start = nullptr;
  size_t size = 0;
  if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                             reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(p))) !=
        hipSuccess ||
      hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE,
                             reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(p))) !=
        hipSuccess) {
    (void)hipGetLastError();
    return r;
  }
  r.lo = reinterpret_cast<uintptr_t>(start);
  r.hi = r.lo + size;
  return r;
}

// Low-latency receive validation (zc_mailbox.h), made on first use.
struct ZcState
{
  ZcMailbox* mb = nullptr;       // page-locked, host-coherent, GPU-mapped
  uint8_t* staging = nullptr;    // page-locked: bursts from pageable memory
  hipStream_t stream = nullptr;  // the server's stream (its own hardware queue)
  bool resident = false;         // resident server (else one launch per burst)
  bool launched = false;
  uint64_t seq = 0;
  uintptr_t mb_dev = 0, staging_dev = 0;  // their device addresses
  PinnedRange pin;               // last page-locked allocation seen
  uintptr_t pin_dev = 0;         // device address of pin.lo
  std::chrono::steady_clock::time_point last{};
};

} // namespace

struct tulips_csum_ctx
{
  explicit tulips_csum_ctx(int threads) : pool(threads) {}
  int device = 0;
  ZcState zc;
  bool zc_resident = false; // tulips_csum_ctx_set_lowlat
  uint64_t chunk = DEFAULT_CHUNK;
  Slot slots[NSLOTS];
  PackPool pool;
  // segmentation output (tulips_csum_segment_frames_host), grown on demand
  uint8_t* d_seg_out = nullptr;
  uint64_t seg_out_bytes = 0;
  uint16_t* d_seg_lens = nullptr;
  uint64_t seg_lens_n = 0;
  uint32_t* d_first = nullptr;
  uint32_t* h_first = nullptr;
};

namespace {

void
free_slot(Slot& s)
{
  if (s.stream) {
    (void)hipStreamSynchronize(s.stream);
  }
  (void)hipHostFree(s.h_bytes);
  (void)hipHostFree(s.h_offs);
  (void)hipHostFree(s.h_lens);
  (void)hipHostFree(s.h_seeds);
  (void)hipHostFree(s.h_src);
  (void)hipHostFree(s.h_dst);
  (void)hipHostFree(s.h_out);
  (void)hipHostFree(s.h_cnt);
  (void)hipHostFree(s.h_fields);
  (void)hipFree(s.d_bytes);
  (void)hipFree(s.d_offs);
  (void)hipFree(s.d_lens);
  (void)hipFree(s.d_seeds);
  (void)hipFree(s.d_src);
  (void)hipFree(s.d_dst);
  (void)hipFree(s.d_out);
  (void)hipFree(s.d_cnt);
  (void)hipFree(s.d_fields);
  if (s.done) {
    (void)hipEventDestroy(s.done);
  }
  if (s.stream) {
    (void)tulips_csum_release_stream(s.stream); // counter shards of the slot
    (void)hipStreamDestroy(s.stream);
  }
  s = Slot();
}

hipError_t
alloc_slot(Slot& s, uint64_t chunk)
{
  hipError_t e;
#define TCS_TRY(x)                                                             \
  if ((e = (x)) != hipSuccess) {                                               \
    return e;                                                                  \
  }
  const size_t m = MAX_SEGS_PER_CHUNK;
  TCS_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
  TCS_TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
  TCS_TRY(hipHostMalloc(reinterpret_cast<void**>(&s.h_bytes), chunk, 0));
  TCS_TRY(hipHostMalloc(reinterpret_cast<void**>(&s.h_offs), m * 8, 0));
  TCS_TRY(hipHostMalloc(reinterpret_cast<void**>(&s.h_lens), m * 2, 0));
  TCS_TRY(hipHostMalloc(reinterpret_cast<void**>(&s.h_seeds), m * 2, 0));
  TCS_TRY(hipHostMalloc(reinterpret_cast<void**>(&s.h_src), m * 4, 0));
  TCS_TRY(hipHostMalloc(reinterpret_cast<void**>(&s.h_dst), m * 4, 0));
  TCS_TRY(hipHostMalloc(reinterpret_cast<void**>(&s.h_out), m * 2, 0));
  TCS_TRY(hipHostMalloc(reinterpret_cast<void**>(&s.h_cnt), 16, 0));
  TCS_TRY(hipHostMalloc(reinterpret_cast<void**>(&s.h_fields), m * 4, 0));
  TCS_TRY(hipMalloc(reinterpret_cast<void**>(&s.d_bytes), chunk));
  TCS_TRY(hipMalloc(reinterpret_cast<void**>(&s.d_offs), m * 8));
  TCS_TRY(hipMalloc(reinterpret_cast<void**>(&s.d_lens), m * 2));
  TCS_TRY(hipMalloc(reinterpret_cast<void**>(&s.d_seeds), m * 2));
  TCS_TRY(hipMalloc(reinterpret_cast<void**>(&s.d_src), m * 4));
  TCS_TRY(hipMalloc(reinterpret_cast<void**>(&s.d_dst), m * 4));
  TCS_TRY(hipMalloc(reinterpret_cast<void**>(&s.d_out), m * 2));
  TCS_TRY(hipMalloc(reinterpret_cast<void**>(&s.d_cnt), 16));
  TCS_TRY(hipMalloc(reinterpret_cast<void**>(&s.d_fields), m * 4));
#undef TCS_TRY
  return hipSuccess;
}

// What a pipeline run computes: checksums (uint16 per segment) or frame
// flags (uint8 per frame, plus optional counters).
struct Job
{
  bool frames = false;
  bool generate = false;          // frames: write both checksum fields
  uint8_t* patch_base = nullptr;  // generate: the caller's frames
  const uint64_t* offsets = nullptr;
  const uint16_t* seeds = nullptr;
  const uint32_t* src = nullptr;
  const uint32_t* dst = nullptr;
  uint32_t mode = 0;
  uint8_t* out = nullptr; // host results, elem() bytes per entry (nullable
                          // for generate)
  uint32_t* counters = nullptr;
  size_t elem() const { return frames ? 1 : 2; }
};

// Collect the results of a finished slot into the caller's arrays.
hipError_t
retire(Slot& s, const Job& job)
{
  if (!s.busy) {
    return hipSuccess;
  }
  const hipError_t e = hipEventSynchronize(s.done);
  if (e == hipSuccess && job.generate) {
    // the generated fields into the caller's frames (Eth 14 + IPv4 10 and
    // Eth 14 + IPv4 20 + TCP 16), where the flags say they were written
    const uint8_t* fl = reinterpret_cast<const uint8_t*>(s.h_out);
    for (uint32_t k = s.i0; k < s.i1; ++k) {
      uint8_t* f = job.patch_base + job.offsets[k];
      const uint32_t v = s.h_fields[k - s.i0];
      if (fl[k - s.i0] & TULIPS_FRAME_IP_CSUM_OK) {
        f[24] = uint8_t(v);
        f[25] = uint8_t(v >> 8);
      }
      if (fl[k - s.i0] & TULIPS_FRAME_L4_CSUM_OK) {
        f[50] = uint8_t(v >> 16);
        f[51] = uint8_t(v >> 24);
      }
    }
  }
  if (e == hipSuccess && job.out) {
    memcpy(job.out + size_t(s.i0) * job.elem(), s.h_out,
           size_t(s.i1 - s.i0) * job.elem());
    if (job.counters) {
      for (int k = 0; k < 4; ++k) {
        job.counters[k] += s.h_cnt[k];
      }
    }
  }
  s.busy = false;
  return e;
}

// Copy segments [i0, i1) into the slot's pinned staging, back to back,
// split over the context's pack threads by segment count.
void
pack(PackPool& pool, Slot& s, const uint8_t* base, const uint64_t* offsets,
     const uint16_t* lengths, uint32_t i0, uint32_t i1)
{
  auto copy_range = [&](uint32_t a, uint32_t b) {
    for (uint32_t j = a; j < b; ++j) {
      memcpy(s.h_bytes + s.h_offs[j - i0], base + offsets[j], lengths[j]);
    }
  };
  const uint64_t total = s.h_offs[i1 - 1 - i0] + lengths[i1 - 1];
  if (total < (1ull << 20) || i1 - i0 < 64) {
    copy_range(i0, i1);
    return;
  }
  const uint32_t cnt = i1 - i0;
  const uint64_t parts = uint64_t(pool.size());
  pool.run([&](int t) {
    copy_range(i0 + uint32_t(uint64_t(cnt) * uint64_t(t) / parts),
               i0 + uint32_t(uint64_t(cnt) * uint64_t(t + 1) / parts));
  });
}

// Stop the context's validation server and free its mailbox.
void
zc_release(ZcState& z)
{
  if (z.mb && z.launched) {
    __atomic_store_n(&z.mb->stop, 1ull, __ATOMIC_RELEASE);
    (void)hipStreamSynchronize(z.stream);
  }
  if (z.mb) {
    (void)hipHostFree(z.mb);
  }
  if (z.staging) {
    (void)hipHostFree(z.staging);
  }
  if (z.stream) {
    (void)hipStreamDestroy(z.stream);
  }
  z = ZcState();
}

} // namespace

namespace tulips_amd {
// tulips_csum_ctx_create with an explicit staging-copy thread count (the
// multi-device context gives each device its share of the CPUs).
int
ctx_create(int device, uint64_t chunk_bytes, int threads, tulips_csum_ctx** ctx)
{
  if (!ctx) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  *ctx = nullptr;
  if (chunk_bytes == 0) {
    chunk_bytes = DEFAULT_CHUNK;
  }
  if (chunk_bytes < TULIPS_CSUM_MAX_SEGMENT + 16) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || device < 0 || device >= ndev) {
    return e != hipSuccess ? status_of(e) : TULIPS_STATUS_INVALID_ARGUMENT;
  }
  int prev = 0;
  (void)hipGetDevice(&prev);
  if ((e = hipSetDevice(device)) != hipSuccess) {
    return status_of(e);
  }
  tulips_csum_ctx* c = nullptr;
  try {
    c = new tulips_csum_ctx(threads); // starts the pack threads
  } catch (...) {
    c = nullptr;
  }
  if (!c) {
    (void)hipSetDevice(prev);
    return TULIPS_STATUS_NO_MORE_RESOURCES;
  }
  c->device = device;
  c->chunk = chunk_bytes;
  for (auto& s : c->slots) {
    if ((e = alloc_slot(s, chunk_bytes)) != hipSuccess) {
      for (auto& t : c->slots) {
        free_slot(t);
      }
      delete c;
      (void)hipSetDevice(prev);
      return status_of(e);
    }
  }
  (void)hipSetDevice(prev);
  *ctx = c;
  return TULIPS_STATUS_OK;
}

// Toeplitz hashes (tulips_rss_toeplitz_batch) of host tuples on the
// context's device, through slot 0's pinned staging, up to
// MAX_SEGS_PER_CHUNK tuples per round trip. Blocks until `out` is written.
int
ctx_rss_hash(tulips_csum_ctx* ctx, const uint32_t* saddr, const uint32_t* daddr,
             const uint16_t* sport, const uint16_t* dport, uint32_t n, const uint8_t* key,
             size_t key_len, uint32_t init, uint32_t* out)
{
  int prev = 0;
  (void)hipGetDevice(&prev);
  hipError_t e = hipSetDevice(ctx->device);
  Slot& s = ctx->slots[0];
  int rc = TULIPS_STATUS_OK;
  for (uint32_t i = 0; i < n && e == hipSuccess && rc == TULIPS_STATUS_OK;
       i += MAX_SEGS_PER_CHUNK) {
    const uint32_t c = std::min<uint32_t>(MAX_SEGS_PER_CHUNK, n - i);
    // the slot's previous work is retired: its pinned buffers are free
    if ((e = hipStreamSynchronize(s.stream)) != hipSuccess) {
      break;
    }
    memcpy(s.h_src, saddr + i, size_t(c) * 4);
    memcpy(s.h_dst, daddr + i, size_t(c) * 4);
    memcpy(s.h_seeds, sport + i, size_t(c) * 2);
    memcpy(s.h_lens, dport + i, size_t(c) * 2);
    if ((e = hipMemcpyAsync(s.d_src, s.h_src, size_t(c) * 4, hipMemcpyHostToDevice,
                            s.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(s.d_dst, s.h_dst, size_t(c) * 4, hipMemcpyHostToDevice,
                            s.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(s.d_seeds, s.h_seeds, size_t(c) * 2, hipMemcpyHostToDevice,
                            s.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(s.d_lens, s.h_lens, size_t(c) * 2, hipMemcpyHostToDevice,
                            s.stream)) != hipSuccess) {
      break;
    }
    rc = tulips_rss_toeplitz_batch(s.d_src, s.d_dst, s.d_seeds, s.d_lens, c, key, key_len,
                                   init, s.d_fields, s.stream);
    if (rc == TULIPS_STATUS_OK &&
        ((e = hipMemcpyAsync(s.h_fields, s.d_fields, size_t(c) * 4, hipMemcpyDeviceToHost,
                             s.stream)) != hipSuccess ||
         (e = hipStreamSynchronize(s.stream)) != hipSuccess)) {
      break;
    }
    if (rc == TULIPS_STATUS_OK) {
      memcpy(out + i, s.h_fields, size_t(c) * 4);
    }
  }
  (void)hipSetDevice(prev);
  return e != hipSuccess ? status_of(e) : rc;
}

} // namespace tulips_amd

extern "C" {

int
tulips_csum_ctx_create(int device, uint64_t chunk_bytes, tulips_csum_ctx** ctx)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  return tulips_amd::ctx_create(device, chunk_bytes, pack_threads(), ctx);
}

int
tulips_csum_ctx_destroy(tulips_csum_ctx* ctx)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (!ctx) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(ctx->device);
  zc_release(ctx->zc);
  for (auto& s : ctx->slots) {
    free_slot(s);
  }
  (void)hipFree(ctx->d_seg_out);
  (void)hipFree(ctx->d_seg_lens);
  (void)hipFree(ctx->d_first);
  (void)hipHostFree(ctx->h_first);
  (void)hipSetDevice(prev);
  delete ctx;
  return TULIPS_STATUS_OK;
}

} // extern "C"

namespace {

int
run(tulips_csum_ctx* ctx, const uint8_t* base, const uint64_t* offsets,
    const uint16_t* lengths, uint32_t n, const Job& job)
{
  int prev = 0;
  (void)hipGetDevice(&prev);
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) {
    return status_of(e);
  }
  const PinnedRange pinned = pinned_range(base);
  int slot = 0;
  uint32_t i = 0;
  while (i < n && e == hipSuccess) {
    Slot& s = ctx->slots[slot];
    if ((e = retire(s, job)) != hipSuccess) {
      break;
    }
    // Cut the chunk: segments [i, j) with at most ctx->chunk bytes.
    uint64_t bytes = 0, lo = UINT64_MAX, hi = 0;
    uint32_t j = i;
    bool in_order = true; // caller's offsets ascending, segments disjoint
    while (j < n && j - i < MAX_SEGS_PER_CHUNK &&
           bytes + lengths[j] <= ctx->chunk) {
      s.h_offs[j - i] = bytes;
      bytes += lengths[j];
      in_order = in_order && (j == i || offsets[j] >= offsets[j - 1] + lengths[j - 1]);
      lo = std::min<uint64_t>(lo, offsets[j]);
      hi = std::max<uint64_t>(hi, offsets[j] + lengths[j]);
      ++j;
    }
    const uint32_t cnt = j - i;
    const uint8_t* dbase = s.d_bytes;
    const uint8_t* hsrc;
    uint64_t hbytes;
    // packed staging is in order by construction (tulips_csum_batch_arena)
    bool arena_ok = true;
    const uintptr_t b0 = reinterpret_cast<uintptr_t>(base);
    if (hi > lo && hi - lo <= ctx->chunk && hi - lo <= 2 * bytes &&
        pinned.holds(b0 + lo, b0 + hi)) {
      arena_ok = in_order;
      // Direct DMA of the caller's span; offsets rebased onto it.
      for (uint32_t k = 0; k < cnt; ++k) {
        s.h_offs[k] = offsets[i + k] - lo;
      }
      hsrc = base + lo;
      hbytes = hi - lo;
    } else {
      pack(ctx->pool, s, base, offsets, lengths, i, j);
      hsrc = s.h_bytes;
      hbytes = bytes;
    }
    memcpy(s.h_lens, lengths + i, size_t(cnt) * 2);
    if (job.seeds) {
      memcpy(s.h_seeds, job.seeds + i, size_t(cnt) * 2);
    }
    if (job.src) {
      memcpy(s.h_src, job.src + i, size_t(cnt) * 4);
      memcpy(s.h_dst, job.dst + i, size_t(cnt) * 4);
    }
    hipStream_t st = s.stream;
#define TCS_Q(x)                                                               \
  if (e == hipSuccess) {                                                       \
    e = (x);                                                                   \
  }
    TCS_Q(hipMemcpyAsync(s.d_bytes, hsrc, hbytes, hipMemcpyHostToDevice, st));
    TCS_Q(hipMemcpyAsync(s.d_offs, s.h_offs, size_t(cnt) * 8,
                         hipMemcpyHostToDevice, st));
    TCS_Q(hipMemcpyAsync(s.d_lens, s.h_lens, size_t(cnt) * 2,
                         hipMemcpyHostToDevice, st));
    if (job.seeds) {
      TCS_Q(hipMemcpyAsync(s.d_seeds, s.h_seeds, size_t(cnt) * 2,
                           hipMemcpyHostToDevice, st));
    }
    if (job.src) {
      TCS_Q(hipMemcpyAsync(s.d_src, s.h_src, size_t(cnt) * 4,
                           hipMemcpyHostToDevice, st));
      TCS_Q(hipMemcpyAsync(s.d_dst, s.h_dst, size_t(cnt) * 4,
                           hipMemcpyHostToDevice, st));
    }
    if (job.generate) {
      TCS_Q(launch_generate(const_cast<uint8_t*>(dbase), s.d_offs, s.d_lens, cnt,
                            reinterpret_cast<uint8_t*>(s.d_out), st, FrameLaunch{},
                            s.d_fields));
      TCS_Q(hipMemcpyAsync(s.h_fields, s.d_fields, size_t(cnt) * 4,
                           hipMemcpyDeviceToHost, st));
    } else if (job.frames) {
      TCS_Q(launch_frames(dbase, s.d_offs, s.d_lens, cnt,
                          reinterpret_cast<uint8_t*>(s.d_out),
                          job.counters ? s.d_cnt : nullptr, st));
      if (job.counters) {
        TCS_Q(hipMemcpyAsync(s.h_cnt, s.d_cnt, 16, hipMemcpyDeviceToHost, st));
      }
    } else {
      LaunchArgs a{};
      a.seeds = job.seeds ? s.d_seeds : nullptr;
      a.src = job.src ? s.d_src : nullptr;
      a.dst = job.src ? s.d_dst : nullptr;
      a.out = s.d_out;
      a.bad = nullptr;
      a.n = cnt;
      a.mode = job.mode;
      a.nontemporal = true;
      a.max_blocks = 0;
      if (arena_ok) {
        // segments in order in the staged bytes: work cut by bytes
        a.kind = TULIPS_CSUM_KIND_SPAN;
        a.unroll = tulips_amd::SPAN_DEFAULT_UNROLL;
        a.group = 0;
        TCS_Q(launch_span(dbase, hbytes, s.d_offs, s.d_lens, a, st));
      } else {
        // the variable-length default geometry (csum_capi.hip default_tuning)
        a.kind = TULIPS_CSUM_KIND_PACKED;
        a.group = 8;
        a.unroll = 4;
        a.spw = 2;
        a.block = 256;
        TCS_Q(launch_var(dbase, s.d_offs, s.d_lens, a, st));
      }
    }
    TCS_Q(hipMemcpyAsync(s.h_out, s.d_out, size_t(cnt) * job.elem(),
                         hipMemcpyDeviceToHost, st));
    TCS_Q(hipEventRecord(s.done, st));
#undef TCS_Q
    s.busy = e == hipSuccess;
    s.i0 = i;
    s.i1 = j;
    i = j;
    slot = (slot + 1) % NSLOTS;
  }
  for (auto& s : ctx->slots) {
    const hipError_t r = retire(s, job);
    if (e == hipSuccess) {
      e = r;
    }
  }
  (void)hipSetDevice(prev);
  return status_of(e);
}

} // namespace

extern "C" {

int
tulips_csum_host_alloc(size_t bytes, void** ptr)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (!ptr || bytes == 0) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  *ptr = nullptr;
  return status_of(hipHostMalloc(ptr, bytes, 0));
}

int
tulips_csum_host_free(void* ptr)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  return ptr ? status_of(hipHostFree(ptr)) : TULIPS_STATUS_OK;
}

int
tulips_csum_batch_host(tulips_csum_ctx* ctx, const uint8_t* base,
                       const uint64_t* offsets, const uint16_t* lengths,
                       const uint16_t* seeds, const uint32_t* src,
                       const uint32_t* dst, uint16_t* out, uint32_t n,
                       uint32_t mode)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (!ctx) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (n == 0) {
    return TULIPS_STATUS_OK;
  }
  const uint32_t m = mode & TULIPS_CSUM_MODE_MASK;
  if (!base || !offsets || !lengths || !out ||
      (mode & ~(TULIPS_CSUM_MODE_MASK | TULIPS_CSUM_COMPLEMENT)) ||
      m > TULIPS_CSUM_TCP || (m == TULIPS_CSUM_TCP && (!src || !dst))) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  Job job;
  job.mode = mode;
  job.seeds = m == TULIPS_CSUM_TCP ? nullptr : seeds;
  job.src = m == TULIPS_CSUM_TCP ? src : nullptr;
  job.dst = m == TULIPS_CSUM_TCP ? dst : nullptr;
  job.out = reinterpret_cast<uint8_t*>(out);
  return run(ctx, base, offsets, lengths, n, job);
}

int
tulips_csum_validate_frames_host(tulips_csum_ctx* ctx, const uint8_t* base,
                                 const uint64_t* offsets,
                                 const uint16_t* lengths, uint32_t n,
                                 uint8_t* flags, uint32_t* counters)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (!ctx) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (counters) {
    memset(counters, 0, 4 * sizeof(uint32_t));
  }
  if (n == 0) {
    return TULIPS_STATUS_OK;
  }
  if (!base || !offsets || !lengths || !flags) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  Job job;
  job.frames = true;
  job.out = flags;
  job.counters = counters;
  return run(ctx, base, offsets, lengths, n, job);
}

} // extern "C"

namespace {

hipError_t
zc_setup(tulips_csum_ctx* ctx)
{
  ZcState& z = ctx->zc;
  if (z.mb) {
    return hipSuccess;
  }
  hipError_t e;
  void* mb = nullptr;
  void* st = nullptr;
  if ((e = hipHostMalloc(&mb, sizeof(ZcMailbox), hipHostMallocCoherent | hipHostMallocMapped)) !=
      hipSuccess) {
    return e;
  }
  memset(mb, 0, sizeof(ZcMailbox));
  z.mb = static_cast<ZcMailbox*>(mb);
  if ((e = hipHostMalloc(&st, ZC_STAGING, hipHostMallocMapped)) != hipSuccess) {
    zc_release(z);
    return e;
  }
  z.staging = static_cast<uint8_t*>(st);
  void* d = nullptr;
  if ((e = hipHostGetDevicePointer(&d, mb, 0)) != hipSuccess) {
    zc_release(z);
    return e;
  }
  z.mb_dev = reinterpret_cast<uintptr_t>(d);
  if ((e = hipHostGetDevicePointer(&d, st, 0)) != hipSuccess) {
    zc_release(z);
    return e;
  }
  z.staging_dev = reinterpret_cast<uintptr_t>(d);
  // a CU-masked stream gets a hardware queue of its own (HIP never pools
  // it with other streams), so the resident server cannot hold up work
  // queued on any other stream of the process
  int cus = 0;
  if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device)) !=
      hipSuccess) {
    zc_release(z);
    return e;
  }
  std::vector<uint32_t> mask(size_t((cus + 31) / 32), 0xffffffffu);
  const char* mode = getenv("TULIPS_ZC_MODE");
  z.resident = ctx->zc_resident || (mode && strcmp(mode, "resident") == 0);
  const char* plain = getenv("TULIPS_ZC_PLAIN_STREAM");
  if ((e = (!z.resident || (plain && plain[0] == '1'))
             ? hipStreamCreateWithFlags(&z.stream, hipStreamNonBlocking)
             : hipExtStreamCreateWithCUMask(&z.stream, uint32_t(mask.size()), mask.data())) !=
      hipSuccess) {
    z.stream = nullptr;
    zc_release(z);
    return e;
  }
  return hipSuccess;
}

// One burst through the resident server; returns NOT_APPLICABLE when the
// burst must take the staged path (too many frames, or pageable frames
// that do not fit the zc staging).
constexpr int ZC_NOT_APPLICABLE = -1;

int
zc_validate(tulips_csum_ctx* ctx, const uint8_t* base, const uint64_t* offsets,
            const uint16_t* lengths, uint32_t n, uint8_t* flags, uint32_t* counters)
{
  if (n > ZC_MAX_FRAMES) {
    return ZC_NOT_APPLICABLE;
  }
  uint64_t lo = UINT64_MAX, hi = 0, bytes = 0;
  for (uint32_t k = 0; k < n; ++k) {
    lo = std::min<uint64_t>(lo, offsets[k]);
    hi = std::max<uint64_t>(hi, offsets[k] + lengths[k]);
    bytes += lengths[k];
  }
  hipError_t e = zc_setup(ctx);
  if (e != hipSuccess) {
    return status_of(e);
  }
  ZcState& z = ctx->zc;
  ZcMailbox* mb = z.mb;
  const uintptr_t b0 = reinterpret_cast<uintptr_t>(base);
  if (hi > lo) {
    // looked up on every call: the caller may have freed the allocation
    // cached here and the range been reused by another (pageable or
    // page-locked) allocation; only an identical [lo, hi) keeps the cached
    // device address
    const PinnedRange now_pin = pinned_range(base + lo);
    if (now_pin.lo != z.pin.lo || now_pin.hi != z.pin.hi || z.pin_dev == 0) {
      z.pin = now_pin;
      z.pin_dev = 0;
      void* d = nullptr;
      if (z.pin.hi > z.pin.lo &&
          hipHostGetDevicePointer(&d, reinterpret_cast<void*>(z.pin.lo), 0) == hipSuccess) {
        z.pin_dev = reinterpret_cast<uintptr_t>(d);
      } else {
        (void)hipGetLastError();
        z.pin = PinnedRange();
      }
    }
  }
  uint64_t dbase;
  bool staged = false;
  if (hi <= lo || z.pin.holds(b0 + lo, b0 + hi)) {
    // frames read in place over PCIe
    dbase = z.pin_dev + (b0 - z.pin.lo);
  } else if (bytes <= ZC_STAGING) {
    uint64_t at = 0;
    for (uint32_t k = 0; k < n; ++k) {
      memcpy(z.staging + at, base + offsets[k], lengths[k]);
      mb->offs[k] = at;
      at += lengths[k];
    }
    dbase = z.staging_dev;
    staged = true;
    lo = 0;
    hi = at;
  } else {
    return ZC_NOT_APPLICABLE;
  }
  // descriptors as 32-bit offsets from the hull's start
  const uint64_t l0 = hi > lo ? lo : 0;
  if ((hi > lo ? hi - lo : 0) >= (1ull << 32)) {
    return ZC_NOT_APPLICABLE;
  }
  const uint64_t gbase = dbase + l0;
  if ((z.seq + 1) % 65536 == 0) {
    ++z.seq; // tags are 16-bit and never 0
  }
  const uint64_t seq = ++z.seq;
  const uint32_t tag = uint32_t(seq & 0xffffu);
  // the workgroups that answer this request (frames.hip launch_zc_server)
  const uint32_t nwg = z.resident ? ZC_RES_WG
                       : n <= ZC_ARG_FRAMES ? 1u
                                            : std::min(ZC_MAX_WG, (n + 63) / 64);
  ZcArgs args{};
  const bool inl = z.resident ? n <= ZC_REQ_FRAMES : n <= ZC_ARG_FRAMES;
  auto off_of = [&](uint32_t k) { return (staged ? mb->offs[k] : offsets[k]) - l0; };
  if (!inl) {
    for (uint32_t k = 0; k < n; ++k) {
      mb->offs[k] = off_of(k);
    }
    memcpy(mb->lens, lengths, size_t(n) * 2);
  }
  if (z.resident) {
    // tagged doorbell words, the first one last (zc_mailbox.h)
    if (inl) {
      for (uint32_t k = 0; k < n; ++k) {
        __atomic_store_n(&mb->req[2 + k], zc_word(tag, (off_of(k) << 16) | lengths[k]),
                         __ATOMIC_RELAXED);
      }
    }
    __atomic_store_n(&mb->req[1], zc_word(tag, gbase), __ATOMIC_RELAXED);
    __atomic_store_n(&mb->req[0], zc_word(tag, n), __ATOMIC_RELEASE);
  } else {
    // done[] of the workgroups about to answer: cleared, so a word left by
    // a request 65,535 tags ago (a larger burst served by more workgroups)
    // can never read as this request's completion; every earlier launch has
    // published all of its words (the host waited for them)
    for (uint32_t w = 0; w < nwg; ++w) {
      __atomic_store_n(&mb->done[w], uint64_t(0), __ATOMIC_RELAXED);
    }
    args.base = gbase;
    args.seq = tag;
    args.n = n;
    if (inl) {
      args.inline_n = n;
      for (uint32_t k = 0; k < n; ++k) {
        args.off[k] = uint32_t(off_of(k));
        args.len[k] = lengths[k];
      }
    }
    __atomic_thread_fence(__ATOMIC_RELEASE);
  }
  // (re)start the server: first use, or it may have timed out since the
  // last burst (it idles out after 100 ms; checked from 50 ms on)
  const auto now = std::chrono::steady_clock::now();
  if (!z.resident) {
    // one workgroup per burst: serves request `seq` and exits
    if ((e = launch_zc_server(reinterpret_cast<ZcMailbox*>(z.mb_dev), &args, z.stream)) !=
        hipSuccess) {
      return status_of(e);
    }
    z.launched = true;
  }
  auto relaunch = [&]() -> hipError_t {
    const hipError_t q = z.launched ? hipStreamQuery(z.stream) : hipSuccess;
    if (!z.resident) {
      return q == hipErrorNotReady ? hipSuccess : q; // an error ends the wait
    }
    if (q == hipErrorNotReady) {
      return hipSuccess; // still serving
    }
    if (q != hipSuccess) {
      return q;
    }
    const hipError_t r =
      launch_zc_server(reinterpret_cast<ZcMailbox*>(z.mb_dev), nullptr, z.stream);
    z.launched = r == hipSuccess;
    return r;
  };
  if (z.resident && (!z.launched || now - z.last > std::chrono::milliseconds(50))) {
    if ((e = relaunch()) != hipSuccess) {
      return status_of(e);
    }
  }
  for (uint64_t k = 1;; ++k) {
    uint32_t fin = 0;
    for (uint32_t w = 0; w < nwg; ++w) {
      fin += __atomic_load_n(&mb->done[w], __ATOMIC_ACQUIRE) == tag ? 1u : 0u;
    }
    if (fin == nwg) {
      break;
    }
    __builtin_ia32_pause();
    if ((k & 4095) == 0) {
      // the server may have exited between our check and the doorbell
      if ((e = relaunch()) != hipSuccess) {
        return status_of(e);
      }
      if (std::chrono::steady_clock::now() - now > std::chrono::seconds(2)) {
        fprintf(stderr,
                "tulips_csum_validate_frames_zc: no answer in 2 s (seq %llu done %llu "
                "seen %llu beat %llu stage %llu launched %d query %d base %llx mb %p/%llx "
                "pin %llx-%llx dev %llx b0 %llx n %u)\n",
                (unsigned long long)tag, (unsigned long long)mb->done[0],
                (unsigned long long)mb->seen, (unsigned long long)mb->beat,
                (unsigned long long)0, int(z.launched),
                int(hipStreamQuery(z.stream)), (unsigned long long)gbase, (void*)mb,
                (unsigned long long)z.mb_dev, (unsigned long long)z.pin.lo,
                (unsigned long long)z.pin.hi, (unsigned long long)z.pin_dev,
                (unsigned long long)b0, n);
        return TULIPS_STATUS_HARDWARE_ERROR;
      }
    }
  }
  z.last = std::chrono::steady_clock::now();
  memcpy(flags, mb->flags, n);
  if (counters) {
    for (int k = 0; k < 4; ++k) {
      counters[k] = 0;
      for (uint32_t w = 0; w < nwg; ++w) {
        counters[k] += mb->counters[w][k];
      }
    }
  }
  return TULIPS_STATUS_OK;
}

} // namespace

extern "C" int
tulips_csum_ctx_set_lowlat(tulips_csum_ctx* ctx, int resident)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (!ctx || (resident != 0 && resident != 1)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (ctx->zc.mb && ctx->zc.resident != (resident != 0)) {
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(ctx->device);
    zc_release(ctx->zc); // made again, in the new form, by the next call
    (void)hipSetDevice(prev);
  }
  ctx->zc_resident = resident != 0;
  return TULIPS_STATUS_OK;
}

extern "C" int
tulips_csum_validate_frames_zc(tulips_csum_ctx* ctx, const uint8_t* base,
                               const uint64_t* offsets, const uint16_t* lengths, uint32_t n,
                               uint8_t* flags, uint32_t* counters)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (!ctx) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (counters) {
    memset(counters, 0, 4 * sizeof(uint32_t));
  }
  if (n == 0) {
    return TULIPS_STATUS_OK;
  }
  if (!base || !offsets || !lengths || !flags) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  int prev = 0;
  (void)hipGetDevice(&prev);
  const hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) {
    return status_of(e);
  }
  int rc = zc_validate(ctx, base, offsets, lengths, n, flags, counters);
  (void)hipSetDevice(prev);
  if (rc == ZC_NOT_APPLICABLE) {
    rc = tulips_csum_validate_frames_host(ctx, base, offsets, lengths, n, flags, counters);
  }
  return rc;
}

namespace {

// grow *p to at least `bytes` (device memory of the ctx's device, current)
hipError_t
grow(void** p, uint64_t* have, uint64_t bytes)
{
  if (*have >= bytes) {
    return hipSuccess;
  }
  (void)hipFree(*p);
  *p = nullptr;
  *have = 0;
  const hipError_t e = hipMalloc(p, bytes);
  if (e == hipSuccess) {
    *have = bytes;
  }
  return e;
}

int
segment_host(tulips_csum_ctx* ctx, const uint8_t* in_base, const uint64_t* in_offsets,
             const uint16_t* in_lengths, uint32_t n, uint32_t mss, uint8_t* out_base,
             uint64_t out_stride, uint32_t out_capacity, uint16_t* out_lengths,
             uint32_t* out_first)
{
  Slot& s = ctx->slots[0];
  hipStream_t st = s.stream;
  hipError_t e = hipSuccess;
  if (!ctx->d_first) {
    if ((e = hipMalloc(reinterpret_cast<void**>(&ctx->d_first),
                       sizeof(uint32_t) * (MAX_SEGS_PER_CHUNK + 1))) != hipSuccess ||
        (e = hipHostMalloc(reinterpret_cast<void**>(&ctx->h_first),
                           sizeof(uint32_t) * (MAX_SEGS_PER_CHUNK + 1), 0)) != hipSuccess) {
      return status_of(e);
    }
  }
  uint64_t produced = 0; // segments of the frames before this chunk
  uint32_t i = 0;
  while (i < n) {
    // frames [i, j) that fit one staging chunk
    uint64_t bytes = 0;
    uint32_t j = i;
    while (j < n && j - i < MAX_SEGS_PER_CHUNK && bytes + in_lengths[j] <= ctx->chunk) {
      s.h_offs[j - i] = bytes;
      bytes += in_lengths[j];
      ++j;
    }
    const uint32_t cnt = j - i;
    // the plan from the headers, on this thread (the reference's transport
    // decides the TSO split on the host too): the device runs the segment
    // kernel alone, and the counts need no read-back
    int rc = tulips_csum_segment_plan_host(in_base, in_offsets + i, in_lengths + i, cnt, mss,
                                           ctx->h_first);
    if (rc != TULIPS_STATUS_OK) {
      return rc;
    }
    const uint32_t made = ctx->h_first[cnt];
    const uint32_t room = produced >= out_capacity
                            ? 0u
                            : uint32_t(std::min<uint64_t>(out_capacity - produced, made));
    for (uint32_t k = 0; k < cnt; ++k) {
      out_first[i + k] = uint32_t(produced + ctx->h_first[k]);
    }
    if (room) {
      pack(ctx->pool, s, in_base, in_offsets, in_lengths, i, j);
      memcpy(s.h_lens, in_lengths + i, size_t(cnt) * 2);
      uint64_t have_lens = ctx->seg_lens_n * 2;
      if ((e = grow(reinterpret_cast<void**>(&ctx->d_seg_out), &ctx->seg_out_bytes,
                    uint64_t(room) * out_stride)) != hipSuccess ||
          (e = grow(reinterpret_cast<void**>(&ctx->d_seg_lens), &have_lens,
                    uint64_t(room) * 2)) != hipSuccess) {
        return status_of(e);
      }
      ctx->seg_lens_n = have_lens / 2;
      if ((e = hipMemcpyAsync(s.d_bytes, s.h_bytes, bytes, hipMemcpyHostToDevice, st)) !=
            hipSuccess ||
          (e = hipMemcpyAsync(s.d_offs, s.h_offs, size_t(cnt) * 8, hipMemcpyHostToDevice,
                              st)) != hipSuccess ||
          (e = hipMemcpyAsync(s.d_lens, s.h_lens, size_t(cnt) * 2, hipMemcpyHostToDevice,
                              st)) != hipSuccess ||
          (e = hipMemcpyAsync(ctx->d_first, ctx->h_first, sizeof(uint32_t) * (cnt + 1),
                              hipMemcpyHostToDevice, st)) != hipSuccess) {
        return status_of(e);
      }
      rc = tulips_csum_segment_frames_planned(s.d_bytes, s.d_offs, s.d_lens, cnt, mss,
                                              ctx->d_first, ctx->d_seg_out, out_stride, room,
                                              ctx->d_seg_lens, st);
      if (rc != TULIPS_STATUS_OK) {
        (void)hipStreamSynchronize(st);
        return rc;
      }
      if ((e = hipMemcpyAsync(out_base + produced * out_stride, ctx->d_seg_out,
                              uint64_t(room) * out_stride, hipMemcpyDeviceToHost, st)) !=
            hipSuccess ||
          (e = hipMemcpyAsync(out_lengths + produced, ctx->d_seg_lens, uint64_t(room) * 2,
                              hipMemcpyDeviceToHost, st)) != hipSuccess ||
          (e = hipStreamSynchronize(st)) != hipSuccess) {
        return status_of(e);
      }
    }
    produced += made;
    i = j;
  }
  out_first[n] = uint32_t(produced);
  return TULIPS_STATUS_OK;
}

} // namespace

extern "C" {

int
tulips_csum_generate_frames_host(tulips_csum_ctx* ctx, uint8_t* base,
                                 const uint64_t* offsets, const uint16_t* lengths,
                                 uint32_t n, uint8_t* flags)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (!ctx) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (n == 0) {
    return TULIPS_STATUS_OK;
  }
  if (!base || !offsets || !lengths) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  Job job;
  job.frames = true;
  job.generate = true;
  job.patch_base = base;
  job.offsets = offsets;
  job.out = flags;
  return run(ctx, base, offsets, lengths, n, job);
}

int
tulips_csum_segment_frames_host(tulips_csum_ctx* ctx, const uint8_t* in_base,
                                const uint64_t* in_offsets,
                                const uint16_t* in_lengths, uint32_t n,
                                uint32_t mss, uint8_t* out_base,
                                uint64_t out_stride, uint32_t out_capacity,
                                uint16_t* out_lengths, uint32_t* out_first)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (!ctx || !out_first || mss == 0 || mss > 0xffffu) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (n == 0) {
    out_first[0] = 0;
    return TULIPS_STATUS_OK;
  }
  if (!in_base || !in_offsets || !in_lengths ||
      (out_capacity && (!out_base || !out_lengths || out_stride < 16 ||
                        (out_stride & 15)))) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  int prev = 0;
  (void)hipGetDevice(&prev);
  const hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) {
    return status_of(e);
  }
  const int rc = segment_host(ctx, in_base, in_offsets, in_lengths, n, mss, out_base,
                              out_stride, out_capacity, out_lengths, out_first);
  (void)hipSetDevice(prev);
  return rc;
}

} // extern "C"
