// csum_multi.hip — one process, several GPUs: the multi-device host context
// (tulips_csum_mctx_* in include/tulips_csum.h).
//
// Segments are independent, so a host batch splits into contiguous shards
// with no exchange between devices. The split is balanced by BYTES, not by
// segment count (a prefix sum of the lengths, tulips_csum_shard_plan): a
// Zipf batch cut by count would hand one device most of the long segments.
// Each shard runs on its device's own host context (pinned staging, streams,
// H2D -> kernel -> D2H pipeline, csum_host.hip) from a persistent worker
// thread per device, so the devices' PCIe links and kernels all run at once;
// results land in the caller's array in segment order. The reference's
// analogue is NIC multi-queue flow spreading
// (src/transport/ena/RedirectionTable.cpp:74-98).
//
// Device-resident batches (tulips_csum_mctx_batch_{fixed,arena}_device,
// SURVEY.md §8e "data starts on GPU 0"): the batch lives in the HBM of the
// caller's stream's device. It is cut into contiguous pieces (byte-balanced;
// for an arena the cut is found on the device by a binary search of the
// offsets), a run of pieces per listed device. A peer pulls each piece over
// xGMI (hipMemcpyPeerAsync on its own copy stream: the peer's DMA engines
// read the source HBM directly), its compute stream checksums piece p while
// piece p + 1 is in flight, and the piece's results go back to the source
// device's `out` in segment order. The first listed entry on the source
// device computes its pieces in place. Everything is stream-ordered after
// the work already queued on the caller's stream, and that stream waits for
// every result before its later work.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/tulips_csum.h"
#include "csum_launch.h"
#include "rss_route.h"

namespace tulips_amd {
int pack_threads();
int ctx_create(int device, uint64_t chunk_bytes, int threads, tulips_csum_ctx** ctx);
int ctx_rss_hash(tulips_csum_ctx* ctx, const uint32_t* saddr, const uint32_t* daddr,
                 const uint16_t* sport, const uint16_t* dport, uint32_t n, const uint8_t* key,
                 size_t key_len, uint32_t init, uint32_t* out);
}

namespace {

// One persistent thread per device; run() hands every worker its job and
// waits for all of them.
class Workers
{
public:
  explicit Workers(int n)
  {
    for (int k = 0; k < n; ++k) {
      threads_.emplace_back([this, k] { loop(k); });
    }
  }
  ~Workers()
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
      job_ = &f;
      pending_ = int(threads_.size());
      ++gen_;
    }
    cv_.notify_all();
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return pending_ == 0; });
    job_ = nullptr;
  }

private:
  void loop(int k)
  {
    // the library's own thread: every HIP call it makes is the library's
    // (allocations, copies, waits on the context's streams)
    hipStreamCaptureMode relaxed = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&relaxed);
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
        f = job_;
      }
      (*f)(k);
      {
        std::lock_guard<std::mutex> g(m_);
        if (--pending_ == 0) {
          done_.notify_one();
        }
      }
    }
  }
  std::vector<std::thread> threads_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* job_ = nullptr;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
};

} // namespace

namespace {

// Per listed device: what a device-resident call needs on that device
// (made on first use, grown on demand).
struct DevSlot
{
  int device = 0;
  hipStream_t copy = nullptr, comp = nullptr;
  std::vector<hipEvent_t> ev;   // per piece: copied
  hipEvent_t done = nullptr;    // this call's work on the device finished
  bool used = false;            // `done` recorded by an earlier call
  uint8_t* buf = nullptr;       // the device's pieces, source layout
  uint64_t buf_bytes = 0;
  uint8_t* meta = nullptr;      // offsets, lengths, side inputs of its pieces
  uint64_t meta_bytes = 0;
  uint16_t* out = nullptr;      // its results before they go home
  uint64_t out_n = 0;
  // Staged form (no peer access to the source, or forced): pieces travel
  // source HBM -> page-locked bounce buffer -> this device's HBM, results
  // back the same way. `stage` is a stream on the source device; its events
  // are made there too.
  int stage_dev = -1;
  hipStream_t stage = nullptr;
  uint8_t* hb[2] = { nullptr, nullptr }; // double-buffered bounce (page-locked)
  uint64_t hb_bytes = 0;
  uint16_t* hres = nullptr;              // results bounce (page-locked)
  uint64_t hres_bytes = 0;
  hipEvent_t staged[2] = { nullptr, nullptr }; // bounce j filled (source device)
  hipEvent_t bfree[2] = { nullptr, nullptr };  // bounce j drained (this device)
  bool bfree_used[2] = { false, false };
  hipEvent_t rdone = nullptr;  // results in hres (this device)
  hipEvent_t sdone = nullptr;  // results home (source device): the call's end
  bool sdone_used = false;
};

} // namespace

namespace {

// Device workspace of the flow router (validate_frames_rss_device), on the
// last source device; grown on demand.
struct RouteWs
{
  int device = -1;
  uint64_t n_cap = 0, cell_cap = 0, tab_cap = 0, packed_cap = 0;
  uint16_t* dev_of = nullptr;     // n (when the caller passes no device_of)
  uint32_t* perm = nullptr;       // n
  uint64_t* poff = nullptr;       // n
  uint16_t* plen = nullptr;       // n
  uint8_t* rflags = nullptr;      // n, routed order
  uint32_t* cells = nullptr;      // 3 x blocks x devices (counts, bytes, bases)
  uint64_t* base_bytes = nullptr; // blocks x devices
  uint64_t* totals = nullptr;     // 2 x tulips_amd::RT_MAX_DEV
  uint64_t* totals_host = nullptr; // page-locked copy
  uint16_t* table = nullptr;
  uint8_t* packed = nullptr;      // frames bound for other devices, by device
  // the last call's final kernel (launch_rss_home reads perm and rflags) done,
  // recorded on that call's stream: the next call, on any stream, waits for
  // it before it overwrites the workspace
  hipEvent_t done = nullptr;
  int done_device = -1;
  bool done_used = false;
};

} // namespace

struct tulips_csum_mctx
{
  std::vector<int> devices;
  std::vector<tulips_csum_ctx*> ctx;
  Workers* workers = nullptr;
  std::vector<uint32_t> bounds;
  std::vector<DevSlot> slots;   // device-resident calls
  uint64_t* plan_host = nullptr; // pinned: the arena cut plan read back
  uint64_t* plan_dev = nullptr;  // on the last source device
  int plan_device = -1;
  uint32_t plan_cap = 0;
  int peer_mode = 0;             // tulips_csum_mctx_set_peer_mode
  RouteWs route;                 // validate_frames_rss_device
};

extern "C" {

int
tulips_csum_shard_plan(const uint16_t* lengths, uint32_t n, uint32_t nshards,
                       uint32_t* bounds)
{
  if (!bounds || nshards == 0 || (n && !lengths)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i) {
    total += lengths[i];
  }
  // shard k starts at the first segment whose byte prefix reaches
  // k * total / nshards (an empty shard only when segments run out)
  bounds[0] = 0;
  uint64_t prefix = 0;
  uint32_t i = 0;
  for (uint32_t k = 1; k < nshards; ++k) {
    const uint64_t target = (total * k + nshards - 1) / nshards;
    while (i < n && prefix < target) {
      prefix += lengths[i++];
    }
    bounds[k] = i;
  }
  bounds[nshards] = n;
  return TULIPS_STATUS_OK;
}

int
tulips_csum_mctx_create(const int* devices, uint32_t ndevices, uint64_t chunk_bytes,
                        tulips_csum_mctx** out)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (!out || !devices || ndevices == 0 || ndevices > 64) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  *out = nullptr;
  tulips_csum_mctx* m = new (std::nothrow) tulips_csum_mctx();
  if (!m) {
    return TULIPS_STATUS_NO_MORE_RESOURCES;
  }
  // each device's staging copy gets its share of this process's CPUs
  const int share = std::max(1, tulips_amd::pack_threads() / int(ndevices));
  for (uint32_t k = 0; k < ndevices; ++k) {
    tulips_csum_ctx* c = nullptr;
    const int rc = tulips_amd::ctx_create(devices[k], chunk_bytes, share, &c);
    if (rc != TULIPS_STATUS_OK) {
      for (auto* x : m->ctx) {
        tulips_csum_ctx_destroy(x);
      }
      delete m;
      return rc;
    }
    m->devices.push_back(devices[k]);
    m->ctx.push_back(c);
  }
  m->bounds.resize(ndevices + 1);
  m->workers = new (std::nothrow) Workers(int(ndevices));
  if (!m->workers) {
    tulips_csum_mctx_destroy(m);
    return TULIPS_STATUS_NO_MORE_RESOURCES;
  }
  *out = m;
  return TULIPS_STATUS_OK;
}

int
tulips_csum_mctx_destroy(tulips_csum_mctx* m)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (!m) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  delete m->workers;
  for (auto* c : m->ctx) {
    tulips_csum_ctx_destroy(c);
  }
  int prev = 0;
  (void)hipGetDevice(&prev);
  for (auto& d : m->slots) {
    (void)hipSetDevice(d.device);
    for (hipStream_t st : { d.copy, d.comp }) {
      if (st) {
        (void)hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
      }
    }
    for (hipEvent_t e : d.ev) {
      (void)hipEventDestroy(e);
    }
    if (d.done) {
      (void)hipEventDestroy(d.done);
    }
    if (d.rdone) {
      (void)hipEventDestroy(d.rdone);
    }
    (void)hipFree(d.buf);
    (void)hipFree(d.meta);
    (void)hipFree(d.out);
    for (int j = 0; j < 2; ++j) {
      if (d.bfree[j]) {
        (void)hipEventDestroy(d.bfree[j]);
      }
    }
    if (d.stage) {
      (void)hipSetDevice(d.stage_dev);
      (void)hipStreamSynchronize(d.stage);
      (void)hipStreamDestroy(d.stage);
      for (int j = 0; j < 2; ++j) {
        (void)hipEventDestroy(d.staged[j]);
      }
      (void)hipEventDestroy(d.sdone);
    }
    for (int j = 0; j < 2; ++j) {
      (void)hipHostFree(d.hb[j]);
    }
    (void)hipHostFree(d.hres);
  }
  if (m->plan_dev) {
    (void)hipSetDevice(m->plan_device);
    (void)hipFree(m->plan_dev);
  }
  if (m->plan_host) {
    (void)hipHostFree(m->plan_host);
  }
  RouteWs& r = m->route;
  if (r.device >= 0) {
    (void)hipSetDevice(r.device);
    (void)hipDeviceSynchronize();
    for (void* p : { (void*)r.dev_of, (void*)r.perm, (void*)r.poff, (void*)r.plen,
                     (void*)r.rflags, (void*)r.cells, (void*)r.base_bytes, (void*)r.totals,
                     (void*)r.table, (void*)r.packed }) {
      (void)hipFree(p);
    }
  }
  if (r.done) {
    (void)hipSetDevice(r.done_device);
    (void)hipEventDestroy(r.done);
  }
  (void)hipHostFree(r.totals_host);
  (void)hipSetDevice(prev);
  delete m;
  return TULIPS_STATUS_OK;
}

int
tulips_csum_mctx_set_peer_mode(tulips_csum_mctx* m, int mode)
{
  if (!m || mode < 0 || mode > 1) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  m->peer_mode = mode;
  return TULIPS_STATUS_OK;
}

int
tulips_csum_mctx_shard_bounds(const tulips_csum_mctx* m, uint32_t* bounds)
{
  if (!m || !bounds) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  memcpy(bounds, m->bounds.data(), sizeof(uint32_t) * m->bounds.size());
  return TULIPS_STATUS_OK;
}

} // extern "C"

namespace {

// Run `one(ctx, i0, i1)` for every device's byte-balanced shard at once;
// the first failing status wins.
int
spread(tulips_csum_mctx* m, const uint16_t* lengths, uint32_t n,
       const std::function<int(tulips_csum_ctx*, uint32_t, uint32_t)>& one)
{
  const uint32_t nd = uint32_t(m->ctx.size());
  int rc = tulips_csum_shard_plan(lengths, n, nd, m->bounds.data());
  if (rc != TULIPS_STATUS_OK) {
    return rc;
  }
  std::vector<int> st(nd, TULIPS_STATUS_OK);
  m->workers->run([&](int k) {
    const uint32_t i0 = m->bounds[k], i1 = m->bounds[k + 1];
    if (i1 > i0) {
      st[k] = one(m->ctx[k], i0, i1);
    }
  });
  for (int s : st) {
    if (s != TULIPS_STATUS_OK) {
      return s;
    }
  }
  return TULIPS_STATUS_OK;
}

} // namespace

extern "C" {

int
tulips_csum_mctx_batch_host(tulips_csum_mctx* m, const uint8_t* base,
                            const uint64_t* offsets, const uint16_t* lengths,
                            const uint16_t* seeds, const uint32_t* src,
                            const uint32_t* dst, uint16_t* out, uint32_t n,
                            uint32_t mode)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (!m) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (n == 0) {
    return TULIPS_STATUS_OK;
  }
  if (!base || !offsets || !lengths || !out) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  return spread(m, lengths, n, [&](tulips_csum_ctx* c, uint32_t i0, uint32_t i1) {
    return tulips_csum_batch_host(c, base, offsets + i0, lengths + i0,
                                  seeds ? seeds + i0 : nullptr, src ? src + i0 : nullptr,
                                  dst ? dst + i0 : nullptr, out + i0, i1 - i0, mode);
  });
}

int
tulips_csum_mctx_validate_frames_host(tulips_csum_mctx* m, const uint8_t* base,
                                      const uint64_t* offsets, const uint16_t* lengths,
                                      uint32_t n, uint8_t* flags, uint32_t* counters)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (!m) {
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
  std::vector<uint32_t> part(4 * m->ctx.size(), 0);
  const int rc = spread(m, lengths, n, [&](tulips_csum_ctx* c, uint32_t i0, uint32_t i1) {
    const size_t k = size_t(std::find(m->ctx.begin(), m->ctx.end(), c) - m->ctx.begin());
    return tulips_csum_validate_frames_host(c, base, offsets + i0, lengths + i0, i1 - i0,
                                            flags + i0,
                                            counters ? part.data() + 4 * k : nullptr);
  });
  if (rc == TULIPS_STATUS_OK && counters) {
    for (size_t k = 0; k < m->ctx.size(); ++k) {
      for (int j = 0; j < 4; ++j) {
        counters[j] += part[4 * k + j];
      }
    }
  }
  return rc;
}

int
tulips_csum_mctx_validate_frames_rss_host(tulips_csum_mctx* m, const uint8_t* base,
                                          const uint64_t* offsets, const uint16_t* lengths,
                                          uint32_t n, const uint8_t* key, size_t key_len,
                                          uint32_t init, const uint16_t* table,
                                          uint32_t table_len, uint8_t* flags,
                                          uint32_t* counters, uint16_t* device_of)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (!m || !key || key_len < 4 || !table || table_len == 0) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  const uint32_t nd = uint32_t(m->ctx.size());
  for (uint32_t k = 0; k < table_len; ++k) {
    if (table[k] >= nd) {
      return TULIPS_STATUS_INVALID_ARGUMENT;
    }
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
  // 1. the 4-tuple of every option-less IPv4/TCP frame, as the NIC's RSS
  //    input: saddr | daddr | sport | dport (ports in host order); other
  //    frames go where table[0] says (the reference keeps slot 0 for L2
  //    flows, src/transport/ena/RedirectionTable.cpp:50-53)
  std::vector<uint32_t> tup_i, sa, da, hash;
  std::vector<uint16_t> sp, dp;
  tup_i.reserve(n);
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t* f = base + offsets[i];
    // non-first fragments carry payload where the ports would be, and a
    // first fragment's flow must land with the rest: fragments (MF set or a
    // fragment offset, bytes 20..21) go to table[0] like non-TCP frames
    if (lengths[i] >= 38 && f[12] == 0x08 && f[13] == 0x00 && f[14] == 0x45 && f[23] == 6 &&
        (f[20] & 0x3f) == 0 && f[21] == 0) {
      uint32_t s4, d4;
      memcpy(&s4, f + 26, 4);
      memcpy(&d4, f + 30, 4);
      tup_i.push_back(i);
      sa.push_back(s4);
      da.push_back(d4);
      sp.push_back(uint16_t((f[34] << 8) | f[35]));
      dp.push_back(uint16_t((f[36] << 8) | f[37]));
    }
  }
  // 2. their Toeplitz hashes on the first device (src/stack/Utils.cpp:86-133)
  hash.resize(tup_i.size());
  if (!tup_i.empty()) {
    const int rc = tulips_amd::ctx_rss_hash(m->ctx[0], sa.data(), da.data(), sp.data(),
                                            dp.data(), uint32_t(tup_i.size()), key, key_len,
                                            init, hash.data());
    if (rc != TULIPS_STATUS_OK) {
      return rc;
    }
  }
  // 3. indirection table -> device (RedirectionTable.cpp:88-96: hash % size)
  std::vector<uint16_t> dev(n, table[0]);
  for (size_t t = 0; t < tup_i.size(); ++t) {
    dev[tup_i[t]] = table[hash[t] % table_len];
  }
  // 4. each device validates its frames (arrival order kept within a
  //    device, so a flow's frames stay in order on its device)
  std::vector<std::vector<uint32_t>> idx(nd);
  for (uint32_t i = 0; i < n; ++i) {
    idx[dev[i]].push_back(i);
  }
  std::vector<std::vector<uint64_t>> offs(nd);
  std::vector<std::vector<uint16_t>> lens(nd);
  std::vector<std::vector<uint8_t>> fl(nd);
  for (uint32_t k = 0; k < nd; ++k) {
    offs[k].resize(idx[k].size());
    lens[k].resize(idx[k].size());
    fl[k].resize(idx[k].size());
    for (size_t j = 0; j < idx[k].size(); ++j) {
      offs[k][j] = offsets[idx[k][j]];
      lens[k][j] = lengths[idx[k][j]];
    }
  }
  std::vector<uint32_t> part(4 * nd, 0);
  std::vector<int> st(nd, TULIPS_STATUS_OK);
  m->workers->run([&](int k) {
    if (!idx[k].empty()) {
      st[k] = tulips_csum_validate_frames_host(m->ctx[k], base, offs[k].data(), lens[k].data(),
                                               uint32_t(idx[k].size()), fl[k].data(),
                                               counters ? part.data() + 4 * k : nullptr);
    }
  });
  m->bounds[0] = 0;
  for (uint32_t k = 0; k < nd; ++k) {
    if (st[k] != TULIPS_STATUS_OK) {
      return st[k];
    }
    m->bounds[k + 1] = m->bounds[k] + uint32_t(idx[k].size());
    for (size_t j = 0; j < idx[k].size(); ++j) {
      flags[idx[k][j]] = fl[k][j];
    }
    if (counters) {
      for (int c = 0; c < 4; ++c) {
        counters[c] += part[4 * k + c];
      }
    }
  }
  if (device_of) {
    memcpy(device_of, dev.data(), size_t(n) * 2);
  }
  return TULIPS_STATUS_OK;
}

} // extern "C"

// ---------------------------------------------------------------------------
// Device-resident batches over several devices.
// ---------------------------------------------------------------------------
namespace {

using tulips_amd::LaunchArgs;

// Piece p: segments [i0, i1) whose bytes lie in [lo, hi) of the source arena.
struct Piece
{
  uint64_t i0, i1, lo, hi;
};

// Thread j: piece j of an in-order arena cut at j * arena / P (the first
// segment starting at or after the cut opens the piece), as {i0, i1, lo, hi}.
__global__ __launch_bounds__(64) void
arena_plan_kernel(const uint64_t* __restrict__ offs, const uint16_t* __restrict__ lens,
                  uint32_t n, uint64_t arena, uint32_t P, uint64_t* __restrict__ plan)
{
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= P) {
    return;
  }
  auto lower = [&](uint64_t cut) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo) / 2;
      if (offs[mid] < cut) {
        lo = mid + 1;
      } else {
        hi = mid;
      }
    }
    return lo;
  };
  // cuts as (arena / P) * j + (arena % P) * j / P: no 64-bit overflow
  auto cut = [&](uint64_t k) { return (arena / P) * k + ((arena % P) * k) / P; };
  const uint32_t i0 = j == 0 ? 0u : lower(cut(j));
  const uint32_t i1 = j + 1 == P ? n : lower(cut(j + 1));
  uint64_t lo = 0, hi = 0;
  if (i1 > i0) {
    lo = offs[i0];
    hi = offs[i1 - 1] + lens[i1 - 1];
    hi = hi > arena ? arena : hi;
    lo = lo > hi ? hi : lo;
  }
  plan[4 * j + 0] = i0;
  plan[4 * j + 1] = i1;
  plan[4 * j + 2] = lo;
  plan[4 * j + 3] = hi;
}

struct DevGuard
{
  int prev = 0;
  DevGuard() { (void)hipGetDevice(&prev); }
  ~DevGuard() { (void)hipSetDevice(prev); }
};

int
status_of(hipError_t e)
{
  return e == hipSuccess             ? TULIPS_STATUS_OK
         : e == hipErrorOutOfMemory  ? TULIPS_STATUS_NO_MORE_RESOURCES
         : e == hipErrorInvalidValue ? TULIPS_STATUS_INVALID_ARGUMENT
                                     : TULIPS_STATUS_HARDWARE_ERROR;
}

#define TCS_TRY(x)                                                             \
  do {                                                                         \
    const hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                                    \
      return e_;                                                               \
    }                                                                          \
  } while (0)

// Streams, events, peer access (made once per context).
hipError_t
ensure_slots(tulips_csum_mctx* m)
{
  if (!m->slots.empty()) {
    return hipSuccess;
  }
  std::vector<DevSlot> slots(m->devices.size());
  for (size_t k = 0; k < slots.size(); ++k) {
    DevSlot& d = slots[k];
    d.device = m->devices[k];
    TCS_TRY(hipSetDevice(d.device));
    TCS_TRY(hipStreamCreateWithFlags(&d.copy, hipStreamNonBlocking));
    TCS_TRY(hipStreamCreateWithFlags(&d.comp, hipStreamNonBlocking));
    TCS_TRY(hipEventCreateWithFlags(&d.done, hipEventDisableTiming));
    // peers read every other listed device's HBM over xGMI
    for (int o : m->devices) {
      int can = 0;
      if (o != d.device && hipDeviceCanAccessPeer(&can, d.device, o) == hipSuccess && can) {
        const hipError_t e = hipDeviceEnablePeerAccess(o, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
          return e;
        }
        (void)hipGetLastError();
      }
    }
  }
  m->slots = std::move(slots);
  return hipSuccess;
}

// Grow `*p` (device memory on `dev`) to at least `bytes`; the slot's streams
// are idle first.
hipError_t
grow(DevSlot& d, void** p, uint64_t* have, uint64_t bytes)
{
  if (bytes <= *have) {
    return hipSuccess;
  }
  TCS_TRY(hipSetDevice(d.device));
  TCS_TRY(hipStreamSynchronize(d.copy));
  TCS_TRY(hipStreamSynchronize(d.comp));
  (void)hipFree(*p);
  *p = nullptr;
  *have = 0;
  TCS_TRY(hipMalloc(p, bytes));
  *have = bytes;
  return hipSuccess;
}

hipError_t
ensure_events(DevSlot& d, size_t n)
{
  TCS_TRY(hipSetDevice(d.device));
  while (d.ev.size() < n) {
    hipEvent_t e = nullptr;
    TCS_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    d.ev.push_back(e);
  }
  return hipSuccess;
}

// What one call spreads: the source arrays and how a piece is checksummed.
struct Job
{
  int src_dev;
  const uint8_t* base;
  bool arena;                 // else fixed stride
  uint64_t stride;            // fixed
  uint32_t length;            // fixed
  uint64_t arena_bytes;       // arena
  const uint64_t* offsets;    // arena
  const uint16_t* lengths;    // arena
  const uint16_t* seeds;
  const uint32_t* src;
  const uint32_t* dst;
  uint16_t* out;
  uint32_t mode;
};

// Checksum piece `pc` whose bytes [pc.lo, pc.hi) sit at `local` (the byte
// at source offset pc.lo), its arrays at the given device pointers, results
// to `out` (on the same device as everything else).
hipError_t
run_piece(const Job& J, const Piece& pc, const uint8_t* local, const uint64_t* offs,
          const uint16_t* lens, const uint16_t* seeds, const uint32_t* src,
          const uint32_t* dst, uint16_t* out, hipStream_t st)
{
  const uint32_t cnt = uint32_t(pc.i1 - pc.i0);
  if (!J.arena) {
    const int rc = tulips_csum_batch_fixed(local, J.stride, J.length, seeds, src, dst, out, cnt,
                                           J.mode, st);
    return rc == TULIPS_STATUS_OK ? hipSuccess
           : rc == TULIPS_STATUS_INVALID_ARGUMENT ? hipErrorInvalidValue
                                                  : hipErrorLaunchFailure;
  }
  LaunchArgs a{};
  a.seeds = seeds;
  a.src = src;
  a.dst = dst;
  a.out = out;
  a.n = cnt;
  a.mode = J.mode;
  a.kind = 5; // TULIPS_CSUM_KIND_SPAN
  a.unroll = tulips_amd::SPAN_DEFAULT_UNROLL;
  a.group = 0;
  a.nontemporal = true;
  a.offs_bias = pc.lo;
  return tulips_amd::launch_span(local, pc.hi - pc.lo, offs, lens, a, st);
}

// Staged-form resources of slot `d` for a call whose source is `src`: a
// stream and events on the source device, bounce buffers of at least
// `piece_bytes` and a results bounce of `res_bytes`. Made or grown with the
// slot's streams idle.
hipError_t
ensure_staging(DevSlot& d, int src, uint64_t piece_bytes, uint64_t res_bytes)
{
  if (d.stage && d.stage_dev != src) {
    TCS_TRY(hipSetDevice(d.stage_dev));
    TCS_TRY(hipStreamSynchronize(d.stage));
    (void)hipStreamDestroy(d.stage);
    for (int j = 0; j < 2; ++j) {
      (void)hipEventDestroy(d.staged[j]);
      d.staged[j] = nullptr;
    }
    (void)hipEventDestroy(d.sdone);
    d.sdone = nullptr;
    d.sdone_used = false;
    d.stage = nullptr;
  }
  if (!d.stage) {
    TCS_TRY(hipSetDevice(src));
    TCS_TRY(hipStreamCreateWithFlags(&d.stage, hipStreamNonBlocking));
    d.stage_dev = src;
    for (int j = 0; j < 2; ++j) {
      TCS_TRY(hipEventCreateWithFlags(&d.staged[j], hipEventDisableTiming));
    }
    TCS_TRY(hipEventCreateWithFlags(&d.sdone, hipEventDisableTiming));
  }
  TCS_TRY(hipSetDevice(d.device));
  if (!d.rdone) {
    TCS_TRY(hipEventCreateWithFlags(&d.rdone, hipEventDisableTiming));
  }
  for (int j = 0; j < 2; ++j) {
    if (!d.bfree[j]) {
      TCS_TRY(hipEventCreateWithFlags(&d.bfree[j], hipEventDisableTiming));
    }
  }
  if (piece_bytes > d.hb_bytes || res_bytes > d.hres_bytes) {
    TCS_TRY(hipStreamSynchronize(d.copy));
    TCS_TRY(hipStreamSynchronize(d.comp));
    TCS_TRY(hipSetDevice(d.stage_dev));
    TCS_TRY(hipStreamSynchronize(d.stage));
    TCS_TRY(hipSetDevice(d.device));
  }
  if (piece_bytes > d.hb_bytes) {
    for (int j = 0; j < 2; ++j) {
      (void)hipHostFree(d.hb[j]);
      d.hb[j] = nullptr;
    }
    d.hb_bytes = 0;
    for (int j = 0; j < 2; ++j) {
      void* p = nullptr;
      TCS_TRY(hipHostMalloc(&p, piece_bytes, 0));
      d.hb[j] = static_cast<uint8_t*>(p);
    }
    d.hb_bytes = piece_bytes;
    d.bfree_used[0] = d.bfree_used[1] = false;
  }
  if (res_bytes > d.hres_bytes) {
    (void)hipHostFree(d.hres);
    d.hres = nullptr;
    d.hres_bytes = 0;
    void* p = nullptr;
    TCS_TRY(hipHostMalloc(&p, res_bytes, 0));
    d.hres = static_cast<uint16_t*>(p);
    d.hres_bytes = res_bytes;
  }
  return hipSuccess;
}

// Whether slot `d` reaches source device `src` by peer DMA (xGMI).
bool
peer_reachable(const tulips_csum_mctx* m, const DevSlot& d, int src)
{
  if (m->peer_mode == 1) {
    return false;
  }
  if (d.device == src) {
    return true; // a device listed again: a local copy
  }
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, d.device, src) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return can != 0;
}

hipError_t
spread_device(tulips_csum_mctx* m, const Job& J, const std::vector<Piece>& pieces,
              uint32_t per_dev, hipStream_t caller)
{
  const size_t nd = m->slots.size();
  DevGuard guard;
  TCS_TRY(hipSetDevice(J.src_dev));
  hipEvent_t start = nullptr;
  TCS_TRY(hipEventCreateWithFlags(&start, hipEventDisableTiming));
  hipError_t e = hipEventRecord(start, caller);
  // the first listed entry on the source device works in place
  size_t home = nd;
  for (size_t k = 0; k < nd; ++k) {
    if (m->slots[k].device == J.src_dev) {
      home = k;
      break;
    }
  }
  const bool mtcp = (J.mode & 0xffu) == 2u;
  // per slot, the event that ends this call's work there (the caller's
  // stream waits for it), and the slots this call queued work on
  std::vector<hipEvent_t> fin(nd, nullptr);
  std::vector<char> touched(nd, 0);
  for (size_t k = 0; k < nd && e == hipSuccess; ++k) {
    DevSlot& d = m->slots[k];
    const size_t p0 = k * per_dev, p1 = std::min(pieces.size(), p0 + per_dev);
    m->bounds[k] = p0 < pieces.size() ? uint32_t(pieces[p0].i0) : uint32_t(pieces.back().i1);
    if (p0 >= p1) {
      continue;
    }
    // this device's run of pieces: segments [s0, s1), bytes from A (16-aligned)
    uint64_t s0 = pieces[p0].i0, s1 = pieces[p1 - 1].i1;
    if (s1 <= s0) {
      continue;
    }
    if (k == home) {
      if ((e = hipSetDevice(d.device)) != hipSuccess ||
          (e = hipStreamWaitEvent(d.comp, start, 0)) != hipSuccess) {
        break;
      }
      touched[k] = 1;
      for (size_t p = p0; p < p1 && e == hipSuccess; ++p) {
        const Piece& pc = pieces[p];
        if (pc.i1 > pc.i0) {
          e = run_piece(J, pc, J.base + pc.lo, J.arena ? J.offsets + pc.i0 : nullptr,
                        J.arena ? J.lengths + pc.i0 : nullptr,
                        (J.seeds && !mtcp) ? J.seeds + pc.i0 : nullptr,
                        mtcp ? J.src + pc.i0 : nullptr, mtcp ? J.dst + pc.i0 : nullptr,
                        J.out + pc.i0, d.comp);
        }
      }
      if (e == hipSuccess) {
        e = hipEventRecord(d.done, d.comp);
        d.used = true;
        fin[k] = d.done;
      }
      continue;
    }
    const uint64_t A = pieces[p0].lo & ~uint64_t(15);
    uint64_t Z = A;
    for (size_t p = p0; p < p1; ++p) {
      Z = std::max(Z, pieces[p].hi);
    }
    const uint64_t nseg = s1 - s0;
    // metadata layout: offsets (8 B), lengths (2 B), seeds (2 B), src, dst (4 B)
    const uint64_t m_off = 0, m_len = m_off + (J.arena ? 8 * nseg : 0);
    const uint64_t m_seed = (m_len + (J.arena ? 2 * nseg : 0) + 15) & ~uint64_t(15);
    const bool seeded = J.seeds && !mtcp;
    const uint64_t m_src = (m_seed + (seeded ? 2 * nseg : 0) + 15) & ~uint64_t(15);
    const uint64_t m_dst = m_src + (mtcp ? 4 * nseg : 0);
    const uint64_t m_end = m_dst + (mtcp ? 4 * nseg : 0) + 16;
    if ((e = grow(d, reinterpret_cast<void**>(&d.buf), &d.buf_bytes, Z - A + 64)) != hipSuccess ||
        (e = grow(d, reinterpret_cast<void**>(&d.meta), &d.meta_bytes, m_end)) != hipSuccess) {
      break;
    }
    uint64_t out_have = d.out_n * 2;
    if ((e = grow(d, reinterpret_cast<void**>(&d.out), &out_have, 2 * nseg + 16)) != hipSuccess ||
        (e = ensure_events(d, p1 - p0)) != hipSuccess) {
      break;
    }
    d.out_n = out_have / 2;
    // staged: per piece, its bytes and its metadata back to back in a bounce
    const bool staged = !peer_reachable(m, d, J.src_dev);
    auto meta_per_seg = [&]() {
      return (J.arena ? 10u : 0u) + (seeded ? 2u : 0u) + (mtcp ? 8u : 0u);
    };
    if (staged) {
      uint64_t most = 0;
      for (size_t p = p0; p < p1; ++p) {
        const Piece& pc = pieces[p];
        const uint64_t a0 = pc.lo & ~uint64_t(15);
        most = std::max<uint64_t>(most, ((pc.hi - a0 + 15) & ~uint64_t(15)) +
                                          (pc.i1 - pc.i0) * meta_per_seg() + 5 * 16);
      }
      if ((e = ensure_staging(d, J.src_dev, most, 2 * nseg + 16)) != hipSuccess) {
        break;
      }
    }
    if ((e = hipSetDevice(d.device)) != hipSuccess) {
      break;
    }
    touched[k] = 1;
    // after the caller's earlier work, and after this slot's previous call
    // stopped reading its buffers (and, staged, sent its results home)
    if ((e = hipStreamWaitEvent(d.copy, start, 0)) != hipSuccess ||
        (d.used && (e = hipStreamWaitEvent(d.copy, d.done, 0)) != hipSuccess) ||
        (d.sdone_used && (e = hipStreamWaitEvent(d.copy, d.sdone, 0)) != hipSuccess)) {
      break;
    }
    if (staged) {
      // the stage stream (source device) starts after the caller's work too
      if ((e = hipSetDevice(J.src_dev)) != hipSuccess ||
          (e = hipStreamWaitEvent(d.stage, start, 0)) != hipSuccess ||
          (e = hipSetDevice(d.device)) != hipSuccess) {
        break;
      }
    }
    const uint64_t* moffs = reinterpret_cast<const uint64_t*>(d.meta + m_off);
    const uint16_t* mlens = reinterpret_cast<const uint16_t*>(d.meta + m_len);
    const uint16_t* mseeds = reinterpret_cast<const uint16_t*>(d.meta + m_seed);
    const uint32_t* msrc = reinterpret_cast<const uint32_t*>(d.meta + m_src);
    const uint32_t* mdst = reinterpret_cast<const uint32_t*>(d.meta + m_dst);
    for (size_t p = p0; p < p1 && e == hipSuccess; ++p) {
      const Piece& pc = pieces[p];
      if (pc.i1 <= pc.i0) {
        continue;
      }
      const uint64_t c = pc.i1 - pc.i0, r = pc.i0 - s0;
      const uint64_t a0 = pc.lo & ~uint64_t(15);
      // (from, to, bytes) of this piece's transfers: bytes, then metadata
      struct Xfer
      {
        const void* from;
        uint8_t* to;
        uint64_t bytes;
      };
      Xfer xs[6];
      int nx = 0;
      xs[nx++] = { J.base + a0, d.buf + (a0 - A), pc.hi - a0 };
      if (J.arena) {
        xs[nx++] = { J.offsets + pc.i0, d.meta + m_off + 8 * r, 8 * c };
        xs[nx++] = { J.lengths + pc.i0, d.meta + m_len + 2 * r, 2 * c };
      }
      if (seeded) {
        xs[nx++] = { J.seeds + pc.i0, d.meta + m_seed + 2 * r, 2 * c };
      }
      if (mtcp) {
        xs[nx++] = { J.src + pc.i0, d.meta + m_src + 4 * r, 4 * c };
        xs[nx++] = { J.dst + pc.i0, d.meta + m_dst + 4 * r, 4 * c };
      }
      if (!staged) {
        for (int x = 0; x < nx && e == hipSuccess; ++x) {
          if (xs[x].bytes) {
            e = hipMemcpyPeerAsync(xs[x].to, d.device, xs[x].from, J.src_dev, xs[x].bytes,
                                   d.copy);
          }
        }
      } else {
        // source HBM -> bounce j on the stage stream (after the bounce's
        // previous contents reached this device), bounce j -> HBM here
        const int j = int((p - p0) & 1);
        uint64_t at[6], pos = 0;
        for (int x = 0; x < nx; ++x) {
          at[x] = pos;
          pos += (xs[x].bytes + 15) & ~uint64_t(15);
        }
        if ((e = hipSetDevice(J.src_dev)) != hipSuccess ||
            (d.bfree_used[j] && (e = hipStreamWaitEvent(d.stage, d.bfree[j], 0)) != hipSuccess)) {
          break;
        }
        for (int x = 0; x < nx && e == hipSuccess; ++x) {
          if (xs[x].bytes) {
            e = hipMemcpyAsync(d.hb[j] + at[x], xs[x].from, xs[x].bytes, hipMemcpyDeviceToHost,
                               d.stage);
          }
        }
        if (e != hipSuccess || (e = hipEventRecord(d.staged[j], d.stage)) != hipSuccess ||
            (e = hipSetDevice(d.device)) != hipSuccess ||
            (e = hipStreamWaitEvent(d.copy, d.staged[j], 0)) != hipSuccess) {
          break;
        }
        for (int x = 0; x < nx && e == hipSuccess; ++x) {
          if (xs[x].bytes) {
            e = hipMemcpyAsync(xs[x].to, d.hb[j] + at[x], xs[x].bytes, hipMemcpyHostToDevice,
                               d.copy);
          }
        }
        if (e == hipSuccess && (e = hipEventRecord(d.bfree[j], d.copy)) == hipSuccess) {
          d.bfree_used[j] = true;
        }
      }
      hipEvent_t ev = d.ev[p - p0];
      if (e == hipSuccess && (e = hipEventRecord(ev, d.copy)) == hipSuccess &&
          (e = hipStreamWaitEvent(d.comp, ev, 0)) == hipSuccess) {
        e = run_piece(J, pc, d.buf + (pc.lo - A), J.arena ? moffs + r : nullptr,
                      J.arena ? mlens + r : nullptr, seeded ? mseeds + r : nullptr,
                      mtcp ? msrc + r : nullptr, mtcp ? mdst + r : nullptr, d.out + r,
                      d.comp);
      }
      if (e == hipSuccess && !staged) {
        e = hipMemcpyPeerAsync(J.out + pc.i0, J.src_dev, d.out + r, d.device, 2 * c, d.comp);
      }
    }
    if (e == hipSuccess) {
      e = hipEventRecord(d.done, d.comp);
      d.used = true;
      fin[k] = d.done;
    }
    if (e == hipSuccess && staged) {
      // all of this device's results in one bounce, then home
      if ((e = hipMemcpyAsync(d.hres, d.out, 2 * nseg, hipMemcpyDeviceToHost, d.comp)) ==
            hipSuccess &&
          (e = hipEventRecord(d.rdone, d.comp)) == hipSuccess &&
          (e = hipSetDevice(J.src_dev)) == hipSuccess &&
          (e = hipStreamWaitEvent(d.stage, d.rdone, 0)) == hipSuccess &&
          (e = hipMemcpyAsync(J.out + s0, d.hres, 2 * nseg, hipMemcpyHostToDevice, d.stage)) ==
            hipSuccess &&
          (e = hipEventRecord(d.sdone, d.stage)) == hipSuccess) {
        d.sdone_used = true;
        fin[k] = d.sdone;
      }
    }
  }
  m->bounds[nd] = pieces.empty() ? 0u : uint32_t(pieces.back().i1);
  // the caller's stream continues once every device's results are home
  if (e == hipSuccess && (e = hipSetDevice(J.src_dev)) == hipSuccess) {
    for (size_t k = 0; k < nd && e == hipSuccess; ++k) {
      if (fin[k]) {
        e = hipStreamWaitEvent(caller, fin[k], 0);
      }
    }
  }
  if (e != hipSuccess) {
    // a failure part-way: the work already queued may still write the
    // caller's `out`; it is drained before the error is reported, so the
    // caller may free or reuse its buffers at once
    for (size_t k = 0; k < nd; ++k) {
      DevSlot& d = m->slots[k];
      if (!touched[k]) {
        continue;
      }
      (void)hipSetDevice(d.device);
      (void)hipStreamSynchronize(d.copy);
      (void)hipStreamSynchronize(d.comp);
      if (d.stage) {
        (void)hipSetDevice(d.stage_dev);
        (void)hipStreamSynchronize(d.stage);
      }
    }
    (void)hipGetLastError();
  }
  (void)hipSetDevice(J.src_dev);
  (void)hipEventDestroy(start);
  return e;
}

// Pieces per device: about 32 MiB each (so copies and kernels overlap), at
// least one, at most 64.
uint32_t
pieces_per_device(uint64_t bytes, size_t nd)
{
  const uint64_t per = bytes / (nd ? nd : 1);
  const uint64_t c = (per + (32ull << 20) - 1) >> 25;
  return uint32_t(std::min<uint64_t>(64, std::max<uint64_t>(1, c)));
}

int
check_common(tulips_csum_mctx* m, void* stream, const uint16_t* out, uint32_t mode,
             const uint32_t* src, const uint32_t* dst, int* src_dev)
{
  if (!m || !out) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if ((mode & ~0x1ffu) != 0 || (mode & 0xffu) > 2 || ((mode & 0xffu) == 2 && (!src || !dst))) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return TULIPS_STATUS_INVALID_ARGUMENT; // the cut plan needs the host
  }
  hipDevice_t d = 0;
  if (hipStreamGetDevice(st, &d) != hipSuccess) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  *src_dev = int(d);
  return TULIPS_STATUS_OK;
}

} // namespace

extern "C" {

int
tulips_csum_mctx_batch_fixed_device(tulips_csum_mctx* m, const uint8_t* base, uint64_t stride,
                                    uint32_t length, const uint16_t* seeds,
                                    const uint32_t* src, const uint32_t* dst, uint16_t* out,
                                    uint32_t n, uint32_t mode, void* stream)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (n == 0) {
    return m ? TULIPS_STATUS_OK : TULIPS_STATUS_INVALID_ARGUMENT;
  }
  int sdev = 0;
  int rc = check_common(m, stream, out, mode, src, dst, &sdev);
  if (rc != TULIPS_STATUS_OK) {
    return rc;
  }
  if (!base || length > TULIPS_CSUM_MAX_SEGMENT) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  Job J{};
  J.src_dev = sdev;
  J.base = base;
  J.stride = stride;
  J.length = length;
  J.seeds = seeds;
  J.src = src;
  J.dst = dst;
  J.out = out;
  J.mode = mode;
  DevGuard guard;
  hipError_t e = ensure_slots(m);
  if (e != hipSuccess) {
    return status_of(e);
  }
  // equal segment counts = equal bytes
  const size_t nd = m->slots.size();
  const uint32_t C = pieces_per_device(uint64_t(n) * stride, nd);
  const uint64_t P = uint64_t(C) * nd;
  std::vector<Piece> pieces(P);
  for (uint64_t p = 0; p < P; ++p) {
    Piece& pc = pieces[p];
    pc.i0 = uint64_t(n) * p / P;
    pc.i1 = uint64_t(n) * (p + 1) / P;
    pc.lo = pc.i0 * stride;
    pc.hi = pc.i1 > pc.i0 ? (pc.i1 - 1) * stride + length : pc.lo;
  }
  return status_of(spread_device(m, J, pieces, C, static_cast<hipStream_t>(stream)));
}

int
tulips_csum_mctx_batch_arena_device(tulips_csum_mctx* m, const uint8_t* base,
                                    uint64_t arena_bytes, const uint64_t* offsets,
                                    const uint16_t* lengths, const uint16_t* seeds,
                                    const uint32_t* src, const uint32_t* dst, uint16_t* out,
                                    uint32_t n, uint32_t mode, void* stream)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  if (n == 0) {
    return m ? TULIPS_STATUS_OK : TULIPS_STATUS_INVALID_ARGUMENT;
  }
  int sdev = 0;
  int rc = check_common(m, stream, out, mode, src, dst, &sdev);
  if (rc != TULIPS_STATUS_OK) {
    return rc;
  }
  if ((!base && arena_bytes) || !offsets || !lengths) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  Job J{};
  J.src_dev = sdev;
  J.base = base;
  J.arena = true;
  J.arena_bytes = arena_bytes;
  J.offsets = offsets;
  J.lengths = lengths;
  J.seeds = seeds;
  J.src = src;
  J.dst = dst;
  J.out = out;
  J.mode = mode;
  DevGuard guard;
  hipError_t e = ensure_slots(m);
  if (e != hipSuccess) {
    return status_of(e);
  }
  const size_t nd = m->slots.size();
  const uint32_t C = pieces_per_device(arena_bytes, nd);
  const uint32_t P = uint32_t(C * nd);
  // the cut plan: found on the source device, read back (one small D2H)
  hipStream_t st = static_cast<hipStream_t>(stream);
  if ((e = hipSetDevice(sdev)) != hipSuccess) {
    return status_of(e);
  }
  if (m->plan_device != sdev || m->plan_cap < P) {
    if (m->plan_dev) {
      DevGuard g2;
      (void)hipSetDevice(m->plan_device);
      (void)hipDeviceSynchronize();
      (void)hipFree(m->plan_dev);
      m->plan_dev = nullptr;
    }
    if (m->plan_host) {
      (void)hipHostFree(m->plan_host);
      m->plan_host = nullptr;
    }
    m->plan_cap = 0;
    if ((e = hipMalloc(&m->plan_dev, 32ull * P)) != hipSuccess ||
        (e = hipHostMalloc(&m->plan_host, 32ull * P, 0)) != hipSuccess) {
      return status_of(e);
    }
    m->plan_device = sdev;
    m->plan_cap = P;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL(arena_plan_kernel, dim3((P + 63) / 64), dim3(64), 0, st, offsets, lengths,
                     n, arena_bytes, P, m->plan_dev);
  if ((e = hipGetLastError()) != hipSuccess ||
      (e = hipMemcpyAsync(m->plan_host, m->plan_dev, 32ull * P, hipMemcpyDeviceToHost, st)) !=
        hipSuccess ||
      (e = hipStreamSynchronize(st)) != hipSuccess) {
    return status_of(e);
  }
  std::vector<Piece> pieces(P);
  for (uint32_t p = 0; p < P; ++p) {
    const uint64_t* q = m->plan_host + 4 * p;
    pieces[p] = Piece{ q[0], q[1], q[2], q[3] };
  }
  return status_of(spread_device(m, J, pieces, C, st));
}

} // extern "C"

// ---------------------------------------------------------------------------
// Flow-affine validation of device-resident frames (rss_route.hip).
// ---------------------------------------------------------------------------
namespace {

using tulips_amd::launch_rss_gather;
using tulips_amd::launch_rss_home;
using tulips_amd::launch_rss_route;
using tulips_amd::launch_rss_scatter;
using tulips_amd::rss_route_blocks;
using tulips_amd::rss_route_windows;
using tulips_amd::RouteStarts;
using tulips_amd::RouteWindows;
using tulips_amd::RT_MAX_DEV;

// (Re)size the router's workspace for n frames / `cells` histogram cells /
// `tab` table entries / `packed` bytes on device `dev`. Growth waits for the
// device (and every slot) first: earlier calls may still read these.
hipError_t
route_ws(tulips_csum_mctx* m, int dev, uint64_t n, uint64_t cells, uint64_t tab, uint64_t packed)
{
  RouteWs& r = m->route;
  const bool moved = r.device != dev;
  const bool grow_n = moved || n > r.n_cap, grow_c = moved || cells > r.cell_cap;
  const bool grow_t = moved || tab > r.tab_cap, grow_p = moved || packed > r.packed_cap;
  if (!(grow_n || grow_c || grow_t || grow_p || !r.totals_host)) {
    return hipSuccess;
  }
  for (auto& d : m->slots) {
    TCS_TRY(hipSetDevice(d.device));
    TCS_TRY(hipStreamSynchronize(d.copy));
    TCS_TRY(hipStreamSynchronize(d.comp));
  }
  if (r.device >= 0) {
    TCS_TRY(hipSetDevice(r.device));
    TCS_TRY(hipDeviceSynchronize());
  }
  auto realloc_dev = [&](bool grow, auto** p, uint64_t bytes) -> hipError_t {
    if (!grow) {
      return hipSuccess;
    }
    if (*p) {
      TCS_TRY(hipSetDevice(r.device));
      (void)hipFree(*p);
      *p = nullptr;
    }
    TCS_TRY(hipSetDevice(dev));
    void* q = nullptr;
    TCS_TRY(hipMalloc(&q, bytes ? bytes : 16));
    *p = static_cast<std::remove_reference_t<decltype(*p)>>(q);
    return hipSuccess;
  };
  const uint64_t nn = std::max<uint64_t>(n, 1), nc = std::max<uint64_t>(cells, 1);
  TCS_TRY(realloc_dev(grow_n, &r.dev_of, 2 * nn));
  TCS_TRY(realloc_dev(grow_n, &r.perm, 4 * nn));
  TCS_TRY(realloc_dev(grow_n, &r.poff, 8 * nn));
  TCS_TRY(realloc_dev(grow_n, &r.plen, 2 * nn));
  TCS_TRY(realloc_dev(grow_n, &r.rflags, nn));
  TCS_TRY(realloc_dev(grow_c, &r.cells, 12 * nc));
  TCS_TRY(realloc_dev(grow_c, &r.base_bytes, 8 * nc));
  TCS_TRY(realloc_dev(moved || !r.totals, &r.totals, 16 * RT_MAX_DEV));
  TCS_TRY(realloc_dev(grow_t, &r.table, 2 * std::max<uint64_t>(tab, 1)));
  TCS_TRY(realloc_dev(grow_p, &r.packed, std::max<uint64_t>(packed, 16)));
  if (grow_n) {
    r.n_cap = nn;
  }
  if (grow_c) {
    r.cell_cap = nc;
  }
  if (grow_t) {
    r.tab_cap = std::max<uint64_t>(tab, 1);
  }
  if (grow_p) {
    r.packed_cap = std::max<uint64_t>(packed, 16);
  }
  if (!r.totals_host) {
    void* h = nullptr;
    TCS_TRY(hipHostMalloc(&h, 16 * RT_MAX_DEV, 0));
    r.totals_host = static_cast<uint64_t*>(h);
  }
  r.device = dev;
  return hipSuccess;
}

hipError_t
validate_rss_device(tulips_csum_mctx* m, int sdev, const uint8_t* base, const uint64_t* offsets,
                    const uint16_t* lengths, uint32_t n, const RouteWindows& win, uint32_t init,
                    const uint16_t* table, uint32_t table_len, uint8_t* flags,
                    uint32_t* counters, uint16_t* device_of, hipStream_t st)
{
  const uint32_t nd = uint32_t(m->slots.size());
  DevGuard guard;
  uint32_t home = nd;
  for (uint32_t k = 0; k < nd; ++k) {
    if (m->slots[k].device == sdev) {
      home = k;
      break;
    }
  }
  const uint64_t cells = uint64_t(rss_route_blocks(n)) * nd;
  TCS_TRY(route_ws(m, sdev, n, cells, table_len, 0));
  RouteWs& r = m->route;
  TCS_TRY(hipSetDevice(sdev));
  // the previous call's devices may still read the workspace (its packed
  // runs, offsets, lengths), and its last kernel (perm, rflags), when that
  // call was ordered on another stream
  for (auto& d : m->slots) {
    if (d.used) {
      TCS_TRY(hipStreamWaitEvent(st, d.done, 0));
    }
  }
  if (r.done_used) {
    TCS_TRY(hipStreamWaitEvent(st, r.done, 0));
  }
  if (r.done && r.done_device != sdev) {
    TCS_TRY(hipSetDevice(r.done_device));
    TCS_TRY(hipEventSynchronize(r.done));
    (void)hipEventDestroy(r.done);
    r.done = nullptr;
    r.done_used = false;
    TCS_TRY(hipSetDevice(sdev));
  }
  if (!r.done) {
    TCS_TRY(hipEventCreateWithFlags(&r.done, hipEventDisableTiming));
    r.done_device = sdev;
  }
  TCS_TRY(hipMemcpyAsync(r.table, table, 2ull * table_len, hipMemcpyHostToDevice, st));
  uint16_t* dev_of = device_of ? device_of : r.dev_of;
  uint32_t* blk_cnt = r.cells;
  uint32_t* blk_bytes = r.cells + cells;
  uint32_t* base_cnt = r.cells + 2 * cells;
  TCS_TRY(launch_rss_route(win, base, offsets, lengths, n, r.table, table_len, init, nd, dev_of,
                           blk_cnt, blk_bytes, base_cnt, r.base_bytes, r.totals, st));
  TCS_TRY(hipMemcpyAsync(r.totals_host, r.totals, 16ull * nd, hipMemcpyDeviceToHost, st));
  TCS_TRY(hipStreamSynchronize(st));
  // frames per device (bounds) and where each other device's packed run
  // starts in the gather buffer
  RouteStarts starts{};
  uint64_t packed = 0;
  m->bounds[0] = 0;
  for (uint32_t k = 0; k < nd; ++k) {
    m->bounds[k + 1] = m->bounds[k] + uint32_t(r.totals_host[k]);
    if (k != home) {
      starts.at[k] = packed;
      packed += r.totals_host[nd + k];
    }
  }
  std::vector<uint64_t> run_bytes(nd);
  for (uint32_t k = 0; k < nd; ++k) {
    run_bytes[k] = r.totals_host[nd + k];
  }
  TCS_TRY(route_ws(m, sdev, n, cells, table_len, packed));
  TCS_TRY(hipSetDevice(sdev));
  TCS_TRY(launch_rss_scatter(offsets, lengths, n, nd, home, dev_of, base_cnt, r.base_bytes,
                             r.totals, r.perm, r.poff, r.plen, st));
  if (packed) {
    TCS_TRY(launch_rss_gather(base, offsets, n, home, dev_of, r.perm, r.poff, r.plen, starts,
                              r.packed, st));
  }
  hipEvent_t routed = nullptr;
  TCS_TRY(hipEventCreateWithFlags(&routed, hipEventDisableTiming));
  hipError_t e = hipEventRecord(routed, st);
  std::vector<hipEvent_t> fin(nd, nullptr);
  for (uint32_t k = 0; k < nd && e == hipSuccess; ++k) {
    DevSlot& d = m->slots[k];
    const uint32_t b0 = m->bounds[k], cnt = m->bounds[k + 1] - b0;
    if (cnt == 0) {
      continue;
    }
    int rc = TULIPS_STATUS_OK;
    if (k == home) {
      if ((e = hipSetDevice(d.device)) != hipSuccess ||
          (e = hipStreamWaitEvent(d.comp, routed, 0)) != hipSuccess) {
        break;
      }
      rc = tulips_csum_validate_frames(base, r.poff + b0, r.plen + b0, cnt, r.rflags + b0,
                                       nullptr, d.comp);
    } else {
      // its packed frames, offsets (within the run), lengths, then flags
      const uint64_t m_len = 8ull * cnt, m_fl = (m_len + 2ull * cnt + 15) & ~uint64_t(15);
      // no peer path to the source (or staging forced): the run, offsets and
      // lengths go source HBM -> page-locked bounce (stage stream, source
      // device) -> this device's HBM, the flags back the same way, as the
      // device-resident batches do (spread_device)
      const bool staged = !peer_reachable(m, d, sdev);
      const uint64_t run16 = (run_bytes[k] + 15) & ~uint64_t(15);
      const uint64_t off16 = (8ull * cnt + 15) & ~uint64_t(15);
      if ((e = grow(d, reinterpret_cast<void**>(&d.buf), &d.buf_bytes, run_bytes[k] + 64)) !=
            hipSuccess ||
          (e = grow(d, reinterpret_cast<void**>(&d.meta), &d.meta_bytes, m_fl + cnt + 16)) !=
            hipSuccess ||
          (staged && (e = ensure_staging(d, sdev, run16 + off16 + 2ull * cnt + 16,
                                         cnt + 16)) != hipSuccess) ||
          (e = hipSetDevice(d.device)) != hipSuccess ||
          (e = hipStreamWaitEvent(d.copy, routed, 0)) != hipSuccess ||
          (d.used && (e = hipStreamWaitEvent(d.copy, d.done, 0)) != hipSuccess) ||
          (d.sdone_used && (e = hipStreamWaitEvent(d.copy, d.sdone, 0)) != hipSuccess)) {
        break;
      }
      if (!staged) {
        // peer DMA over xGMI
        if ((e = hipMemcpyPeerAsync(d.buf, d.device, r.packed + starts.at[k], sdev,
                                    run_bytes[k], d.copy)) != hipSuccess ||
            (e = hipMemcpyPeerAsync(d.meta, d.device, r.poff + b0, sdev, 8ull * cnt,
                                    d.copy)) != hipSuccess ||
            (e = hipMemcpyPeerAsync(d.meta + m_len, d.device, r.plen + b0, sdev, 2ull * cnt,
                                    d.copy)) != hipSuccess) {
          break;
        }
      } else {
        uint8_t* hb = d.hb[0];
        if ((e = hipSetDevice(sdev)) != hipSuccess ||
            (e = hipStreamWaitEvent(d.stage, routed, 0)) != hipSuccess ||
            (d.bfree_used[0] && (e = hipStreamWaitEvent(d.stage, d.bfree[0], 0)) != hipSuccess) ||
            (run_bytes[k] && (e = hipMemcpyAsync(hb, r.packed + starts.at[k], run_bytes[k],
                                                 hipMemcpyDeviceToHost, d.stage)) != hipSuccess) ||
            (e = hipMemcpyAsync(hb + run16, r.poff + b0, 8ull * cnt, hipMemcpyDeviceToHost,
                                d.stage)) != hipSuccess ||
            (e = hipMemcpyAsync(hb + run16 + off16, r.plen + b0, 2ull * cnt,
                                hipMemcpyDeviceToHost, d.stage)) != hipSuccess ||
            (e = hipEventRecord(d.staged[0], d.stage)) != hipSuccess ||
            (e = hipSetDevice(d.device)) != hipSuccess ||
            (e = hipStreamWaitEvent(d.copy, d.staged[0], 0)) != hipSuccess ||
            (run_bytes[k] && (e = hipMemcpyAsync(d.buf, hb, run_bytes[k], hipMemcpyHostToDevice,
                                                 d.copy)) != hipSuccess) ||
            (e = hipMemcpyAsync(d.meta, hb + run16, 8ull * cnt, hipMemcpyHostToDevice,
                                d.copy)) != hipSuccess ||
            (e = hipMemcpyAsync(d.meta + m_len, hb + run16 + off16, 2ull * cnt,
                                hipMemcpyHostToDevice, d.copy)) != hipSuccess ||
            (e = hipEventRecord(d.bfree[0], d.copy)) != hipSuccess) {
          break;
        }
        d.bfree_used[0] = true;
      }
      if ((e = ensure_events(d, 1)) != hipSuccess || (e = hipSetDevice(d.device)) != hipSuccess ||
          (e = hipEventRecord(d.ev[0], d.copy)) != hipSuccess ||
          (e = hipStreamWaitEvent(d.comp, d.ev[0], 0)) != hipSuccess) {
        break;
      }
      rc = tulips_csum_validate_frames(d.buf, reinterpret_cast<const uint64_t*>(d.meta),
                                       reinterpret_cast<const uint16_t*>(d.meta + m_len), cnt,
                                       d.meta + m_fl, nullptr, d.comp);
      if (rc == TULIPS_STATUS_OK && !staged) {
        e = hipMemcpyPeerAsync(r.rflags + b0, sdev, d.meta + m_fl, d.device, cnt, d.comp);
      }
      if (rc == TULIPS_STATUS_OK && staged && e == hipSuccess) {
        // the flags home through the results bounce; the caller's stream
        // waits for the stage stream's copy (sdone) instead of `done`
        if ((e = hipMemcpyAsync(d.hres, d.meta + m_fl, cnt, hipMemcpyDeviceToHost, d.comp)) ==
              hipSuccess &&
            (e = hipEventRecord(d.done, d.comp)) == hipSuccess &&
            (e = hipEventRecord(d.rdone, d.comp)) == hipSuccess &&
            (e = hipSetDevice(sdev)) == hipSuccess &&
            (e = hipStreamWaitEvent(d.stage, d.rdone, 0)) == hipSuccess &&
            (e = hipMemcpyAsync(r.rflags + b0, d.hres, cnt, hipMemcpyHostToDevice, d.stage)) ==
              hipSuccess &&
            (e = hipEventRecord(d.sdone, d.stage)) == hipSuccess) {
          d.used = true;
          d.sdone_used = true;
          fin[k] = d.sdone;
        }
        if (e != hipSuccess) {
          break;
        }
        continue;
      }
    }
    if (rc != TULIPS_STATUS_OK && e == hipSuccess) {
      e = rc == TULIPS_STATUS_NO_MORE_RESOURCES ? hipErrorOutOfMemory : hipErrorLaunchFailure;
    }
    if (e == hipSuccess && (e = hipEventRecord(d.done, d.comp)) == hipSuccess) {
      d.used = true;
      fin[k] = d.done;
    }
  }
  if (e == hipSuccess && (e = hipSetDevice(sdev)) == hipSuccess) {
    for (uint32_t k = 0; k < nd && e == hipSuccess; ++k) {
      if (fin[k]) {
        e = hipStreamWaitEvent(st, fin[k], 0);
      }
    }
  }
  if (e == hipSuccess) {
    e = launch_rss_home(r.perm, r.rflags, n, flags, counters, st);
  }
  if (e == hipSuccess && (e = hipEventRecord(r.done, st)) == hipSuccess) {
    r.done_used = true;
  }
  if (e != hipSuccess) {
    for (auto& d : m->slots) { // drain before reporting (the caller may free)
      (void)hipSetDevice(d.device);
      (void)hipStreamSynchronize(d.copy);
      (void)hipStreamSynchronize(d.comp);
    }
    (void)hipSetDevice(sdev);
    (void)hipStreamSynchronize(st);
    (void)hipGetLastError();
  }
  (void)hipSetDevice(sdev);
  (void)hipEventDestroy(routed);
  return e;
}

} // namespace

extern "C" int
tulips_csum_mctx_validate_frames_rss_device(tulips_csum_mctx* m, const uint8_t* base,
                                            const uint64_t* offsets, const uint16_t* lengths,
                                            uint32_t n, const uint8_t* key, size_t key_len,
                                            uint32_t init, const uint16_t* table,
                                            uint32_t table_len, uint8_t* flags,
                                            uint32_t* counters, uint16_t* device_of,
                                            void* stream)
{
  tulips_amd::RelaxedCapture relaxed; // beside other threads' captures
  tulips_amd::RouteWindows win;
  if (!m || !table || table_len == 0 || table_len > 65536 ||
      !rss_route_windows(key, key_len, &win)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  const uint32_t nd = uint32_t(m->devices.size());
  for (uint32_t k = 0; k < table_len; ++k) {
    if (table[k] >= nd) {
      return TULIPS_STATUS_INVALID_ARGUMENT;
    }
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return TULIPS_STATUS_INVALID_ARGUMENT; // the per-device counts need the host
  }
  hipDevice_t sd = 0;
  if (hipStreamGetDevice(st, &sd) != hipSuccess) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  if (n == 0) {
    DevGuard g;
    (void)hipSetDevice(int(sd));
    return counters ? status_of(hipMemsetAsync(counters, 0, 16, st)) : TULIPS_STATUS_OK;
  }
  if (!base || !offsets || !lengths || (!flags && !counters)) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  DevGuard guard;
  hipError_t e = ensure_slots(m);
  if (e != hipSuccess) {
    return status_of(e);
  }
  return status_of(validate_rss_device(m, int(sd), base, offsets, lengths, n, win, init, table,
                                       table_len, flags, counters, device_of, st));
}
