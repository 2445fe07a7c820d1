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
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/tulips_csum.h"

namespace tulips_amd {
int pack_threads();
int ctx_create(int device, uint64_t chunk_bytes, int threads, tulips_csum_ctx** ctx);
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

struct tulips_csum_mctx
{
  std::vector<int> devices;
  std::vector<tulips_csum_ctx*> ctx;
  Workers* workers = nullptr;
  std::vector<uint32_t> bounds;
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
  if (!m) {
    return TULIPS_STATUS_INVALID_ARGUMENT;
  }
  delete m->workers;
  for (auto* c : m->ctx) {
    tulips_csum_ctx_destroy(c);
  }
  delete m;
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

} // extern "C"
