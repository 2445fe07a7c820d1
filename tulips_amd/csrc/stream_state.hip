// stream_state.hip — per-(device, stream) state registry (stream_state.h),
// graph ownership of captured arrays, and tulips_csum_release_stream.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <utility>
#include <vector>

#include "../../include/tulips_csum.h"
#include "csum_launch.h"
#include "stream_state.h"

namespace tulips_amd {
namespace {

std::mutex g_mutex;
std::map<std::pair<int, hipStream_t>, std::shared_ptr<StreamState>> g_states;

// Arrays of destroyed graphs, queued by the user objects' destructors (which
// may run on a runtime thread, during any HIP call or at process exit: the
// queue is never destroyed, and the destructor makes no HIP call).
std::mutex* const g_reclaim_mutex = new std::mutex;
std::vector<GraphArrays*>* const g_reclaim = new std::vector<GraphArrays*>;
std::atomic<uint32_t> g_reclaim_n{ 0 };

constexpr size_t SHARD_BYTES = sizeof(uint32_t) * CNT_LINE * CNT_SHARDS;
static_assert(SHARD_BYTES % 8 == 0, "shards are made as 64-bit words");

void
on_graph_destroyed(void* p)
{
  std::lock_guard<std::mutex> g(*g_reclaim_mutex);
  g_reclaim->push_back(static_cast<GraphArrays*>(p));
  g_reclaim_n.fetch_add(1, std::memory_order_release);
}

hipError_t
stream_device(hipStream_t stream, int* dev)
{
  hipDevice_t d = 0;
  hipError_t e = hipStreamGetDevice(stream, &d);
  if (e != hipSuccess) {
    return e;
  }
  *dev = int(d);
  return hipSuccess;
}

// Zeroes words [0, n) of p (a kernel: inside a capture it is a kernel node
// of the graph, which a captured hipMemsetAsync on an array allocated in the
// capture did not reliably become).
__global__ __launch_bounds__(256) void
zero_words_kernel(uint64_t* __restrict__ p, uint64_t n)
{
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += uint64_t(gridDim.x) * 256) {
    p[i] = 0;
  }
}

hipError_t
launch_zero_words(uint64_t* p, uint64_t n, hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  const uint64_t want = (n + 255) / 256;
  (void)hipGetLastError();
  hipLaunchKernelGGL(zero_words_kernel, dim3(uint32_t(want < 1024 ? want : 1024)), dim3(256), 0,
                     stream, p, n);
  return hipGetLastError();
}

// An array of `words` zeroed words on `device`, zeroed in `stream`'s order:
// outside a capture the caller synchronises `stream` before anything else
// can read it; inside a capture (the allocation made in relaxed capture
// mode) the zeroing is a kernel node of the graph, run before the captured
// kernels at every replay. Inside a capture the array is handed to the
// capture's graph (capture_keep) whether or not the zeroing could be
// recorded, so nothing is freed while the capture is in progress.
hipError_t
zeroed_words(StreamState& s, uint64_t words, bool capturing, uint64_t** out)
{
  *out = nullptr;
  void* p = nullptr;
  hipError_t e = device_malloc(s.device, &p, sizeof(uint64_t) * words);
  if (e != hipSuccess) {
    return e;
  }
  if (capturing) {
    capture_keep(s, std::vector<void*>{ p });
  }
  e = launch_zero_words(static_cast<uint64_t*>(p), words, s.stream);
  if (e != hipSuccess) {
    if (!capturing) {
      (void)sync_stream(s.stream);
      device_free(s.device, std::vector<void*>{ p });
    }
    return e;
  }
  *out = static_cast<uint64_t*>(p);
  return hipSuccess;
}

} // namespace

hipError_t
device_malloc(int device, void** p, size_t bytes)
{
  *p = nullptr;
  int prev = 0;
  hipError_t e = hipGetDevice(&prev);
  if (e != hipSuccess) {
    return e;
  }
  if (prev != device && (e = hipSetDevice(device)) != hipSuccess) {
    return e;
  }
  {
    RelaxedCapture relaxed;
    e = hipMalloc(p, bytes);
  }
  if (prev != device) {
    (void)hipSetDevice(prev);
  }
  return e;
}

void
device_free(int device, const std::vector<void*>& ps)
{
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  {
    RelaxedCapture relaxed;
    for (void* p : ps) {
      if (p) {
        (void)hipFree(p);
      }
    }
  }
  (void)hipSetDevice(prev);
}

hipError_t
sync_stream(hipStream_t stream)
{
  RelaxedCapture relaxed;
  return hipStreamSynchronize(stream);
}

void
reclaim_graph_arrays()
{
  if (g_reclaim_n.load(std::memory_order_acquire) == 0) {
    return;
  }
  std::vector<GraphArrays*> todo;
  {
    std::lock_guard<std::mutex> g(*g_reclaim_mutex);
    todo.swap(*g_reclaim);
    g_reclaim_n.store(0, std::memory_order_relaxed);
  }
  // another thread may be capturing in global mode: device_free's relaxed
  // mode allows these frees (the graphs that used them are gone)
  for (GraphArrays* a : todo) {
    device_free(a->device, a->ptrs);
    delete a;
  }
}

hipError_t
stream_state(hipStream_t stream, std::shared_ptr<StreamState>* out)
{
  int dev = 0;
  const hipError_t e = stream_device(stream, &dev);
  if (e != hipSuccess) {
    return e;
  }
  if (g_reclaim_n.load(std::memory_order_relaxed) != 0 && !stream_capturing(stream)) {
    reclaim_graph_arrays();
  }
  std::lock_guard<std::mutex> g(g_mutex);
  std::shared_ptr<StreamState>& s = g_states[std::make_pair(dev, stream)];
  if (!s) {
    s = std::make_shared<StreamState>();
    s->device = dev;
    s->stream = stream;
  }
  *out = s;
  return hipSuccess;
}

bool
stream_capturing(hipStream_t stream)
{
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return cs != hipStreamCaptureStatusNone;
}

hipError_t
capture_record(StreamState& s, StreamState::Capture** out)
{
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t graph = nullptr;
  if (hipStreamGetCaptureInfo_v2(s.stream, &cs, &id, &graph, nullptr, nullptr) != hipSuccess ||
      cs != hipStreamCaptureStatusActive || !graph) {
    (void)hipGetLastError();
    return hipErrorStreamCaptureUnsupported;
  }
  if (!s.cap.live || s.cap.id != id) {
    // the first call of this capture on this stream: the arrays of an
    // earlier capture stay with that capture's graph
    s.cap = StreamState::Capture();
    s.cap.live = true;
    s.cap.id = id;
    GraphArrays* owner = new GraphArrays;
    owner->device = s.device;
    hipUserObject_t obj = nullptr;
    if (hipUserObjectCreate(&obj, owner, on_graph_destroyed, 1,
                            hipUserObjectNoDestructorSync) != hipSuccess) {
      (void)hipGetLastError();
      delete owner;
      owner = nullptr;
    } else if (hipGraphRetainUserObject(graph, obj, 1, hipGraphUserObjectMove) != hipSuccess) {
      (void)hipGetLastError();
      // our reference is still ours: dropping it runs the destructor, which
      // queues the (empty) record for the next reclaim
      (void)hipUserObjectRelease(obj, 1);
      owner = nullptr;
    }
    s.cap.owner = owner;
    s.span_salt = s.span_salt * 0x9E3779B1u + 0x7F4A7C15u;
    s.cap.salt = s.span_salt;
  }
  *out = &s.cap;
  return hipSuccess;
}

void
capture_keep(StreamState& s, const std::vector<void*>& ps)
{
  std::vector<void*>& to = s.cap.owner ? s.cap.owner->ptrs : s.orphans;
  to.insert(to.end(), ps.begin(), ps.end());
}

hipError_t
call_shards(StreamState& s, bool capturing, uint32_t** out)
{
  if (capturing) {
    // shards of the capture's own, zeroed by a kernel node of the graph
    StreamState::Capture* c = nullptr;
    uint64_t* words = nullptr;
    if (capture_record(s, &c) != hipSuccess ||
        zeroed_words(s, SHARD_BYTES / 8, true, &words) != hipSuccess) {
      (void)hipGetLastError();
      return hipErrorStreamCaptureUnsupported;
    }
    *out = reinterpret_cast<uint32_t*>(words);
    return hipSuccess;
  }
  if (!s.shards) {
    void* p = nullptr;
    hipError_t e = device_malloc(s.device, &p, SHARD_BYTES);
    if (e == hipSuccess && (e = hipMemsetAsync(p, 0, SHARD_BYTES, s.stream)) != hipSuccess) {
      device_free(s.device, std::vector<void*>{ p });
    }
    if (e != hipSuccess) {
      return e;
    }
    s.shards = static_cast<uint32_t*>(p);
  }
  *out = s.shards;
  return hipSuccess;
}

hipError_t
span_slots(StreamState& s, bool capturing, uint64_t need, uint64_t** out, uint64_t* nslots,
           uint32_t* salt)
{
  if (!capturing) {
    if (need > s.span_nslots) {
      const uint64_t want = need < 4096 ? 4096 : need;
      uint64_t* made = nullptr;
      hipError_t e = zeroed_words(s, want, false, &made);
      if (e == hipSuccess && (e = sync_stream(s.stream)) != hipSuccess) {
        device_free(s.device, std::vector<void*>{ made });
      }
      if (e != hipSuccess) {
        return e;
      }
      device_free(s.device, std::vector<void*>{ s.span_slots }); // idle: the stream synchronised
      s.span_slots = made;
      s.span_nslots = want;
    }
    // words keep the tags of earlier launches (span_kernel.h): zeroed every
    // 2^20 direct calls, so no word outlives that many calls of this stream
    // (a tag only repeats after 2^40 dispatches on the stream's queue)
    if ((++s.span_calls & ((1u << 20) - 1)) == 0) {
      const hipError_t e = hipMemsetAsync(s.span_slots, 0, s.span_nslots * 8, s.stream);
      if (e != hipSuccess) {
        return e;
      }
    }
    *out = s.span_slots;
    *nslots = s.span_nslots;
    *salt = 0;
    return hipSuccess;
  }
  StreamState::Capture* c = nullptr;
  if (capture_record(s, &c) != hipSuccess) {
    return hipErrorStreamCaptureUnsupported;
  }
  if (c->nwords < need) {
    // a graph may be replayed on other streams (other hardware queues, whose
    // dispatch ids overlap this one's): the kernel's tag adds a hash of the
    // queue (span_kernel.h launch_tag), and a salt per captured array sets
    // its tags apart from every other array's as well. A larger array made
    // later in the same capture replaces this one for the calls after it
    // (the graph keeps both).
    const uint64_t size = need < 4096 ? 4096 : need;
    uint64_t* words = nullptr;
    if (zeroed_words(s, size, true, &words) != hipSuccess) {
      (void)hipGetLastError();
      return hipErrorStreamCaptureUnsupported;
    }
    c->words = words;
    c->nwords = size;
  }
  *out = c->words;
  *nslots = c->nwords;
  *salt = c->salt;
  return hipSuccess;
}

void
drop_shards(StreamState& s, uint32_t* shards)
{
  if (shards == s.shards) {
    s.retired.push_back(s.shards);
    s.shards = nullptr; // the next call makes fresh ones
  }
}

} // namespace tulips_amd

extern "C" int
tulips_csum_release_stream(void* stream)
{
  using namespace tulips_amd;
  hipStream_t st = static_cast<hipStream_t>(stream);
  std::vector<std::shared_ptr<StreamState>> gone;
  {
    std::lock_guard<std::mutex> g(g_mutex);
    for (auto it = g_states.begin(); it != g_states.end();) {
      if (it->first.second == st) {
        gone.push_back(it->second);
        it = g_states.erase(it);
      } else {
        ++it;
      }
    }
  }
  for (auto& s : gone) {
    std::lock_guard<std::recursive_mutex> g(s->call); // no call of this stream in flight
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(s->device);
    if (sync_stream(st) != hipSuccess) {
      (void)hipGetLastError();
    }
    (void)hipSetDevice(prev);
    // the stream's direct arrays; those of its captures belong to their
    // graphs (freed when the graphs are gone), except orphans
    std::vector<void*> ps;
    ps.push_back(s->shards);
    for (auto* p : s->retired) ps.push_back(p);
    ps.push_back(s->seg.blocks);
    ps.push_back(s->seg.runs);
    ps.push_back(s->seg.desc);
    ps.push_back(s->span_slots);
    for (auto* p : s->orphans) ps.push_back(p);
    device_free(s->device, ps);
    s->shards = nullptr;
    s->retired.clear();
    s->seg = StreamState::SegWs();
    s->span_slots = nullptr;
    s->span_nslots = 0;
    s->orphans.clear();
    s->cap = StreamState::Capture();
  }
  if (g_reclaim_n.load(std::memory_order_relaxed) != 0 && !stream_capturing(st)) {
    reclaim_graph_arrays();
  }
  return TULIPS_STATUS_OK;
}
