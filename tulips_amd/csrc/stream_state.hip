// stream_state.hip — per-(device, stream) state registry (stream_state.h)
// and tulips_csum_release_stream.
#include <hip/hip_runtime.h>
#include <stdint.h>

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

constexpr size_t SHARD_BYTES = sizeof(uint32_t) * CNT_LINE * CNT_SHARDS;
static_assert(SHARD_BYTES % 8 == 0, "shards are made as 64-bit words");

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

void
free_on(int device, const std::vector<void*>& ps)
{
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  for (void* p : ps) {
    if (p) {
      (void)hipFree(p);
    }
  }
  (void)hipSetDevice(prev);
}

} // namespace

hipError_t
device_malloc(int device, void** p, size_t bytes)
{
  int prev = 0;
  hipError_t e = hipGetDevice(&prev);
  if (e != hipSuccess) {
    return e;
  }
  if (prev != device && (e = hipSetDevice(device)) != hipSuccess) {
    return e;
  }
  *p = nullptr;
  e = hipMalloc(p, bytes);
  if (prev != device) {
    (void)hipSetDevice(prev);
  }
  return e;
}

hipError_t
device_malloc_in_capture(int device, bool capturing, void** p, size_t bytes)
{
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  if (capturing) {
    (void)hipThreadExchangeStreamCaptureMode(&mode);
  }
  const hipError_t e = device_malloc(device, p, bytes);
  if (capturing) {
    (void)hipThreadExchangeStreamCaptureMode(&mode);
  }
  return e;
}

bool
capture_id(hipStream_t stream, unsigned long long* id)
{
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamGetCaptureInfo(stream, &cs, id) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return cs == hipStreamCaptureStatusActive;
}

hipError_t
stream_state(hipStream_t stream, std::shared_ptr<StreamState>* out)
{
  int dev = 0;
  const hipError_t e = stream_device(stream, &dev);
  if (e != hipSuccess) {
    return e;
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

hipError_t zeroed_words(int device, uint64_t words, bool capturing, int count,
                        hipStream_t stream, std::vector<uint64_t*>* out);

hipError_t
call_shards(StreamState& s, bool capturing, uint32_t** out)
{
  if (capturing && (!s.shards || s.spare.empty())) {
    // a capture on a stream with no spare left (or none made yet: no direct
    // counting call before it): shards of its own, made in relaxed capture
    // mode and zeroed by a kernel node of the graph, owned by the graph
    std::vector<uint64_t*> made;
    const hipError_t e = zeroed_words(s.device, SHARD_BYTES / 8, true, 1, s.stream, &made);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return hipErrorStreamCaptureUnsupported;
    }
    *out = reinterpret_cast<uint32_t*>(made[0]);
    s.graph_owned.push_back(*out);
    return hipSuccess;
  }
  if (!s.shards) {
    // direct shards plus the spares captured calls will take, one
    // allocation each, zeroed in stream order before any kernel uses them
    std::vector<uint32_t*> made;
    hipError_t e = hipSuccess;
    for (int k = 0; k <= SPARE_SHARDS && e == hipSuccess; ++k) {
      void* p = nullptr;
      if ((e = device_malloc(s.device, &p, SHARD_BYTES)) == hipSuccess) {
        made.push_back(static_cast<uint32_t*>(p));
        e = hipMemsetAsync(p, 0, SHARD_BYTES, s.stream);
      }
    }
    if (e != hipSuccess) {
      free_on(s.device, std::vector<void*>(made.begin(), made.end()));
      return e;
    }
    s.shards = made[0];
    s.spare.assign(made.begin() + 1, made.end());
  }
  if (!capturing) {
    *out = s.shards;
    return hipSuccess;
  }
  *out = s.spare.back();
  s.spare.pop_back();
  s.graph_owned.push_back(*out);
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

// `count` arrays of zeroed words on `device`, zeroed in `stream`'s order:
// outside a capture the caller synchronises `stream` before anything else
// can read them; inside a capture (the thread's capture mode relaxed for the
// allocations, so hipMalloc is allowed) the zeroing is a kernel node of the
// graph on the capturing stream, run before the captured kernels at every
// replay. No stream is created or destroyed while a capture is in progress:
// doing that (a private zeroing stream, as before) corrupted the HIP
// runtime's graph state, and a later hipGraphLaunch crashed on it (the r04
// SIGSEGV; tests/test_fuzz.py::test_fuzz_captured_graphs).
hipError_t
zeroed_words(int device, uint64_t words, bool capturing, int count, hipStream_t stream,
             std::vector<uint64_t*>* out)
{
  std::vector<void*> made;
  hipError_t e = hipSuccess;
  {
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    if (capturing) {
      (void)hipThreadExchangeStreamCaptureMode(&mode);
    }
    for (int k = 0; k < count && e == hipSuccess; ++k) {
      void* p = nullptr;
      if ((e = device_malloc(device, &p, sizeof(uint64_t) * words)) == hipSuccess) {
        made.push_back(p);
      }
    }
    if (capturing) {
      (void)hipThreadExchangeStreamCaptureMode(&mode);
    }
  }
  for (void* p : made) {
    if (e == hipSuccess) {
      e = launch_zero_words(static_cast<uint64_t*>(p), words, stream);
    }
  }
  if (e != hipSuccess) {
    if (!capturing) {
      (void)hipStreamSynchronize(stream);
    }
    free_on(device, made);
    return e;
  }
  out->clear();
  for (void* p : made) {
    out->push_back(static_cast<uint64_t*>(p));
  }
  return hipSuccess;
}

hipError_t
span_slots(StreamState& s, bool capturing, uint64_t need, uint64_t** out, uint64_t* nslots,
           uint32_t* salt)
{
  if (!capturing) {
    if (need > s.span_nslots) {
      // direct words plus spares for captures, all zeroed before use
      const uint64_t want = need < 4096 ? 4096 : need;
      std::vector<uint64_t*> made;
      hipError_t e = zeroed_words(s.device, want, false, 1 + SPARE_SHARDS, s.stream, &made);
      if (e == hipSuccess) {
        e = hipStreamSynchronize(s.stream); // the old arrays are idle
      }
      if (e != hipSuccess) {
        free_on(s.device, std::vector<void*>(made.begin(), made.end()));
        return e;
      }
      std::vector<void*> old(s.span_spare.begin(), s.span_spare.end());
      old.push_back(s.span_slots);
      free_on(s.device, old);
      s.span_slots = made[0];
      s.span_nslots = want;
      s.span_spare.assign(made.begin() + 1, made.end());
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
  unsigned long long id = 0;
  if (!capture_id(s.stream, &id)) {
    return hipErrorStreamCaptureUnsupported;
  }
  // only the capture in progress on this stream can add calls to its array
  for (auto it = s.span_capture.begin(); it != s.span_capture.end();) {
    it = it->first == id ? std::next(it) : s.span_capture.erase(it);
  }
  auto it = s.span_capture.find(id);
  if (it != s.span_capture.end() && it->second.size >= need) {
    *out = it->second.words;
    *nslots = it->second.size;
    *salt = it->second.salt;
    return hipSuccess;
  }
  uint64_t* p = nullptr;
  uint64_t size = 0;
  if (!s.span_spare.empty() && s.span_nslots >= need) {
    p = s.span_spare.back();
    s.span_spare.pop_back();
    size = s.span_nslots;
  } else {
    size = need < 4096 ? 4096 : need;
    std::vector<uint64_t*> made;
    if (zeroed_words(s.device, size, true, 1, s.stream, &made) != hipSuccess) {
      (void)hipGetLastError();
      return hipErrorStreamCaptureUnsupported;
    }
    p = made[0];
  }
  s.span_owned.push_back(p);
  // a graph may be replayed on other streams (other hardware queues, whose
  // dispatch ids overlap this one's): the kernel's tag adds a hash of the
  // queue (span_kernel.h launch_tag), and a salt per captured array sets
  // its tags apart from every other array's as well
  s.span_salt = s.span_salt * 0x9E3779B1u + 0x7F4A7C15u;
  s.span_capture[id] = StreamState::Capture{ p, size, s.span_salt };
  *out = p;
  *nslots = size;
  *salt = s.span_salt;
  return hipSuccess;
}

void
drop_shards(StreamState& s, uint32_t* shards)
{
  if (shards == s.shards) {
    s.retired.push_back(s.shards);
    s.shards = nullptr; // the next call makes fresh ones (and fresh spares)
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
    if (hipStreamSynchronize(st) != hipSuccess) {
      (void)hipGetLastError();
    }
    (void)hipSetDevice(prev);
    std::vector<void*> ps;
    ps.push_back(s->shards);
    for (auto* p : s->spare) ps.push_back(p);
    for (auto* p : s->graph_owned) ps.push_back(p);
    for (auto* p : s->retired) ps.push_back(p);
    ps.push_back(s->seg.blocks);
    ps.push_back(s->seg.runs);
    ps.push_back(s->seg.desc);
    for (auto* p : s->seg_owned) ps.push_back(p);
    ps.push_back(s->span_slots);
    for (auto* p : s->span_spare) ps.push_back(p);
    for (auto* p : s->span_owned) ps.push_back(p);
    free_on(s->device, ps);
    s->shards = nullptr;
    s->spare.clear();
    s->graph_owned.clear();
    s->retired.clear();
    s->seg = StreamState::SegWs();
    s->seg_owned.clear();
    s->seg_capture.clear();
    s->span_slots = nullptr;
    s->span_nslots = 0;
    s->span_spare.clear();
    s->span_owned.clear();
    s->span_capture.clear();
  }
  return TULIPS_STATUS_OK;
}
