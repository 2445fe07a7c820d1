// stream_state.h — the library's per-(device, stream) state: counter shards
// for the counting calls (verify, counted frame validation), the split-form
// span words of the arena calls and the segmentation workspace.
//
// Rules (include/tulips_csum.h):
//  * A call that uses the state holds the stream's `call` mutex from its
//    first launch through its last, so two host threads issuing counting or
//    segmentation calls on the same stream (e.g. the legacy NULL stream) get
//    their launches queued as whole sequences, never interleaved.
//  * The device is the stream's own (hipStreamGetDevice), not the calling
//    thread's current device; state is allocated on that device.
//  * Direct (uncaptured) calls share the stream's arrays, grown on demand;
//    tulips_csum_release_stream frees them.
//  * A call captured in a HIP graph runs on arrays made for that capture (in
//    relaxed capture mode; zeroed by a kernel node of the graph where they
//    must start at zero). The graph owns them through a HIP user object
//    (hipUserObjectCreate + hipGraphRetainUserObject, moved to the graph):
//    instantiated executables hold their own references, and when the last
//    of the graph and its executables is destroyed the runtime calls the
//    object's destructor. That only queues the arrays; the library's next
//    uncaptured call on any stream (or tulips_csum_release_stream) frees
//    them (reclaim_graph_arrays), so no HIP call runs inside the runtime's
//    callback. Nothing a direct call does can free or reuse them while a
//    graph may still replay.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <mutex>
#include <vector>

namespace tulips_amd {

// The arrays one capture took on one stream; owned by the graph through a
// user object whose destructor queues this for reclaim_graph_arrays.
struct GraphArrays
{
  int device = 0;
  std::vector<void*> ptrs;
};

struct StreamState
{
  int device = 0;
  hipStream_t stream = nullptr;
  // held across one call's launch sequence (recursive: a counting call
  // holds it around launches that take it themselves, e.g. the split span)
  std::recursive_mutex call;

  // counter shards (csum_launch.h CNT_SHARDS x CNT_LINE words) of the
  // direct calls, and sets dropped after a failed launch (freed at release)
  uint32_t* shards = nullptr;
  std::vector<uint32_t*> retired;

  // segmentation workspace (segment.hip): the scan's block totals, the run
  // starts and the per-frame descriptors
  struct SegWs
  {
    uint32_t* blocks = nullptr;
    uint32_t* runs = nullptr;
    uint64_t nruns = 0;
    void* desc = nullptr; // 16 B per input frame
    uint64_t ndesc = 0;
  };
  // direct calls: grown on demand, the old arrays freed once the stream is
  // idle (no graph ever holds them)
  SegWs seg;

  // SPAN split-form words (span_kernel.h csum_span_kernel): one 64-bit word
  // per arena range, tagged with the launch's dispatch id and queue, so a
  // word left by an earlier launch is never added to. Direct calls share
  // `span_slots`, re-zeroed every 2^20 calls.
  uint64_t* span_slots = nullptr;
  uint64_t span_nslots = 0;
  uint64_t span_calls = 0;
  uint32_t span_salt = 0; // advanced per captured word array

  // The capture in progress on this stream (the last one seen): its calls
  // share one word array and one segmentation workspace (they run in order
  // in the graph); every array it takes goes to `owner`, the graph's.
  struct Capture
  {
    bool live = false;
    unsigned long long id = 0;
    GraphArrays* owner = nullptr; // null when the runtime refused the user object
    uint64_t* words = nullptr;
    uint64_t nwords = 0;
    uint32_t salt = 0;
    SegWs seg;
  };
  Capture cap;
  // arrays of captures whose graph could not take ownership (a runtime
  // without user objects): freed at tulips_csum_release_stream
  std::vector<void*> orphans;
};

// The state of `stream` (created on first use). The returned pointer stays
// valid while held even if the stream is released meanwhile. When `stream`
// is not capturing, first frees the arrays of graphs destroyed since the
// last call (reclaim_graph_arrays).
hipError_t stream_state(hipStream_t stream, std::shared_ptr<StreamState>* out);

// Frees the arrays of every graph whose last reference the runtime dropped
// (queued by the user objects' destructors). Must not run inside a capture
// on the calling thread's stream; the thread's capture mode is relaxed
// around the frees.
void reclaim_graph_arrays();

// Whether `stream` is capturing (a stream that cannot be queried counts as
// not capturing; the launches will report the error).
bool stream_capturing(hipStream_t stream);

// The record of the capture in progress on s.stream (caller holds s.call),
// made on the capture's first call on this stream: a fresh word array and
// workspace slot, and a user object moved to the capture's graph.
// hipErrorStreamCaptureUnsupported when the capture cannot be read.
hipError_t capture_record(StreamState& s, StreamState::Capture** out);

// Hands arrays made for the capture in progress to its graph (or to
// s.orphans when the graph holds no user object of ours).
void capture_keep(StreamState& s, const std::vector<void*>& ps);

// Counter shards for one counting call on `s` (caller holds s.call): the
// stream's direct shards, or, inside a capture, a zeroed set of the graph's.
// hipErrorStreamCaptureUnsupported when a capture's set cannot be made.
hipError_t call_shards(StreamState& s, bool capturing, uint32_t** out);

// The split-form span words for one call on `s` (caller holds s.call):
// at least `need` words (their count in *nslots) and the array's tag salt;
// inside a capture the capture's array (the graph's).
// hipErrorStreamCaptureUnsupported when a capture's array cannot be had.
hipError_t span_slots(StreamState& s, bool capturing, uint64_t need, uint64_t** out,
                      uint64_t* nslots, uint32_t* salt);

// After a failed launch in a direct counting call: the shards may hold
// partial sums, so the stream gets fresh zeroed ones on its next call.
void drop_shards(StreamState& s, uint32_t* shards);

// hipMalloc / hipFree on `device` (restoring the caller's current device),
// with the thread's capture mode relaxed around them: inside a capture the
// allocation is the graph's (capture_keep), and outside one it must not be
// refused, nor break the capture, because ANOTHER thread is capturing in
// global mode (torch.cuda.graph's default) — what the library allocates or
// frees is never used by that capture.
hipError_t device_malloc(int device, void** p, size_t bytes);
void device_free(int device, const std::vector<void*>& ps);

// hipStreamSynchronize, in relaxed capture mode for the same reason: on both
// runtimes a global-mode sync (like a global-mode hipMalloc / hipFree) from
// one thread invalidates another thread's global-mode capture
// (tools/probe_capture_modes.py, profiles/capture_modes_r06o.jsonl).
hipError_t sync_stream(hipStream_t stream);

} // namespace tulips_amd
