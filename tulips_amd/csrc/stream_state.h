// stream_state.h — the library's per-(device, stream) state: counter shards
// for the counting calls (verify, counted frame validation) and the
// segmentation workspace.
//
// Rules (include/tulips_csum.h):
//  * A call that uses the state holds the stream's `call` mutex from its
//    first launch through its last, so two host threads issuing counting or
//    segmentation calls on the same stream (e.g. the legacy NULL stream) get
//    their launches queued as whole sequences, never interleaved.
//  * The device is the stream's own (hipStreamGetDevice), not the calling
//    thread's current device; state is allocated on that device.
//  * A counting call captured in a HIP graph gets shards of its own, owned by
//    the graph from then on, so replays never share shards with direct calls
//    on the capture stream: a spare from the set made with the stream's
//    direct shards, or, when none is left (or no direct counting call came
//    first), shards made in relaxed capture mode and zeroed on a private
//    stream.
//  * Segmentation calls captured in a graph run on a workspace made for that
//    capture and owned by the graph (no warm-up needed, nothing a later
//    direct call does can free it under the graph).
//  * tulips_csum_release_stream frees everything a stream holds, including
//    the shards and workspaces owned by graphs captured on it (destroy those
//    graphs first).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <memory>
#include <mutex>
#include <vector>

namespace tulips_amd {

struct StreamState
{
  int device = 0;
  hipStream_t stream = nullptr;
  // held across one call's launch sequence (recursive: a counting call
  // holds it around launches that take it themselves, e.g. the split span)
  std::recursive_mutex call;

  // counter shards (csum_launch.h CNT_SHARDS x CNT_LINE words each)
  uint32_t* shards = nullptr;          // direct (uncaptured) calls
  std::vector<uint32_t*> spare;        // for captured calls, made with `shards`
  std::vector<uint32_t*> graph_owned;  // handed to captured calls
  std::vector<uint32_t*> retired;      // dropped after a failed launch

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
  // direct (uncaptured) calls: grown on demand, the old arrays freed once the
  // stream is idle (no graph ever holds them)
  SegWs seg;
  // a capture's calls on this stream share one workspace made for that
  // capture (relaxed capture mode), owned by its graph: later direct calls
  // never free or regrow it, and a replay never shares arrays with direct
  // calls on this stream or with another graph
  std::map<unsigned long long, SegWs> seg_capture;
  std::vector<void*> seg_owned;

  // SPAN split-form words (span_kernel.h csum_span_kernel): one 64-bit word
  // per arena range, tagged with the launch's dispatch id and queue, so a word left by
  // an earlier launch (two-part segments leave theirs as they are) is never
  // added to. The calls one
  // capture records on this stream run in order in the graph, so they share
  // one array (a spare, or made in relaxed capture mode), owned by the graph
  // from then on and salted apart from other arrays
  uint32_t span_salt = 0;
  uint64_t* span_slots = nullptr;
  uint64_t span_nslots = 0;
  uint64_t span_calls = 0; // direct arena calls (the words are re-zeroed every 2^20)
  std::vector<uint64_t*> span_spare;
  std::vector<uint64_t*> span_owned;
  struct Capture
  {
    uint64_t* words;
    uint64_t size;
    uint32_t salt;
  };
  std::map<unsigned long long, Capture> span_capture;
};

constexpr int SPARE_SHARDS = 16;

// The state of `stream` (created on first use). The returned pointer stays
// valid while held even if the stream is released meanwhile.
hipError_t stream_state(hipStream_t stream, std::shared_ptr<StreamState>* out);

// Whether `stream` is capturing (a stream that cannot be queried counts as
// not capturing; the launches will report the error).
bool stream_capturing(hipStream_t stream);

// Counter shards for one counting call on `s` (caller holds s.call):
// the stream's direct shards, or, inside a capture, a zeroed set the graph
// keeps (a spare, or made then). hipErrorStreamCaptureUnsupported when a
// capture's set cannot be made.
hipError_t call_shards(StreamState& s, bool capturing, uint32_t** out);

// The split-form span words for one call on `s` (caller holds s.call): at
// least `need` words (their count in *nslots) and the array's tag salt;
// inside a capture an array the graph keeps.
// hipErrorStreamCaptureUnsupported when a capture's array cannot be had.
hipError_t span_slots(StreamState& s, bool capturing, uint64_t need, uint64_t** out,
                      uint64_t* nslots, uint32_t* salt);

// After a failed launch in a direct counting call: the shards may hold
// partial sums, so the stream gets fresh zeroed ones on its next call.
void drop_shards(StreamState& s, uint32_t* shards);

// hipMalloc on `device` (restores the caller's current device).
hipError_t device_malloc(int device, void** p, size_t bytes);

// hipMalloc on `device` from inside a capture: the thread's capture mode is
// relaxed around the allocation (plain device_malloc when not capturing).
hipError_t device_malloc_in_capture(int device, bool capturing, void** p, size_t bytes);

// The id of the capture in progress on `stream` (false when none can be read).
bool capture_id(hipStream_t stream, unsigned long long* id);

} // namespace tulips_amd
