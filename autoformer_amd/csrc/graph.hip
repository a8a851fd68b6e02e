// graph.hip — host-side helpers of the step's stream plumbing.
//
// (Round 3 also built a main / side split of the captured step here -- two hipGraphs replayed
// concurrently on the main and weight-gradient streams.  It replayed correctly once and produced
// NaN from the second replay on in every arrangement measured, including with the side graph
// skipped (profiles/r3_graph_split.txt); the cause was not found and round 4 removed it.  A
// captured step is one hipGraph: train.TrainStep.capture.)
#include "common.h"

#define GCHK(x, what)                                                    \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      avc_set_error("%s: %s (%s)", what, hipGetErrorString(e_), #x);      \
      return -1;                                                         \
    }                                                                    \
  } while (0)

// ---------------------------------------------------------------- host-side event helpers
// Cross-stream ordering of the step (weight-gradient side stream, pack prefetch) with raw HIP
// events on raw stream handles: torch.cuda.Event / current_stream() cost ~10-15 us of Python
// per use, ~1 ms per AutoVC step at ~90 uses.  Events are created once (a ring on the Python
// side) and re-recorded; hipStreamWaitEvent waits for the record current at the time of the call.
extern "C" int avc_event_create(void** out) {
  AVC_CHECK_ARG(out, "avc_event_create: null");
  hipEvent_t e = nullptr;
  GCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming), "avc_event_create");
  *out = e;
  return 0;
}

extern "C" int avc_event_record(void* ev, void* stream) {
  AVC_CHECK_ARG(ev, "avc_event_record: null event");
  GCHK(hipEventRecord(reinterpret_cast<hipEvent_t>(ev), as_stream(stream)), "avc_event_record");
  return 0;
}

extern "C" int avc_stream_wait_event(void* stream, void* ev) {
  AVC_CHECK_ARG(ev, "avc_stream_wait_event: null event");
  GCHK(hipStreamWaitEvent(as_stream(stream), reinterpret_cast<hipEvent_t>(ev), 0), "avc_stream_wait_event");
  return 0;
}
