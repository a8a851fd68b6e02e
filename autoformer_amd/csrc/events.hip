// events.hip — host-side event helpers of the training step's stream plumbing.
//
// Cross-stream ordering of the step (weight-gradient side stream, optimizer / all-reduce comm stream,
// pack prefetch) with raw HIP events on raw stream handles: torch.cuda.Event / current_stream() cost
// ~10-15 us of Python per use, ~1 ms per AutoVC step at ~90 uses.  Events are created once (a ring on
// the Python side, layers.ev_record) and re-recorded; hipStreamWaitEvent waits for the record current
// at the time of the call.  A recorded step (replay.py) re-issues the same record / wait calls.
//
// The events carry no system-scope fence (the default flushes and invalidates the L2s for host
// visibility; the consumers here are kernels on the same GPU, for which the device-scope release is
// enough).
//
// Round 5 also rebuilt a captured step as main / side hipGraph segments here; both forms lost to the
// recorded replay (6.10-6.17 ms against 5.73, profiles/r5_graph_modes.txt) and were removed in round 6.
#include "common.h"

#define GCHK(x, what)                                                    \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      avc_set_error("%s: %s (%s)", what, hipGetErrorString(e_), #x);      \
      return -1;                                                         \
    }                                                                    \
  } while (0)

extern "C" int avc_event_create(void** out) {
  AVC_CHECK_ARG(out, "avc_event_create: null");
  hipEvent_t e = nullptr;
  GCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence), "avc_event_create");
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
