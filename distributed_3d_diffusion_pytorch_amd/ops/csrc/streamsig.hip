// Cross-stream signals out of a replayed HIP graph (engine/graphs.py,
// comm_mode "event"): an EXTERNAL event-record node captured into graph A at
// the point where a gradient bucket is complete, and an ordinary stream wait
// on that event after each replay, so the bucket's all-reduce -- issued
// eagerly on a comm stream -- overlaps the backward kernels the replay still
// runs for the layers below it.  (torch's Event(external=True) is refused on
// ROCm builds; the HIP API itself has hipEventRecordExternal, so the runtime
// calls are made here.  A probe checks the ordering on the box before the
// graph step relies on it.)
#include "common.h"

D3D_API void* d3d_event_create() {
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  return (void*)e;
}

D3D_API int d3d_event_destroy(void* e) { return e ? (int)hipEventDestroy((hipEvent_t)e) : 0; }

// Inside a stream capture: an external event-record node (the replay records
// the event when it reaches this point); outside: a plain record.
D3D_API int d3d_event_record_external(void* e, hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return -1;
  if (cs == hipStreamCaptureStatusActive) return (int)hipEventRecordWithFlags((hipEvent_t)e, st, hipEventRecordExternal);
  return (int)hipEventRecord((hipEvent_t)e, st);
}

D3D_API int d3d_stream_wait_event(hipStream_t st, void* e) { return (int)hipStreamWaitEvent(st, (hipEvent_t)e, 0); }
