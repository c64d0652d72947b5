// HIP events for bench.py's live kernel timing (scdhip.ops.LaunchTimer).  Recorded on the stream a kernel is
// launched on; inside a stream capture (the training step graph, scdhip/graph.py) the record becomes an external
// event-record node of the graph (hipEventRecordExternal), so every replay re-stamps the event and the pair times
// that replay's launch.
#include "scd_common.h"

extern "C" int scd_event_create(void** ev) {
    if (!ev) return SCD_ERR_ARG;
    return (int)hipEventCreateWithFlags((hipEvent_t*)ev, hipEventDefault);
}

extern "C" int scd_event_destroy(void* ev) { return ev ? (int)hipEventDestroy((hipEvent_t)ev) : 0; }

extern "C" int scd_event_record(void* ev, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hipError_t e = hipStreamIsCapturing(st, &cs);
    if (e != hipSuccess) return (int)e;
    if (cs != hipStreamCaptureStatusActive) return (int)hipEventRecord((hipEvent_t)ev, st);
    if (hipEventRecordWithFlags((hipEvent_t)ev, st, hipEventRecordExternal) == hipSuccess) return 0;
    (void)hipGetLastError();
    // the same node added by hand: an event-record node after the stream's current capture frontier, which then
    // becomes the frontier (what an external record does)
    unsigned long long id = 0;
    hipGraph_t graph = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t ndeps = 0;
    e = hipStreamGetCaptureInfo_v2(st, &cs, &id, &graph, &deps, &ndeps);
    if (e != hipSuccess) return (int)e;
    hipGraphNode_t node;
    e = hipGraphAddEventRecordNode(&node, graph, deps, ndeps, (hipEvent_t)ev);
    if (e != hipSuccess) return (int)e;
    return (int)hipStreamUpdateCaptureDependencies(st, &node, 1, hipStreamSetCaptureDependencies);
}

extern "C" int scd_event_elapsed_ms(void* start, void* end, float* ms) {
    if (!ms) return SCD_ERR_ARG;
    hipError_t e = hipEventSynchronize((hipEvent_t)end);
    if (e != hipSuccess) return (int)e;
    return (int)hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end);
}
