// Graph-external events: an event-record NODE inside a captured graph that a
// stream outside the graph can wait on after the replay is launched (and a
// wait node that waits for an event recorded outside).  PyTorch's ROCm build
// refuses torch.cuda.Event(external=True); hipEventRecordWithFlags(...,
// hipEventRecordExternal) returns hipErrorInvalidValue under capture on this
// ROCm, so the node is inserted into the capturing graph directly:
// hipStreamGetCaptureInfo_v2 -> hipGraphAddEventRecordNode on the current
// dependency set -> hipStreamUpdateCaptureDependencies(set = the new node).
// Used to start each gradient bucket's all-reduce as soon as the replayed
// backward has written it (parallel/grad_reducer.py, DIST.GRAPH_COMM=events)
// and by the two-graph backward (RUNTIME.WGRAD_XGRAPH) -- both validated by
// scripts/graph_external_event_probe.py before use.
#include "common.h"

MDA_API int mda_event_create(void** ev) {
  return (int)hipEventCreateWithFlags((hipEvent_t*)ev, hipEventDisableTiming);
}

MDA_API int mda_event_destroy(void* ev) { return (int)hipEventDestroy((hipEvent_t)ev); }

namespace {
// add `node` after the capture's current dependencies; it becomes the new set
int capture_node(hipStream_t st, bool record, hipEvent_t ev) {
  hipStreamCaptureStatus status;
  unsigned long long id = 0;
  hipGraph_t graph = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t ndeps = 0;
  hipError_t e = hipStreamGetCaptureInfo_v2(st, &status, &id, &graph, &deps, &ndeps);
  if (e != hipSuccess) return (int)e;
  if (status != hipStreamCaptureStatusActive) return -10 - (int)status;  // -10 none, -12 invalidated
  hipGraphNode_t node;
  e = record ? hipGraphAddEventRecordNode(&node, graph, deps, ndeps, ev)
             : hipGraphAddEventWaitNode(&node, graph, deps, ndeps, ev);
  if (e != hipSuccess) return (int)e;
  return (int)hipStreamUpdateCaptureDependencies(st, &node, 1, hipStreamSetCaptureDependencies);
}
}  // namespace

// mode 0: plain record; 1: hipEventRecordExternal flag; 2: explicit graph node
// (the stream must be capturing)
MDA_API int mda_event_record(void* ev, int64_t mode, hipStream_t st) {
  if (mode == 2) return capture_node(st, true, (hipEvent_t)ev);
  return (int)hipEventRecordWithFlags((hipEvent_t)ev, st,
                                      mode == 1 ? hipEventRecordExternal : hipEventRecordDefault);
}

MDA_API int mda_stream_wait_event(void* ev, int64_t mode, hipStream_t st) {
  if (mode == 2) return capture_node(st, false, (hipEvent_t)ev);
  return (int)hipStreamWaitEvent(st, (hipEvent_t)ev, mode == 1 ? hipEventWaitExternal : 0);
}

// Diagnostics: the shader clock at this point of a stream.  One wave reads
// the core-clock counter (s_memtime) and the constant 100 MHz counter
// (s_memrealtime) before and after a ~2 us spin and stores the ratio as MHz
// into out[slot] (a float vector store).  scripts/replay_ramp.py puts one at
// every step boundary of a timed window to see whether the first steps after
// an idle GPU run at a lower clock.
namespace {
__global__ void clock_probe_kernel(float* out, int slot) {
  if (threadIdx.x != 0) return;
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  uint64_t r1 = r0, c1 = c0;
  while (r1 - r0 < 200) {  // 2 us of the 100 MHz clock
    r1 = __builtin_amdgcn_s_memrealtime();
    c1 = __builtin_amdgcn_s_memtime();
  }
  out[slot] = (float)((double)(c1 - c0) * 100.0 / (double)(r1 - r0));
}
}  // namespace

MDA_API int mda_clock_probe(float* out, int64_t slot, hipStream_t st) {
  hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, st, out, (int)slot);
  return (int)hipGetLastError();
}
