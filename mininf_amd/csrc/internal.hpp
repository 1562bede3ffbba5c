// Host-side helpers shared between the library's translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

// Fixed-order fp64 reduction of per-(segment, particle) partials part[v][nseg][K] (sites.hip
// k_finalize): values v < num_sites are multiplied by scale[v] and summed into total[k] (and
// written to site_lp[v*K + k] when non-NULL); the remaining num_slots values are multiplied by
// slot_scale and written to slot_grad[(v - num_sites)*K + k].
// With long segment lists (> 512) and a `scratch` of mi_finalize_scratch_bytes, the reduction
// runs in two launches (segment chunks in parallel, then the chunk sums); otherwise in one.
size_t mi_finalize_scratch_bytes(int64_t nseg, int64_t K, int nv);
// rank1: bit v marks value v as stored in mi_reduce's rank-one layout (one-launch path only).
int mi_launch_finalize(const float* part, int64_t nseg, int64_t K, int num_sites, int num_slots,
                       const double* scale, double slot_scale, float* total, double* site_lp,
                       float* slot_grad, double* scratch, hipStream_t stream, int rank1 = 0);

// Record a caller's timing event on `stream`. Under stream capture the record becomes an event
// record node of the graph, appended after the capture's current dependencies (every replay of
// the graph then records it, so a replayed kernel can be timed); otherwise a plain record.
inline hipError_t mi_record_event(void* event, hipStream_t stream) {
  hipStreamCaptureStatus status = hipStreamCaptureStatusNone;
  hipGraph_t graph = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t ndeps = 0;
  hipError_t e = hipStreamGetCaptureInfo_v2(stream, &status, nullptr, &graph, &deps, &ndeps);
  if (e != hipSuccess) return e;
  if (status != hipStreamCaptureStatusActive)
    return hipEventRecord(static_cast<hipEvent_t>(event), stream);
  hipGraphNode_t node = nullptr;
  e = hipGraphAddEventRecordNode(&node, graph, deps, ndeps, static_cast<hipEvent_t>(event));
  if (e != hipSuccess) return e;
  return hipStreamUpdateCaptureDependencies(stream, &node, 1, hipStreamSetCaptureDependencies);
}
