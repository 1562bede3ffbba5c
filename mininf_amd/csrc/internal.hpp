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

// Timing events around a site kernel (the `start_event` / `stop_event` arguments) are for eager
// launches only. Round 5 first recorded them under capture with hipEventRecordWithFlags(...,
// hipEventRecordExternal) (commit c13b392): on this stack that call returns hipErrorInvalidValue
// inside a capture, which invalidates the whole capture sequence, so the draw launched next
// (mi_normal_rsample_exp) failed with the same code (gpurun_out/dbg1_one.err). Replayed kernels
// are timed by span stamps instead (mi_group.stamps / mi_linear.stamps). An entry point given
// events while `stream` is capturing returns MI_EUNSUPPORTED before it enqueues anything, so the
// capture stays valid.
inline hipError_t mi_stream_capturing(hipStream_t stream, bool* capturing) {
  hipStreamCaptureStatus status = hipStreamCaptureStatusNone;
  const hipError_t e = hipStreamIsCapturing(stream, &status);
  *capturing = status != hipStreamCaptureStatusNone;
  return e;
}

inline hipError_t mi_record_event(void* event, hipStream_t stream) {
  return hipEventRecord(static_cast<hipEvent_t>(event), stream);
}
