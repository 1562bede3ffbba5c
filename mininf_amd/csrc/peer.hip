// One-shot peer-write all-reduce for small buckets (the sharded step's gradient bucket
// of C2 / C4 is a few hundred bytes, where a ring collective's per-hop latency dominates): every
// rank writes its bucket straight into a slot of every peer's receive region (over xGMI, through
// the peers' memory mapped with IPC handles), raises a flag there, waits for the peers' flags in
// its own region and sums the slots in rank order. One kernel, no host involvement: capturable
// into the step's hipGraph like the RCCL call it replaces (distributed.GradientBucket).
//
// Region of each rank (mi_peer_region_bytes), written by the peers and read by its owner:
//   flags [2 parities][MI_PEER_MAX_RANKS] uint64 | slots [2][MI_PEER_MAX_RANKS][max_floats] float
//   | the owner's call counter (uint64)
// Call k (the counter + 1) uses parity k & 1: a rank can only start call k + 2 -- which reuses the
// parity -- after every peer raised its call-(k + 1) flag, i.e. after every peer finished reading
// the call-k slots. Flags carry the call number, so they are never reset.
//
// Coherence: the regions are fine-grained device memory; the data and flag stores and the flag
// and slot loads are system-scope (they bypass the non-coherent caches), the data stores are
// fenced before the flag store.
//
// Failure is loud and sticky. A missing peer ends the wait after a bounded number of polls; the
// kernel then ORs 1 into the caller's error word (pinned host memory: the host reads it without a
// synchronisation), writes NaN into `out` instead of a sum over stale slots, and does NOT advance
// the call counter. Every later call sees the error word at entry and does the same without
// touching any peer's region, so a failed rank never overwrites slots a late peer may still read;
// its peers in turn time out on their next call and fail the same way. The host raises at its next
// read of the word (PeerCommunicator.all_reduce before enqueuing, StepGraph's replay checks).
#include "common.hpp"
#include "internal.hpp"

#include <cstdint>

namespace mi {

constexpr int kPeerThreads = 256;
constexpr uint32_t kPeerPolls = 1u << 20;   // about a second of polling, then the error word

MI_DEV uint64_t* peer_flags(unsigned char* region, int parity) {
  return reinterpret_cast<uint64_t*>(region) + parity * MI_PEER_MAX_RANKS;
}
MI_DEV float* peer_slot(unsigned char* region, int64_t max_floats, int parity, int rank) {
  float* slots = reinterpret_cast<float*>(region + 2 * MI_PEER_MAX_RANKS * sizeof(uint64_t));
  return slots + ((int64_t)parity * MI_PEER_MAX_RANKS + rank) * max_floats;
}
MI_DEV uint64_t* peer_counter(unsigned char* region, int64_t max_floats) {
  return reinterpret_cast<uint64_t*>(peer_slot(region, max_floats, 2, 0));
}

MI_DEV void peer_poison(float* out, int64_t n) {
  for (int64_t i = threadIdx.x; i < n; i += kPeerThreads) out[i] = __builtin_nanf("");
}

__global__ __launch_bounds__(kPeerThreads) void k_peer_allreduce(const mi_peer P,
                                                                 const float* in,   // (may be out)
                                                                 float* out,
                                                                 int64_t n,
                                                                 uint32_t* __restrict__ error) {
  __shared__ int failed;
  // a failed communicator stays failed: no peer writes, no counter advance, a poisoned result
  if (__hip_atomic_load(error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
    peer_poison(out, n);
    return;
  }
  if (threadIdx.x == 0) failed = 0;
  unsigned char* own = static_cast<unsigned char*>(P.regions[P.rank]);
  uint64_t* counter = peer_counter(own, P.max_floats);
  const uint64_t call = __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1;
  const int parity = (int)(call & 1);
  // this rank's bucket into its slot of every peer's region
  for (int q = 0; q < P.world; ++q) {
    if (q == P.rank) continue;
    float* dst = peer_slot(static_cast<unsigned char*>(P.regions[q]), P.max_floats, parity, P.rank);
    for (int64_t i = threadIdx.x; i < n; i += kPeerThreads)
      __hip_atomic_store(dst + i, in[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __threadfence_system();
  __syncthreads();
  // then its flag in every peer's region (lane q: peer q), released after the data
  const int q = (int)threadIdx.x;
  if (q < P.world && q != P.rank)
    __hip_atomic_store(peer_flags(static_cast<unsigned char*>(P.regions[q]), parity) + P.rank,
                       call, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  // wait for every peer's flag in this rank's region (bounded)
  if (q < P.world && q != P.rank) {
    const uint64_t* f = peer_flags(own, parity) + q;
    uint32_t polls = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != call) {
      if (++polls == kPeerPolls) {
        failed = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (failed) {   // (uniform after the barrier)
    if (threadIdx.x == 0)
      __hip_atomic_fetch_or(error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    peer_poison(out, n);
    return;
  }
  // the sum in rank order (the caller's own bucket read from `in`)
  for (int64_t i = threadIdx.x; i < n; i += kPeerThreads) {
    float acc = 0.0f;
    for (int r = 0; r < P.world; ++r)
      acc += r == P.rank ? in[i]
                         : __hip_atomic_load(peer_slot(own, P.max_floats, parity, r) + i,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    out[i] = acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(counter, call, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace mi

namespace {
int to_code(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }
}  // namespace

extern "C" {

int mi_peer_region_bytes(int64_t max_floats, size_t* bytes) {
  if (bytes == nullptr || max_floats < 1 || max_floats > MI_PEER_MAX_FLOATS) return MI_EINVAL;
  *bytes = 2 * MI_PEER_MAX_RANKS * sizeof(uint64_t) +
           (size_t)2 * MI_PEER_MAX_RANKS * (size_t)max_floats * sizeof(float) + sizeof(uint64_t);
  return 0;
}

int mi_peer_alloc(size_t bytes, void** region, void* handle) {
  if (region == nullptr || handle == nullptr || bytes == 0) return MI_EINVAL;
  hipError_t e = hipExtMallocWithFlags(region, bytes, hipDeviceMallocFinegrained);
  if (e == hipSuccess) e = hipMemset(*region, 0, bytes);
  if (e == hipSuccess) e = hipIpcGetMemHandle(static_cast<hipIpcMemHandle_t*>(handle), *region);
  return to_code(e);
}

int mi_peer_open(const void* handle, void** region) {
  if (handle == nullptr || region == nullptr) return MI_EINVAL;
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  return to_code(hipIpcOpenMemHandle(region, h, hipIpcMemLazyEnablePeerAccess));
}

int mi_peer_close(void* region) { return to_code(hipIpcCloseMemHandle(region)); }

int mi_peer_free(void* region) { return to_code(hipFree(region)); }

int mi_peer_allreduce(const mi_peer* peer, const float* in, float* out, int64_t n,
                      uint32_t* error, void* stream) {
  if (peer == nullptr || in == nullptr || out == nullptr || error == nullptr || n < 0 ||
      n > peer->max_floats || peer->world < 1 || peer->world > MI_PEER_MAX_RANKS ||
      peer->rank < 0 || peer->rank >= peer->world)
    return MI_EINVAL;
  for (int q = 0; q < peer->world; ++q)
    if (peer->regions[q] == nullptr) return MI_EINVAL;
  hipLaunchKernelGGL(mi::k_peer_allreduce, dim3(1), dim3(mi::kPeerThreads), 0,
                     static_cast<hipStream_t>(stream), *peer, in, out, n, error);
  return to_code(hipGetLastError());
}

int mi_peer_call_count(const mi_peer* peer, uint64_t* count) {
  if (peer == nullptr || count == nullptr || peer->rank < 0 || peer->rank >= MI_PEER_MAX_RANKS ||
      peer->regions[peer->rank] == nullptr || peer->max_floats < 1)
    return MI_EINVAL;
  const uint64_t* counter = reinterpret_cast<const uint64_t*>(
      static_cast<const unsigned char*>(peer->regions[peer->rank]) +
      2 * MI_PEER_MAX_RANKS * sizeof(uint64_t) +
      (size_t)2 * MI_PEER_MAX_RANKS * (size_t)peer->max_floats * sizeof(float));
  return to_code(hipMemcpy(count, counter, sizeof(uint64_t), hipMemcpyDeviceToHost));
}

}  // extern "C"
