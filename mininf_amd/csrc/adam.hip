// One-launch Adam step (mininf_amd.optim.Adam): the optimizer step of the reference's training
// loop (README.md:66-69, `optimizer.step()` of torch.optim.Adam) for every parameter of a step in
// a single kernel, including the step-count increment that torch's capturable fused Adam runs as
// a separate `_foreach_add_` launch.
//
// Arithmetic restated from torch's fused Adam (ATen/native/cuda/fused_adam_utils.cuh adam_math,
// ADAM_MODE::ORIGINAL, no AMSGrad): hyper-parameters in double, the moments and the parameter in
// float, bias corrections 1 - beta^step in double -- bit-identical to torch.optim.Adam(fused=True).
//
// Every block reads its tensor's step s and uses s + 1; the last block of the tensor to finish
// (completion count, two levels: groups of kGroup blocks, then the tensor) stores s + 1, so no
// block can read the advanced value.
//
// The bias corrections (two double pows, a few hundred dependent instructions) are computed once
// per tensor and step: the tensor's first block computes those of the next step while its loads
// are in flight and stores them in the counter words' cache (a slot per tensor and step parity,
// keyed by step and betas); the next launch's blocks read them instead of each computing them
// (tools/stream_probe.hip: the per-block pows cost 1.5 us of a 7 us update at 512 blocks, 5 us at
// 2048). A slot that does not match (first step, a loaded step count, changed betas) falls back to
// the pows -- the same function of the same inputs either way.
#include "adam_math.hpp"
#include "common.hpp"
#include "internal.hpp"

#include <algorithm>
#include <cstdlib>
#include <cmath>

namespace mi {

constexpr int kAdamThreads = 256;
constexpr int kAdamGroup = 32;

// counter words after the completion counters: [tensor][step parity] slots of kCoefWords
constexpr int kCoefWords = 8;   // step s + 1 (float), bc1, bc2_sqrt, -, beta1 (double), beta2
constexpr int kCoefOffset = MI_ADAM_MAX_TENSORS * (1 + kAdamGroup);
static_assert(kCoefOffset + MI_ADAM_MAX_TENSORS * 2 * kCoefWords <= MI_ADAM_COUNTER_WORDS,
              "counter words");

MI_DEV unsigned* coef_slot(unsigned* counters, int t, float s1) {
  return counters + kCoefOffset + (t * 2 + ((int)s1 & 1)) * kCoefWords;
}

struct AdamPlan {
  int first[MI_ADAM_MAX_TENSORS + 1];   // first block of each tensor
  int64_t chunk[MI_ADAM_MAX_TENSORS];   // elements per block
};

template <typename T, int N>
MI_DEV T pick_adam(const T (&arr)[N], int a) {
  T v = arr[0];
#pragma unroll
  for (int q = 1; q < N; ++q)
    if (a == q) v = arr[q];
  return v;
}

MI_DEV mi_adam_tensor tensor_at(const mi_adam& A, int t) { return adam_tensor_at(A, t); }

// NT: non-temporal 16-byte loads and stores (measured slower on C5: the launch uses plain ones)
typedef float f4v __attribute__((ext_vector_type(4)));
MI_DEV float4 ld(const float4* p, bool nt) {
  if (!nt) return *p;
  const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
MI_DEV void st(float4* p, const float4& v, bool nt) {
  if (!nt) {
    *p = v;
    return;
  }
  const f4v w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<f4v*>(p));
}

template <bool NT, int U>
__global__ __launch_bounds__(kAdamThreads) void k_adam_step(const mi_adam A, const AdamPlan P,
                                                             unsigned* __restrict__ counters,
                                                             int count) {
  int t = 0;
#pragma unroll
  for (int q = 1; q < MI_ADAM_MAX_TENSORS; ++q)
    if (q < A.num && (int)blockIdx.x >= P.first[q]) t = q;
  const mi_adam_tensor T = tensor_at(A, t);
  const int first = pick_adam(P.first, t);
  const int nblocks = pick_adam(P.first, t + 1) - first;
  const int64_t chunk = pick_adam(P.chunk, t);
  const int b = (int)blockIdx.x - first;

  const int64_t i0 = (int64_t)b * chunk;
  const int64_t i1 = min(T.numel, i0 + chunk);
  const bool vec = ((reinterpret_cast<uintptr_t>(T.param) | reinterpret_cast<uintptr_t>(T.grad) |
                     reinterpret_cast<uintptr_t>(T.exp_avg) |
                     reinterpret_cast<uintptr_t>(T.exp_avg_sq)) & 15) == 0;
  float4* __restrict__ param = reinterpret_cast<float4*>(T.param);
  const float4* __restrict__ grad = reinterpret_cast<const float4*>(T.grad);
  float4* __restrict__ exp_avg = reinterpret_cast<float4*>(T.exp_avg);
  float4* __restrict__ exp_avg_sq = reinterpret_cast<float4*>(T.exp_avg_sq);
  // U quads per lane per pass (16-byte accesses; chunk is a multiple of 4 * kAdamThreads, so a
  // lane's quads are whole except the tensor's last, partial one)
  constexpr int64_t kStride = 4 * kAdamThreads;
  float4 p[U], g[U], m[U], v[U];
  auto load_pass = [&](int64_t base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = base + u * kStride;
      if (e + 3 < i1) {
        const int64_t q = e >> 2;
        p[u] = ld(param + q, NT);
        g[u] = ld(grad + q, NT);
        m[u] = ld(exp_avg + q, NT);
        v[u] = ld(exp_avg_sq + q, NT);
      }
    }
  };
  int64_t i = i0 + 4 * (int64_t)threadIdx.x;
  // the first pass's loads go out before the bias corrections (two double pows, a few hundred
  // dependent instructions): without the barrier the compiler hoists them ahead of every load
  if (vec) load_pass(i);
  __builtin_amdgcn_sched_barrier(0);

  // bias corrections in double, then handed to the update as float (adam_math's opmath_t
  // parameters)
  const float s1 = *T.step + 1.0f;
  // The step advances once every workgroup of the tensor has read it: counted at the end
  // (count 1), or right after the read (count 2: the atomic's return is awaited only at the end,
  // behind this workgroup's own traffic); count 0 leaves the step alone (timing probes only).
  auto last_block = [&]() {
    unsigned* tc = counters + t * (1 + kAdamGroup);
    const int groups = (nblocks + kAdamGroup - 1) / kAdamGroup;
    bool done = true;
    if (groups > 1) {
      const int g = b / kAdamGroup;
      const unsigned in_group = (unsigned)min(kAdamGroup, nblocks - g * kAdamGroup);
      unsigned* gc = tc + 1 + g;
      done = atomicAdd(gc, 1u) == in_group - 1u;
      if (done) *gc = 0u;
    }
    if (done && atomicAdd(tc, 1u) == (unsigned)(groups > 1 ? groups : nblocks) - 1u) {
      *tc = 0u;
      return true;
    }
    return false;
  };
  bool started_last = false;
  if (count == 2) {
    // every wave's step read complete (lgkmcnt(0) only: the first pass's loads stay in flight),
    // then the barrier
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    if (threadIdx.x == 0) started_last = last_block();
  }
  // bias corrections: the cached ones of this step if the slot matches, else computed here
  // (adam_math.hpp: torch's fused Adam arithmetic either way)
  AdamCoef coef;
  {
    const unsigned* slot = coef_slot(counters, t, s1);
    const bool hit = __uint_as_float(slot[0]) == s1 &&
                     __hiloint2double(slot[5], slot[4]) == A.beta1 &&
                     __hiloint2double(slot[7], slot[6]) == A.beta2;
    if (hit) {
      coef.bc1 = __uint_as_float(slot[1]);
      coef.bc2_sqrt = __uint_as_float(slot[2]);
      coef.step_size = (float)(A.lr / (double)coef.bc1);
    } else {
      coef = adam_coef(A, s1);
    }
  }
  // the tensor's first block: the next step's corrections, into the other parity's slot (no block
  // of this launch reads it)
  if (b == 0 && threadIdx.x < 64) {
    const float s2 = s1 + 1.0f;
    const AdamCoef next = adam_coef(A, s2);
    if (threadIdx.x == 0) {
      unsigned* slot = coef_slot(counters, t, s2);
      slot[1] = __float_as_uint(next.bc1);
      slot[2] = __float_as_uint(next.bc2_sqrt);
      slot[4] = (unsigned)__double2loint(A.beta1);
      slot[5] = (unsigned)__double2hiint(A.beta1);
      slot[6] = (unsigned)__double2loint(A.beta2);
      slot[7] = (unsigned)__double2hiint(A.beta2);
      slot[0] = __float_as_uint(s2);
    }
  }
  auto update = [&](float& param, float grad, float& m, float& v) {
    adam_update(A, coef, param, grad, m, v);
  };
  auto step4 = [&](float4& p, const float4& g, float4& m, float4& v) {
    update(p.x, g.x, m.x, v.x);
    update(p.y, g.y, m.y, v.y);
    update(p.z, g.z, m.z, v.z);
    update(p.w, g.w, m.w, v.w);
  };
  if (vec) {
    for (; i + 3 < i1; i += U * kStride) {
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (i + u * kStride + 3 < i1) step4(p[u], g[u], m[u], v[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t e = i + u * kStride;
        if (e + 3 < i1) {
          const int64_t q = e >> 2;
          st(param + q, p[u], NT);
          st(exp_avg + q, m[u], NT);
          st(exp_avg_sq + q, v[u], NT);
        }
      }
      load_pass(i + U * kStride);
    }
  }
  // element by element: the partial last quad (its lane), or every element of an unaligned tensor
  const int64_t tail = i1 & ~int64_t{3};
  const bool owns_tail = tail < i1 && ((tail - i0) >> 2) % kAdamThreads == threadIdx.x;
  for (int64_t j = vec ? (owns_tail ? tail : i1) : i0 + threadIdx.x; j < i1;
       j += vec ? 1 : kAdamThreads) {
    float pe = T.param[j], me = T.exp_avg[j], ve = T.exp_avg_sq[j];
    update(pe, T.grad[j], me, ve);
    T.param[j] = pe;
    T.exp_avg[j] = me;
    T.exp_avg_sq[j] = ve;
  }

  if (count == 1) {
    __syncthreads();   // every thread of the block has read the step
    if (threadIdx.x == 0 && last_block()) *T.step = s1;
  } else if (count == 2 && threadIdx.x == 0 && started_last) {
    *T.step = s1;
  }
}

}  // namespace mi

namespace {

int to_code(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

}  // namespace

extern "C" {

int mi_adam_step(const mi_adam* adam, uint32_t* counters, void* stream) {
  if (adam == nullptr || counters == nullptr || adam->num < 1 ||
      adam->num > MI_ADAM_MAX_TENSORS)
    return MI_EINVAL;
  mi::AdamPlan P{};
  int64_t total = 0;
  for (int t = 0; t < adam->num; ++t) {
    const mi_adam_tensor& T = adam->tensors[t];
    if (T.param == nullptr || T.grad == nullptr || T.exp_avg == nullptr ||
        T.exp_avg_sq == nullptr || T.step == nullptr || T.numel < 1)
      return MI_EINVAL;
    total += T.numel;
  }
  // About 1024 workgroups over all tensors (C5's 2 x 1e6 parameters: 1024 of 2048 elements; with
  // per-block pows 500 of 4096 had run faster, 12.5 us against 17, profiles/r03_adam_sweep.log --
  // tools/stream_probe.hip without them: 7.0 us at 512, 6.6 at 1024, 6.7 at 2048); at least
  // 4 * kAdamThreads elements per workgroup and at most kAdamGroup^2 workgroups per tensor.
  constexpr int64_t target_blocks = 1024;
  constexpr int64_t min_chunk = 4 * mi::kAdamThreads;
  const int64_t even = (total + target_blocks - 1) / target_blocks;
  int blocks = 0;
  for (int t = 0; t < adam->num; ++t) {
    const mi_adam_tensor& T = adam->tensors[t];
    int64_t chunk = std::max({min_chunk, even,
                              (T.numel + mi::kAdamGroup * mi::kAdamGroup - 1) /
                                  (mi::kAdamGroup * mi::kAdamGroup)});
    chunk = (chunk + 4 * mi::kAdamThreads - 1) / (4 * mi::kAdamThreads) * (4 * mi::kAdamThreads);
    P.first[t] = blocks;
    P.chunk[t] = chunk;
    blocks += (int)((T.numel + chunk - 1) / chunk);
  }
  for (int t = adam->num; t <= MI_ADAM_MAX_TENSORS; ++t) P.first[t] = blocks;
  // the step counts are advanced by the first workgroup (12.5 us vs 14.2 us counting at the end,
  // C5; r03 sweeps also kept plain over non-temporal accesses and two quads per lane per pass)
  constexpr int count = 2;
  const dim3 grid((unsigned)blocks), block(mi::kAdamThreads);
  const hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL((mi::k_adam_step<false, 2>), grid, block, 0, s, *adam, P, counters, count);
  return to_code(hipGetLastError());
}

}  // extern "C"
