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
#include "common.hpp"
#include "internal.hpp"

#include <algorithm>
#include <cstdlib>
#include <cmath>

namespace mi {

constexpr int kAdamThreads = 256;
constexpr int kAdamGroup = 32;

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

MI_DEV mi_adam_tensor tensor_at(const mi_adam& A, int t) {
  switch (t) {
#define MI_ADAM_CASE(Q) case Q: return A.tensors[Q];
    MI_ADAM_CASE(1) MI_ADAM_CASE(2) MI_ADAM_CASE(3) MI_ADAM_CASE(4) MI_ADAM_CASE(5)
    MI_ADAM_CASE(6) MI_ADAM_CASE(7)
#undef MI_ADAM_CASE
    default: return A.tensors[0];
  }
}

__global__ __launch_bounds__(kAdamThreads) void k_adam_step(const mi_adam A, const AdamPlan P,
                                                             unsigned* __restrict__ counters) {
  int t = 0;
#pragma unroll
  for (int q = 1; q < MI_ADAM_MAX_TENSORS; ++q)
    if (q < A.num && (int)blockIdx.x >= P.first[q]) t = q;
  const mi_adam_tensor T = tensor_at(A, t);
  const int first = pick_adam(P.first, t);
  const int nblocks = pick_adam(P.first, t + 1) - first;
  const int64_t chunk = pick_adam(P.chunk, t);
  const int b = (int)blockIdx.x - first;

  // bias corrections in double, then handed to the update as float (adam_math's opmath_t
  // parameters)
  const float s1 = *T.step + 1.0f;
  const float bc1 = (float)(1.0 - pow(A.beta1, (double)s1));
  const float bc2_sqrt = (float)sqrt(1.0 - pow(A.beta2, (double)s1));
  const float step_size = (float)(A.lr / (double)bc1);
  const int64_t i0 = (int64_t)b * chunk;
  const int64_t i1 = min(T.numel, i0 + chunk);
  auto update = [&](float& param, float grad, float& m, float& v) {
    if (A.maximize) grad = -grad;
    // the contractions spelled out: fma(beta, moment, (1 - beta) * grad [* grad]), the form
    // torch's kernel compiles to (the compiler may pick another when left to itself)
    if (A.weight_decay != 0.0) grad = (float)fma((double)param, A.weight_decay, (double)grad);
    m = (float)fma(A.beta1, (double)m, (1.0 - A.beta1) * (double)grad);
    v = (float)fma(A.beta2, (double)v, ((1.0 - A.beta2) * (double)grad) * (double)grad);
    const float denom = (float)((double)(sqrtf(v) / bc2_sqrt) + A.eps);
    param -= step_size * m / denom;
  };
  const bool vec = ((reinterpret_cast<uintptr_t>(T.param) | reinterpret_cast<uintptr_t>(T.grad) |
                     reinterpret_cast<uintptr_t>(T.exp_avg) |
                     reinterpret_cast<uintptr_t>(T.exp_avg_sq)) & 15) == 0;
  int64_t i = i0 + 4 * (int64_t)threadIdx.x;
  if (vec) {   // 16-byte loads and stores (chunk is a multiple of 4 * kAdamThreads)
    float4* __restrict__ param = reinterpret_cast<float4*>(T.param);
    const float4* __restrict__ grad = reinterpret_cast<const float4*>(T.grad);
    float4* __restrict__ exp_avg = reinterpret_cast<float4*>(T.exp_avg);
    float4* __restrict__ exp_avg_sq = reinterpret_cast<float4*>(T.exp_avg_sq);
    auto step4 = [&](float4& p, const float4& g, float4& m, float4& v) {
      update(p.x, g.x, m.x, v.x);
      update(p.y, g.y, m.y, v.y);
      update(p.z, g.z, m.z, v.z);
      update(p.w, g.w, m.w, v.w);
    };
    // two quads per lane per pass: all eight 16-byte loads in flight before the first update
    constexpr int64_t kStride = 4 * kAdamThreads;
    for (; i + kStride + 3 < i1; i += 2 * kStride) {
      const int64_t q0 = i >> 2, q1 = (i + kStride) >> 2;
      float4 p0 = param[q0], p1 = param[q1];
      const float4 g0 = grad[q0], g1 = grad[q1];
      float4 m0 = exp_avg[q0], m1 = exp_avg[q1];
      float4 v0 = exp_avg_sq[q0], v1 = exp_avg_sq[q1];
      step4(p0, g0, m0, v0);
      step4(p1, g1, m1, v1);
      param[q0] = p0;
      param[q1] = p1;
      exp_avg[q0] = m0;
      exp_avg[q1] = m1;
      exp_avg_sq[q0] = v0;
      exp_avg_sq[q1] = v1;
    }
    for (; i + 3 < i1; i += kStride) {
      const int64_t q = i >> 2;
      float4 p = param[q];
      const float4 g = grad[q];
      float4 m = exp_avg[q], v = exp_avg_sq[q];
      step4(p, g, m, v);
      param[q] = p;
      exp_avg[q] = m;
      exp_avg_sq[q] = v;
    }
  }
  // the rest (the tail, or unaligned tensors) element by element
  for (int64_t j = (vec ? i : i0 + threadIdx.x); j < i1; j += vec ? 1 : kAdamThreads) {
    if (vec && j >= i + 4) break;
    float p = T.param[j], m = T.exp_avg[j], v = T.exp_avg_sq[j];
    update(p, T.grad[j], m, v);
    T.param[j] = p;
    T.exp_avg[j] = m;
    T.exp_avg_sq[j] = v;
  }

  __syncthreads();   // every thread of the block has read the step
  if (threadIdx.x == 0) {
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
      *T.step = s1;
    }
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
  int blocks = 0;
  for (int t = 0; t < adam->num; ++t) {
    const mi_adam_tensor& T = adam->tensors[t];
    if (T.param == nullptr || T.grad == nullptr || T.exp_avg == nullptr ||
        T.exp_avg_sq == nullptr || T.step == nullptr || T.numel < 1)
      return MI_EINVAL;
    // at most kAdamGroup^2 blocks per tensor, 8 elements per thread at least
    static const int64_t min_chunk = [] {   // elements per block at least (MININF_AMD_ADAM_CHUNK)
      const char* v = std::getenv("MININF_AMD_ADAM_CHUNK");
      const int64_t n = v != nullptr ? std::atoll(v) : 8 * mi::kAdamThreads;
      return std::max<int64_t>(4 * mi::kAdamThreads, n);
    }();
    int64_t chunk = std::max<int64_t>(min_chunk,
                                      (T.numel + mi::kAdamGroup * mi::kAdamGroup - 1) /
                                          (mi::kAdamGroup * mi::kAdamGroup));
    chunk = (chunk + 4 * mi::kAdamThreads - 1) / (4 * mi::kAdamThreads) * (4 * mi::kAdamThreads);
    P.first[t] = blocks;
    P.chunk[t] = chunk;
    blocks += (int)((T.numel + chunk - 1) / chunk);
  }
  for (int t = adam->num; t <= MI_ADAM_MAX_TENSORS; ++t) P.first[t] = blocks;
  hipLaunchKernelGGL(mi::k_adam_step, dim3((unsigned)blocks), dim3(mi::kAdamThreads), 0,
                     static_cast<hipStream_t>(stream), *adam, P, counters);
  return to_code(hipGetLastError());
}

}  // extern "C"
