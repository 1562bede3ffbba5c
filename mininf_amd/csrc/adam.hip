// One-launch Adam step (mininf_amd.optim.Adam): the optimizer step of the reference's training
// loop (README.md:66-69, `optimizer.step()` of torch.optim.Adam) for every parameter of a step in
// a single kernel, including the step-count increment that torch's capturable fused Adam runs as
// a separate `_foreach_add_` launch.
//
// Arithmetic restated from torch's fused Adam (ATen/native/cuda/fused_adam_utils.cuh adam_math,
// ADAM_MODE::ORIGINAL, no AMSGrad): hyper-parameters in double, the moments and the parameter in
// float, bias corrections 1 - beta^step in double -- bit-identical to torch.optim.Adam(fused=True).
//
// Every block reads its tensor's step s and uses s + 1; the last block of the tensor to count
// itself after its read (two levels: groups of kAdamGroup blocks, then the tensor) stores s + 1, so no
// block can read the advanced value.
//
// The bias corrections (two double pows, a few hundred dependent instructions) are computed once
// per tensor and step: the bookkeeping wave of the tensor's first block computes those of the next
// step and stores them in the counter words' cache (a slot per tensor and step parity,
// keyed by step and betas); the next launch's blocks read them instead of each computing them
// (C5's update 12.63 -> 12.43 us, the step 182.5 -> 181.5 us, profiles/r05_adam_ab.json). A slot
// that does not match (first step, a loaded step count, changed betas) falls back to the pows --
// the same function of the same inputs either way.
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

// Every kernel argument a block needs, loaded in one batch at its start: the plan's block ranges and
// chunks and the NT tensors' fields, each pinned to a register (an empty asm) so that the selection
// of the block's tensor runs on registers. Left to itself the compiler turned the selects into
// indexed loads of the argument segment -- two more dependent round trips before the block's first
// data loads (the C5 update: ~3 us of a 12 us launch).
// (a pointer through its address, handed back in the global address space: global, not flat,
// accesses)
template <typename V>
MI_DEV V* pin_ptr(V* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t a = pin(reinterpret_cast<uint64_t>(p));
  return (V*)reinterpret_cast<__attribute__((address_space(1))) V*>(a);
#else
  return p;   // (host pass: never called)
#endif
}

template <int NT>
struct Picked {
  mi_adam_tensor T;
  int first, nblocks, t;
  int64_t chunk;
};

template <int NT>
MI_DEV Picked<NT> pick_tensor(const mi_adam& A, const AdamPlan& P) {
  int first[NT + 1];
  int64_t chunk[NT];
  float* param[NT];
  const float* grad[NT];
  float* m[NT];
  float* v[NT];
  int64_t numel[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) {
    first[q] = pin(P.first[q]);
    chunk[q] = pin(P.chunk[q]);
    param[q] = pin_ptr(A.tensors[q].param);
    grad[q] = pin_ptr(A.tensors[q].grad);
    m[q] = pin_ptr(A.tensors[q].exp_avg);
    v[q] = pin_ptr(A.tensors[q].exp_avg_sq);
    numel[q] = pin(A.tensors[q].numel);
  }
  first[NT] = pin(P.first[NT]);
  const int num = pin(A.num);
  int t = 0;
#pragma unroll
  for (int q = 1; q < NT; ++q)
    if (q < num && (int)blockIdx.x >= first[q]) t = q;
  Picked<NT> r;
  // (the step word's address by the ordinary indexed argument load: its read must stay a scalar
  // load, which the barrier's lgkmcnt wait covers -- see k_adam_step; it is off the data loads' path)
  r.T = mi_adam_tensor{param[0], grad[0], m[0], v[0], nullptr, numel[0]};
  r.first = first[0];
  r.nblocks = first[1] - first[0];
  r.chunk = chunk[0];
#pragma unroll
  for (int q = 1; q < NT; ++q) {
    const bool on = q == t;
    r.T.param = on ? param[q] : r.T.param;
    r.T.grad = on ? grad[q] : r.T.grad;
    r.T.exp_avg = on ? m[q] : r.T.exp_avg;
    r.T.exp_avg_sq = on ? v[q] : r.T.exp_avg_sq;
    r.T.numel = on ? numel[q] : r.T.numel;
    r.first = on ? first[q] : r.first;
    r.nblocks = on ? first[q + 1] - first[q] : r.nblocks;
    r.chunk = on ? chunk[q] : r.chunk;
  }
  r.t = t;
  r.T.step = A.tensors[t].step;
  return r;
}

// The launch's workgroups are kAdamThreads streaming threads plus one bookkeeping wave: the
// streaming waves update their elements; the extra wave counts the workgroup in the tensor's
// completion count (device-scope atomics on shared words: the return of each is a memory round
// trip, longer under contention) and, in the tensor's first workgroup, computes the next step's bias
// corrections -- neither stalls a streaming wave (counted by streaming wave 0 and computed by
// streaming lanes, they had held that wave's elements back: the C5 update ran 12.1 us in
// tools/stream_probe.hip against 7.8 for the same arithmetic without them).
constexpr int kAdamBlock = kAdamThreads + 64;

// NT: tensor slots the launch selects from (A.num <= NT: fewer kernel-argument loads before the
// block's first data loads)
template <int U, int NT>
__global__ __launch_bounds__(kAdamBlock) void k_adam_step(const mi_adam A, const AdamPlan P,
                                                          unsigned* __restrict__ counters) {
  const Picked<NT> pk = pick_tensor<NT>(A, P);
  const mi_adam_tensor T = pk.T;
  const int t = pk.t, first = pk.first, nblocks = pk.nblocks;
  const int64_t chunk = pk.chunk;
  const int b = (int)blockIdx.x - first;
  const bool books = threadIdx.x >= kAdamThreads;   // the bookkeeping wave

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
        p[u] = param[q];
        g[u] = grad[q];
        m[u] = exp_avg[q];
        v[u] = exp_avg_sq[q];
      }
    }
  };
  int64_t i = i0 + 4 * (int64_t)threadIdx.x;
  // the first pass's loads go out before anything that waits (the step read, the bias corrections)
  if (vec && !books) load_pass(i);
  __builtin_amdgcn_sched_barrier(0);

  const float s1 = *T.step + 1.0f;
  // both parities' cached bias corrections, read with the step (one memory round trip, not two
  // dependent ones: which slot applies depends on the step); named words, not an array (a private
  // array indexed by the parity was placed in LDS through the thread's flat index)
  const uint32_t* cw = counters + kCoefOffset + t * 2 * kCoefWords;
  const uint32_t e0 = cw[0], e1 = cw[1], e2 = cw[2], e4 = cw[4], e5 = cw[5], e6 = cw[6], e7 = cw[7];
  const uint32_t o0 = cw[8], o1 = cw[9], o2 = cw[10], o4 = cw[12], o5 = cw[13], o6 = cw[14],
                 o7 = cw[15];
  // The step advances once every workgroup of the tensor has read it: every wave's step read
  // complete (lgkmcnt(0) only: the first pass's loads stay in flight), the barrier, then the
  // bookkeeping wave counts the workgroup (two levels: groups of kAdamGroup, then the tensor); the
  // tensor's last workgroup to count stores s + 1 (every workgroup has read s by then).
  // The empty asm consumes s1, so the compiler itself waits for the step read's result before the
  // barrier whatever kind of load it emits (today a scalar load, covered by lgkmcnt; a vector
  // load would get its vmcnt wait here) -- the explicit waitcnt alone only covers scalar loads.
  __asm__ volatile("" ::"v"(s1));
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  if (books) {
    if (threadIdx.x == kAdamThreads) {
      unsigned* tc = counters + t * (1 + kAdamGroup);
      const int groups = (nblocks + kAdamGroup - 1) / kAdamGroup;
      bool done = true;
      if (groups > 1) {
        const int gi = b / kAdamGroup;
        const unsigned in_group = (unsigned)min(kAdamGroup, nblocks - gi * kAdamGroup);
        unsigned* gc = tc + 1 + gi;
        done = atomicAdd(gc, 1u) == in_group - 1u;
        if (done) *gc = 0u;
      }
      if (done && atomicAdd(tc, 1u) == (unsigned)(groups > 1 ? groups : nblocks) - 1u) {
        *tc = 0u;
        *T.step = s1;
      }
    }
    // the tensor's first workgroup: the next step's corrections, into the other parity's slot (no
    // workgroup of this launch reads it)
    if (b == 0) {
      const float s2 = s1 + 1.0f;
      const AdamCoef next = adam_coef(A, s2);
      if (threadIdx.x == kAdamThreads) {
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
    return;
  }
  // bias corrections: the cached ones of this step if the slot matches, else computed here
  // (adam_math.hpp: torch's fused Adam arithmetic either way)
  AdamCoef coef;
  {
    const bool odd = ((int)s1 & 1) != 0;
    const uint32_t k0 = odd ? o0 : e0, k1 = odd ? o1 : e1, k2 = odd ? o2 : e2;
    const uint32_t k4 = odd ? o4 : e4, k5 = odd ? o5 : e5, k6 = odd ? o6 : e6, k7 = odd ? o7 : e7;
    const bool hit = __uint_as_float(k0) == s1 && __hiloint2double(k5, k4) == A.beta1 &&
                     __hiloint2double(k7, k6) == A.beta2;
    if (hit) {
      coef.bc1 = __uint_as_float(k1);
      coef.bc2_sqrt = __uint_as_float(k2);
      coef.step_size = (float)(A.lr / (double)coef.bc1);
    } else {
      coef = adam_coef(A, s1);
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
          param[q] = p[u];
          exp_avg[q] = m[u];
          exp_avg_sq[q] = v[u];
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
  // About 512 workgroups over all tensors: measured on C5's 2 x 1e6 parameters (tools/adam_probe.py,
  // graph replays; profiles/r05_adam_ab.json): 500 workgroups of 4096 elements 12.4 us, 1000 of
  // 2048 17.6 us (15.9 with every block computing its own bias corrections); at least
  // 4 * kAdamThreads elements per workgroup and at most kAdamGroup^2 workgroups per tensor.
  constexpr int64_t target_blocks = 512;
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
  const dim3 grid((unsigned)blocks), block(mi::kAdamBlock);
  const hipStream_t s = static_cast<hipStream_t>(stream);
  if (adam->num <= 2)
    hipLaunchKernelGGL((mi::k_adam_step<2, 2>), grid, block, 0, s, *adam, P, counters);
  else if (adam->num <= 4)
    hipLaunchKernelGGL((mi::k_adam_step<2, 4>), grid, block, 0, s, *adam, P, counters);
  else
    hipLaunchKernelGGL((mi::k_adam_step<2, MI_ADAM_MAX_TENSORS>), grid, block, 0, s, *adam, P,
                       counters);
  return to_code(hipGetLastError());
}

}  // extern "C"
