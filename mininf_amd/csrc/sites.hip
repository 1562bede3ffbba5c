// Site log-probability accumulation over the particle x element space of a model trace.
//
// Replaces, for the Normal / Bernoulli / Beta / Categorical families, the per-site
// `distribution.log_prob(value)` of the reference tracer (mininf/core.py:241, masked branch
// core.py:231-239), the per-site sums and minibatch scaling of LogProbTracer.total/contribution
// (core.py:247-273) and the autograd backward of those torch ops. Formulas restate
// torch/distributions (file:line cited at each family below).
//
// Three launch shapes, chosen on the host from the operand strides (mi_group_forward):
//   ROW   -- a dense operand is contiguous along elements (x[k, i], stride_i == 1): lanes run along
//            i, each wave owns a 64*ELEMS element segment and walks particle rows; coalesced
//            256-B loads/stores per wave instruction; per-row wave-shuffle reduction.
//   COL   -- a dense operand is contiguous along particles (x[i, k] as produced by a vmapped
//            `X @ theta`, stride_k == 1) or there is no dense operand: lanes run along k and loop
//            over elements; per-lane accumulation, no cross-lane reduction per element.
//   BCAST -- one site whose parameters are per-particle scalars and whose value is shared data
//            x[i] (the biased-coin / C2 shape): the value chunk is staged once in LDS and read as
//            a broadcast float4 while each lane owns P particles; the per-particle constant part of
//            log p is hoisted out of the element loop, leaving one FMA per (particle, element).
// All three write per-(segment, particle) partial sums (fp32) that k_finalize reduces in fp64 in a
// fixed order, so results are deterministic run to run.
#include "adam_math.hpp"
#include "beta_grad.hpp"
#include "common.hpp"
#include "entropy.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "internal.hpp"
#include "jit.hpp"

namespace mi {

// Uniform (scalar-branch) selection from compile-time-indexed register arrays; `idx` is always
// wave-uniform (it comes from the kernel argument block), so no VALU select chains are emitted.
template <int N>
MI_DEV float pick(const float (&v)[N], int idx) {
  float out = 0.0f;
#pragma unroll
  for (int j = 0; j < N; ++j)
    if (idx == j) out = v[j];
  return out;
}

template <int N>
MI_DEV void add_at(float (&v)[N], int idx, float x) {
#pragma unroll
  for (int j = 0; j < N; ++j)
    if (idx == j) v[j] += x;
}

// One (particle k, element i) of a site group: loads every operand once, evaluates every site,
// accumulates per-site log p and per-slot particle gradients, writes dense operand gradients.
MI_DEV void group_element(const mi_group& G, int64_t k, int64_t i, float (&lp)[MI_MAX_SITES],
                          float (&slot)[MI_MAX_SLOTS], uint32_t (&fl)[MI_MAX_SITES]) {
  float ov[MI_MAX_OPERANDS];
  float og[MI_MAX_OPERANDS];
#pragma unroll
  for (int o = 0; o < MI_MAX_OPERANDS; ++o) {
    og[o] = 0.0f;
    ov[o] = 0.0f;
    if (o < G.num_operands) {
      const mi_operand& op = G.operands[o];
      ov[o] = op.data[k * op.stride_k + i * op.stride_i];
    }
  }
#pragma unroll
  for (int s = 0; s < MI_MAX_SITES; ++s) {
    if (s < G.num_sites) {
      const mi_site& st = G.sites[s];
      float r[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) r[q] = st.operand[q] < 0 ? st.constant[q] : pick(ov, st.operand[q]);
      bool observed = true;
      if (st.mask != nullptr) observed = st.mask[k * st.mask_stride_k + i * st.mask_stride_i] != 0;
      Elem e;
      eval_family(st.family, r[0], r[1], r[2], e);
      lp[s] += observed ? e.lp : 0.0f;
      fl[s] |= (e.param_bad ? MI_FLAG_PARAM : 0u) | ((observed && e.support_bad) ? MI_FLAG_SUPPORT : 0u);
      if (G.compute_grads) {
        const float w = observed ? (float)st.scale : 0.0f;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int o = st.operand[q];
          if (o >= 0) {
            const int mode = G.operands[o].grad_mode;
            if (mode == MI_GRAD_DENSE) add_at(og, o, w * e.d[q]);
            else if (mode == MI_GRAD_PARTICLE) add_at(slot, G.operands[o].slot, w * e.d[q]);
          }
        }
      }
    }
  }
  if (G.compute_grads) {
#pragma unroll
    for (int o = 0; o < MI_MAX_OPERANDS; ++o) {
      if (o < G.num_operands) {
        const mi_operand& op = G.operands[o];
        if (op.grad_mode == MI_GRAD_DENSE)
          op.grad[k * op.grad_stride_k + i * op.grad_stride_i] = G.grad_scale * og[o];
      }
    }
  }
}

// Partial sums layout: part[(v * nseg + seg) * K + k] for value v in
// [0, num_sites) (per-site log p) followed by [num_sites, num_sites + num_slots) (slot grads).

// -------------------------------------------------------------------------------------------------
// ROW: lanes along elements.
// -------------------------------------------------------------------------------------------------
template <int ELEMS>
__global__ __launch_bounds__(256) void k_group_row(const mi_group G, float* __restrict__ part,
                                                   int64_t nseg, int64_t rows_per_block,
                                                   uint32_t* __restrict__ flags) {
  const int lane = threadIdx.x & 63;
  const int64_t seg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  uint32_t fl[MI_MAX_SITES] = {0u, 0u, 0u, 0u};
  if (seg < nseg) {
    const int64_t base = seg * (64 * ELEMS);
    const int64_t k_begin = (int64_t)blockIdx.y * rows_per_block;
    const int64_t k_end = min(G.K, k_begin + rows_per_block);
    const int nv = G.num_sites + G.num_slots;
    for (int64_t kb = k_begin; kb < k_end; kb += 64) {
      float keep[MI_MAX_SITES + MI_MAX_SLOTS];
#pragma unroll
      for (int v = 0; v < MI_MAX_SITES + MI_MAX_SLOTS; ++v) keep[v] = 0.0f;
      const int rows = (int)min((int64_t)64, k_end - kb);
      for (int r = 0; r < rows; ++r) {
        const int64_t k = kb + r;
        float lp[MI_MAX_SITES] = {0.f, 0.f, 0.f, 0.f};
        float slot[MI_MAX_SLOTS] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < ELEMS; ++e) {
          const int64_t i = base + e * 64 + lane;
          if (i < G.N) group_element(G, k, i, lp, slot, fl);
        }
#pragma unroll
        for (int s = 0; s < MI_MAX_SITES; ++s) {
          if (s < G.num_sites) {
            const float t = wave_sum(lp[s]);
            keep[s] = (lane == r) ? t : keep[s];
          }
        }
#pragma unroll
        for (int j = 0; j < MI_MAX_SLOTS; ++j) {
          if (j < G.num_slots) {
            const float t = wave_sum(slot[j]);
            keep[MI_MAX_SITES + j] = (lane == r) ? t : keep[MI_MAX_SITES + j];
          }
        }
      }
      if (lane < rows) {
#pragma unroll
        for (int s = 0; s < MI_MAX_SITES; ++s)
          if (s < G.num_sites) part[((int64_t)s * nseg + seg) * G.K + kb + lane] = keep[s];
#pragma unroll
        for (int j = 0; j < MI_MAX_SLOTS; ++j)
          if (j < G.num_slots)
            part[((int64_t)(G.num_sites + j) * nseg + seg) * G.K + kb + lane] = keep[MI_MAX_SITES + j];
      }
      (void)nv;
    }
  }
#pragma unroll
  for (int s = 0; s < MI_MAX_SITES; ++s)
    if (s < G.num_sites) publish_flags(flags + s, fl[s]);
}

// -------------------------------------------------------------------------------------------------
// COL: lanes along particles. `kw` lanes (power of two <= 64) cover consecutive particles, the
// 64 / kw lane groups of a wave take interleaved elements.
// -------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_group_col(const mi_group G, float* __restrict__ part,
                                                   int64_t nseg, int64_t seg_len, int kw,
                                                   uint32_t* __restrict__ flags) {
  const int lane = threadIdx.x & 63;
  const int64_t seg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int kq = lane & (kw - 1);
  const int isub = lane / kw;
  const int istep = 64 / kw;
  const int64_t k = (int64_t)blockIdx.y * kw + kq;
  uint32_t fl[MI_MAX_SITES] = {0u, 0u, 0u, 0u};
  float lp[MI_MAX_SITES] = {0.f, 0.f, 0.f, 0.f};
  float slot[MI_MAX_SLOTS] = {0.f, 0.f, 0.f, 0.f};
  if (seg < nseg && k < G.K) {
    const int64_t i_begin = seg * seg_len;
    const int64_t i_end = min(G.N, i_begin + seg_len);
#pragma unroll 4
    for (int64_t i = i_begin + isub; i < i_end; i += istep) group_element(G, k, i, lp, slot, fl);
  }
  if (kw < 64) {
#pragma unroll
    for (int s = 0; s < MI_MAX_SITES; ++s)
      if (s < G.num_sites) lp[s] = wave_sum_strided(lp[s], kw);
#pragma unroll
    for (int j = 0; j < MI_MAX_SLOTS; ++j)
      if (j < G.num_slots) slot[j] = wave_sum_strided(slot[j], kw);
  }
  if (seg < nseg && k < G.K && isub == 0) {
#pragma unroll
    for (int s = 0; s < MI_MAX_SITES; ++s)
      if (s < G.num_sites) part[((int64_t)s * nseg + seg) * G.K + k] = lp[s];
#pragma unroll
    for (int j = 0; j < MI_MAX_SLOTS; ++j)
      if (j < G.num_slots) part[((int64_t)(G.num_sites + j) * nseg + seg) * G.K + k] = slot[j];
  }
#pragma unroll
  for (int s = 0; s < MI_MAX_SITES; ++s)
    if (s < G.num_sites) publish_flags(flags + s, fl[s]);
}

// -------------------------------------------------------------------------------------------------
// BCAST: one site, parameters are per-particle scalars (or constants), the value is shared data.
// -------------------------------------------------------------------------------------------------
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kBcastThreads = 256;
constexpr int kBcastP = 8;          // particles per lane
constexpr int kBcastChunk = 2048;   // elements staged per block

MI_DEV float role_scalar(const mi_group& G, const mi_site& st, int q, int64_t k) {
  const int o = st.operand[q];
  if (o < 0) return st.constant[q];
  const mi_operand& op = G.operands[o];
  return op.data[k * op.stride_k];
}

MI_DEV float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int wave = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[wave] = v;
  __syncthreads();
  float out = 0.0f;
#pragma unroll
  for (int w = 0; w < kBcastThreads / 64; ++w) out += scratch[w];
  return out;
}

// Per-particle constants of a BCAST site, computed once per particle (not once per element chunk):
//   Bernoulli: l, dl/dparam, softplus(l), sigmoid(l)
//   Normal:    loc, scale, log(scale) + log sqrt(2 pi)
//   Beta:      a - 1, b - 1, lgamma(a + b) - lgamma(a) - lgamma(b), psi(a+b) - psi(a), psi(a+b) - psi(b)
// laid out as prep[j * K + k]; parameter-constraint violations are flagged here.
constexpr int kPrep = 5;

template <int FAMILY>
__global__ __launch_bounds__(256) void k_bcast_prep(const mi_group G, float* __restrict__ prep,
                                                    uint32_t* __restrict__ flags) {
  const mi_site& st = G.sites[0];
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t fl = 0u;
  if (k < G.K) {
    const float a = role_scalar(G, st, 0, k), b = role_scalar(G, st, 1, k);
    float c[kPrep] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    bool bad;
    if (FAMILY == MI_BERNOULLI_LOGITS || FAMILY == MI_BERNOULLI_PROBS) {
      float l = a, dl = 1.0f;
      if (FAMILY == MI_BERNOULLI_PROBS) {
        bad = !(a >= 0.0f && a <= 1.0f);
        bernoulli_probs_to_logits(a, l, dl);
      } else {
        bad = l != l;
      }
      // log p(x | l) = x l - softplus(l);  d/dl = x - sigmoid(l)   (bernoulli.py:121-125)
      const float t = expf(-fabsf(l));
      c[0] = l;
      c[1] = dl;
      c[2] = fmaxf(l, 0.0f) + log1pf(t);
      c[3] = l >= 0.0f ? 1.0f / (1.0f + t) : t / (1.0f + t);
    } else if (FAMILY == MI_NORMAL) {
      bad = !(b > 0.0f) || (a != a);
      c[0] = a;
      c[1] = b;
      c[2] = (float)((double)logf(b) + (double)kHalfLog2Pi);
    } else {
      bad = !(a > 0.0f) || !(b > 0.0f);
      const double psi_ab = digamma((double)a + (double)b);
      c[0] = a - 1.0f;
      c[1] = b - 1.0f;
      c[2] = (float)((double)lgammaf(a + b) - (double)lgammaf(a) - (double)lgammaf(b));
      c[3] = (float)(psi_ab - digamma((double)a));
      c[4] = (float)(psi_ab - digamma((double)b));
    }
    fl = bad ? MI_FLAG_PARAM : 0u;
#pragma unroll
    for (int j = 0; j < kPrep; ++j) prep[j * G.K + k] = c[j];
  }
  publish_flags(flags, fl);
}

// FAMILY in {MI_BERNOULLI_LOGITS, MI_BERNOULLI_PROBS, MI_NORMAL, MI_BETA}
template <int FAMILY, bool MASKED>
__global__ __launch_bounds__(kBcastThreads) void k_site_bcast(const mi_group G,
                                                              const float* __restrict__ prep,
                                                              float* __restrict__ part,
                                                              int64_t nchunk,
                                                              uint32_t* __restrict__ flags) {
  constexpr bool BERN = FAMILY == MI_BERNOULLI_LOGITS || FAMILY == MI_BERNOULLI_PROBS;
  constexpr int NF = BERN ? 1 : 2;
  // Bernoulli stages each value twice, (x, x), so a 16-byte LDS read feeds packed FMAs directly.
  __shared__ float4 feat[NF][BERN ? kBcastChunk / 2 : kBcastChunk / 4];
  __shared__ float scratch[kBcastThreads / 64];
  __shared__ float sums[4];

  const mi_site& st = G.sites[0];
  const mi_operand& vop = G.operands[st.operand[2]];
  const int64_t c = blockIdx.x;
  const int64_t i0 = c * kBcastChunk;
  const int64_t len = min((int64_t)kBcastChunk, G.N - i0);

  // ---- stage: features of the value chunk, particle-independent sums, support flags ----------
  float* f0 = reinterpret_cast<float*>(feat[0]);
  float* f1 = reinterpret_cast<float*>(feat[NF - 1]);
  float s_m = 0.0f, s_a = 0.0f, s_b = 0.0f, s_zero = 0.0f, s_one = 0.0f;
  uint32_t fl = 0u;
  for (int j = threadIdx.x; j < kBcastChunk; j += kBcastThreads) {
    float v = 0.0f, m = 0.0f;
    if (j < len) {
      const int64_t i = i0 + j;
      v = vop.data[i * vop.stride_i];
      m = 1.0f;
      if (MASKED) m = st.mask[i * st.mask_stride_i] != 0 ? 1.0f : 0.0f;
    }
    const bool obs = m != 0.0f;
    if (FAMILY == MI_BERNOULLI_LOGITS || FAMILY == MI_BERNOULLI_PROBS) {
      fl |= (obs && !(v == 0.0f || v == 1.0f)) ? MI_FLAG_SUPPORT : 0u;
      const float f = obs ? v : 0.0f;
      f0[2 * j] = f;
      f0[2 * j + 1] = f;
      s_a += f;
    } else if (FAMILY == MI_NORMAL) {
      fl |= (obs && v != v) ? MI_FLAG_SUPPORT : 0u;
      f0[j] = obs ? v : 0.0f;
      f1[j] = m;
    } else {  // MI_BETA: log v and log(1 - v); exact 0 / 1 values are counted separately
      fl |= (obs && !(v >= 0.0f && v <= 1.0f)) ? MI_FLAG_SUPPORT : 0u;
      const bool zero = obs && v == 0.0f, one = obs && v == 1.0f;
      const float la = (obs && !zero) ? logf(v) : 0.0f;
      const float lb = (obs && !one) ? logf(1.0f - v) : 0.0f;
      f0[j] = la;
      f1[j] = lb;
      s_a += la;
      s_b += lb;
      s_zero += zero ? 1.0f : 0.0f;
      s_one += one ? 1.0f : 0.0f;
    }
    s_m += m;
  }
  s_m = block_sum(s_m, scratch);
  s_a = block_sum(s_a, scratch);
  if (FAMILY == MI_BETA) {
    s_b = block_sum(s_b, scratch);
    s_zero = block_sum(s_zero, scratch);
    s_one = block_sum(s_one, scratch);
  }
  (void)sums;
  __syncthreads();

  // ---- per-particle element loop -------------------------------------------------------------
  const int64_t kbase = (int64_t)blockIdx.y * (kBcastThreads * kBcastP) + threadIdx.x;
  // Hoisted per-particle coefficients of the element loop (k_bcast_prep).
  const int64_t K = G.K;
  float ca[kBcastP], cb[kBcastP];
#pragma unroll
  for (int p = 0; p < kBcastP; ++p) {
    const int64_t k = min(kbase + p * kBcastThreads, K - 1);
    ca[p] = prep[k];
    cb[p] = prep[K + k];
  }

  double acc1[kBcastP], acc2[kBcastP];
#pragma unroll
  for (int p = 0; p < kBcastP; ++p) acc1[p] = acc2[p] = 0.0;

  // One quad of staged features against all P particles of this lane. `exact` quads hold four real
  // elements; the others (the chunk's tail) use the masked formulation, which is neutral for the
  // zero padding.
  auto quad = [&](const float4 x, const float4 y, float (&in1)[kBcastP], float (&in2)[kBcastP],
                  bool exact) {
    if (FAMILY == MI_BERNOULLI_LOGITS || FAMILY == MI_BERNOULLI_PROBS) {
      // log p(x | l) = x l - softplus(l): one FMA per (particle, element)
#pragma unroll
      for (int p = 0; p < kBcastP; ++p) {
        in1[p] = fmaf(x.x, ca[p], in1[p]);
        in1[p] = fmaf(x.y, ca[p], in1[p]);
        in1[p] = fmaf(x.z, ca[p], in1[p]);
        in1[p] = fmaf(x.w, ca[p], in1[p]);
      }
    } else if (FAMILY == MI_NORMAL) {
#pragma unroll
      for (int p = 0; p < kBcastP; ++p) {
        const float d0 = x.x - ca[p], d1 = x.y - ca[p], d2 = x.z - ca[p], d3 = x.w - ca[p];
        if (MASKED || !exact) {
          const float e0 = y.x * d0, e1 = y.y * d1, e2 = y.z * d2, e3 = y.w * d3;
          in1[p] += (e0 + e1) + (e2 + e3);
          in2[p] = fmaf(e0, d0, fmaf(e1, d1, fmaf(e2, d2, fmaf(e3, d3, in2[p]))));
        } else {
          in1[p] += (d0 + d1) + (d2 + d3);
          in2[p] = fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, fmaf(d3, d3, in2[p]))));
        }
      }
    } else {
#pragma unroll
      for (int p = 0; p < kBcastP; ++p) {
        in1[p] = fmaf(x.x, ca[p], fmaf(x.y, ca[p], fmaf(x.z, ca[p], fmaf(x.w, ca[p], in1[p]))));
        in1[p] = fmaf(y.x, cb[p], fmaf(y.y, cb[p], fmaf(y.z, cb[p], fmaf(y.w, cb[p], in1[p]))));
      }
    }
  };

  const int nq = (int)((len + 3) / 4);
  const int full = (int)(len / 4) & ~15;
  if constexpr (FAMILY == MI_BERNOULLI_LOGITS || FAMILY == MI_BERNOULLI_PROBS) {
    // x l summed over the chunk for 8 particles: packed FMAs (v_pk_fma_f32) on particle pairs,
    // two evals per lane per instruction. The zero padding of the last quad is neutral.
    f32x2 cav[kBcastP / 2];
#pragma unroll
    for (int j = 0; j < kBcastP / 2; ++j) cav[j] = f32x2{ca[2 * j], ca[2 * j + 1]};
    // feat[0][j] = (x_2j, x_2j, x_2j+1, x_2j+1); the chunk's zero padding is neutral.
    const int npair = (int)((len + 1) / 2);
    for (int j0 = 0; j0 < npair; j0 += 64) {
      // two accumulator sets (even / odd elements): 8 independent FMA chains per lane, flushed to
      // fp64 every 128 elements
      f32x2 in[2][kBcastP / 2];
#pragma unroll
      for (int j = 0; j < kBcastP / 2; ++j) in[0][j] = in[1][j] = f32x2{0.0f, 0.0f};
      if (j0 + 64 <= npair) {
#pragma unroll
        for (int h = 0; h < 8; ++h) {
          float4 xs[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) xs[j] = feat[0][j0 + 8 * h + j];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const f32x2 xa = f32x2{xs[j].x, xs[j].y}, xb = f32x2{xs[j].z, xs[j].w};
#pragma unroll
            for (int pp = 0; pp < kBcastP / 2; ++pp) {
              in[0][pp] = __builtin_elementwise_fma(xa, cav[pp], in[0][pp]);
              in[1][pp] = __builtin_elementwise_fma(xb, cav[pp], in[1][pp]);
            }
          }
        }
      } else {
        for (int j = j0; j < npair; ++j) {
          const float4 x = feat[0][j];
          const f32x2 xa = f32x2{x.x, x.y}, xb = f32x2{x.z, x.w};
#pragma unroll
          for (int pp = 0; pp < kBcastP / 2; ++pp) {
            in[0][pp] = __builtin_elementwise_fma(xa, cav[pp], in[0][pp]);
            in[1][pp] = __builtin_elementwise_fma(xb, cav[pp], in[1][pp]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < kBcastP / 2; ++j) {
        const f32x2 t = in[0][j] + in[1][j];
        acc1[2 * j] += (double)t.x;
        acc1[2 * j + 1] += (double)t.y;
      }
    }
  } else {
  for (int q0 = 0; q0 < full; q0 += 16) {
    float in1[kBcastP], in2[kBcastP];
#pragma unroll
    for (int p = 0; p < kBcastP; ++p) in1[p] = in2[p] = 0.0f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float4 xs[8], ys[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xs[j] = feat[0][q0 + 8 * h + j];
        ys[j] = NF > 1 ? feat[NF - 1][q0 + 8 * h + j] : xs[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) quad(xs[j], ys[j], in1, in2, true);
    }
#pragma unroll
    for (int p = 0; p < kBcastP; ++p) {
      acc1[p] += (double)in1[p];
      acc2[p] += (double)in2[p];
    }
  }
  {
    float in1[kBcastP], in2[kBcastP];
#pragma unroll
    for (int p = 0; p < kBcastP; ++p) in1[p] = in2[p] = 0.0f;
    for (int q = full; q < nq; ++q) {
      const float4 x = feat[0][q];
      const float4 y = NF > 1 ? feat[NF - 1][q] : x;
      quad(x, y, in1, in2, false);
    }
#pragma unroll
    for (int p = 0; p < kBcastP; ++p) {
      acc1[p] += (double)in1[p];
      acc2[p] += (double)in2[p];
    }
  }
  }

  // ---- epilogue: constant parts, gradients, partial writes -------------------------------------
  const int o_a = st.operand[0], o_b = st.operand[1];
  const bool grads = G.compute_grads != 0;
  const int slot_a = (grads && o_a >= 0 && G.operands[o_a].grad_mode == MI_GRAD_PARTICLE) ? G.operands[o_a].slot : -1;
  const int slot_b = (grads && o_b >= 0 && G.operands[o_b].grad_mode == MI_GRAD_PARTICLE) ? G.operands[o_b].slot : -1;
  const double M = s_m;
  const float w = (float)st.scale;
#pragma unroll
  for (int p = 0; p < kBcastP; ++p) {
    const int64_t k = kbase + p * kBcastThreads;
    double lp = 0.0;
    float ga = 0.0f, gb = 0.0f;
    const int64_t kc = min(k, K - 1);
    if (FAMILY == MI_BERNOULLI_LOGITS || FAMILY == MI_BERNOULLI_PROBS) {
      const double softplus = prep[2 * K + kc], sig = prep[3 * K + kc];
      lp = acc1[p] - M * softplus;
      ga = (float)(((double)s_a - M * sig) * (double)cb[p]);
    } else if (FAMILY == MI_NORMAL) {
      const double sigma = cb[p];
      const double inv2 = 1.0 / (sigma * sigma);
      lp = -0.5 * acc2[p] * inv2 - M * (double)prep[2 * K + kc];
      ga = (float)(acc1[p] * inv2);
      gb = (float)(acc2[p] * inv2 / sigma - M / sigma);
    } else {
      double base = acc1[p] + M * (double)prep[2 * K + kc];
      // xlogy semantics for exact 0 / 1 values (dirichlet.py:94)
      if (s_zero > 0.0f && ca[p] != 0.0f) base += ca[p] > 0.0f ? -__builtin_inf() : __builtin_inf();
      if (s_one > 0.0f && cb[p] != 0.0f) base += cb[p] > 0.0f ? -__builtin_inf() : __builtin_inf();
      lp = base;
      ga = (float)((double)s_a + M * (double)prep[3 * K + kc] -
                   (s_zero > 0.0f ? __builtin_inf() : 0.0));
      gb = (float)((double)s_b + M * (double)prep[4 * K + kc] -
                   (s_one > 0.0f ? __builtin_inf() : 0.0));
    }
    if (k < G.K) {
      part[((int64_t)0 * nchunk + c) * G.K + k] = (float)lp;
      if (slot_a >= 0) part[((int64_t)(1 + slot_a) * nchunk + c) * G.K + k] = w * ga;
      if (slot_b >= 0) part[((int64_t)(1 + slot_b) * nchunk + c) * G.K + k] = w * gb;
    }
  }
  publish_flags(flags, fl);
}

// Bernoulli BCAST over unmasked contiguous data, the shared values read by the scalar unit.
// Every lane of a wave needs the same x_i, so the chunk is read with s_load (constant address
// space, wave-uniform addresses) into SGPRs, and a v_pk_fma_f32 takes the SGPR pair (x_i, x_i+1)
// against the VGPR pair (l_k, l_k) of one particle: two evals per lane per instruction with no LDS
// traffic (the LDS kernel above moves 1 KB of broadcast data per 8 packed FMAs).
//
// log p(x | l) = x l - softplus(l) and d/dl = x - sigmoid(l), so a chunk's partials are
//   lp:   sum_i x_i l_k            slot: w dl_k sum_i x_i
// and the particle-constant parts, -N softplus(l_k) and -N w dl_k sigmoid(l_k), are written once,
// by the chunk-0 blocks, into one extra segment (index gridDim.x): no chunk repeats the
// transcendentals, and k_finalize adds the extra segment like any other (nseg = chunks + 1).
// Partial sums: fp32 over at most 64 terms (as k_site_bcast), carried in fp64.
typedef const __attribute__((address_space(4))) float smem_float;

// One workgroup of a group's side job (mi_side): the mi_beta_dgrad factors of 256 (draw, component)
// pairs, one per thread -- latency-bound fp64 chains that run beside the site workgroups.
MI_DEV void beta_side_block(const mi_side& S, int64_t b) {
  const int64_t t = b * kBcastThreads + threadIdx.x;
  if (t >= 2 * S.K * S.N) return;
  const int j = (int)(t & 1);
  const int64_t e = t >> 1, i = e % S.N;
  const float a = S.c1[i * S.c1_stride], bb = S.c0[i * S.c0_stride];
  const float tot = a + bb;  // concentration.sum(-1) in fp32, dirichlet.py:18
  const double psi_t = digamma((double)tot);
  const float xv = S.x[e];
  S.out[t] = (
                   j == 0 ? dirichlet_grad(xv, a, tot, digamma((double)a), psi_t) * (double)(1.0f - xv)
                          : -dirichlet_grad(1.0f - xv, bb, tot, digamma((double)bb), psi_t) * (double)xv);
}


// Grid (1-D): gy particle blocks of each chunk, chunks padded to a multiple of 8, dealt so that
// every particle block of chunk c runs on the same XCD (workgroups go to the 8 XCDs round-robin:
// block b -> XCD b % 8 = c % 8) and the chunk is fetched into that XCD's L2 once; then the side
// job's workgroups.
// rank1: the slot value is written in the rank-one layout of mi_reduce.rank1 (the chunk sums u[c]
// from the particle-block-0 workgroups, f[k] = w dl_k and e[k] = -N w sigmoid(l_k) dl_k from the
// chunk-0 workgroups) instead of one partial per (chunk, particle): half the partial slab.
// SUFF (MININF_AMD_BCAST_SUFFSTAT=1, a measurement of the floor, not the default): the
// per-(particle, element) FMA loop replaced by its closed form l_k * sum_i x_i -- the same value
// in exact arithmetic (C2's per-eval arithmetic is reducible).
// chunk: elements per chunk, a multiple of 32 and at most kSmemMaxChunk (the host sizes it so that
// chunks x particle blocks fill the chip's workgroup slots: make_plan).
constexpr int kSmemMaxChunk = 4096;
template <int FAMILY, int kSmemP, bool SUFF = false>
__global__ __launch_bounds__(kBcastThreads) void k_site_bcast_smem(const mi_group G,
                                                                   float* __restrict__ part,
                                                                   int64_t nseg, int gy,
                                                                   int mode, int chunk,
                                                                   uint32_t* __restrict__ flags) {
  __shared__ float scratch[kBcastThreads / 64];
  kernarg_prefetch<(int)sizeof(mi_group)>();
  // mode bit 0: rank-one slot layout; bit 1: progress-balanced wave priority (below)
  const int rank1 = mode & 1;
  const bool balance = (mode & 2) != 0;
  const int64_t chunks = nseg - 1;
  const int64_t padded = (chunks + 7) / 8 * 8;
  const int64_t b = blockIdx.x;
  if (b >= padded * gy) {   // workgroups past the chunks: the side job (mi_side)
    const unsigned long long ts = span_begin(G.stamps);   // (the launch's span includes them)
    beta_side_block(G.side, b - padded * gy);
    span_end(G.stamps, ts);
    return;
  }
  const int64_t c = (b / (8 * gy)) * 8 + b % 8;
  const int64_t kblock = (b / 8) % gy;
  if (c >= chunks) return;   // padding
  const unsigned long long t0 = span_begin(G.stamps);
  const mi_site& st = G.sites[0];
  const float* xg = G.operands[st.operand[2]].data;
  const int64_t i0 = c * chunk;
  const int len = (int)min((int64_t)chunk, G.N - i0);
  uint32_t fl = 0u;

  // ---- per-particle logits (as k_bcast_prep) ---------------------------------------------------
  // Only the logits live through the FMA loop (as the duplicated pairs ld): d l / d theta is
  // computed again after it, from the same values by the same code (r06: 102 -> 78 VGPR with the
  // particle-constant segment below; 86.2 vs 87.6 us per C2 step, profiles/r06_ab.json ab14).
  const int64_t K = G.K;
  const int64_t kbase = kblock * (kBcastThreads * kSmemP) + threadIdx.x;
  auto logits = [&](int p, float& l, float& d) -> bool {
    const int64_t k = kbase + p * kBcastThreads;
    const float a = role_scalar(G, st, 0, min(k, K - 1));
    d = 1.0f;
    if (FAMILY == MI_BERNOULLI_PROBS) {
      bernoulli_probs_to_logits(a, l, d);
      return !(a >= 0.0f && a <= 1.0f);
    }
    l = a;
    return a != a;
  };
  f32x2 ld[kSmemP];
#pragma unroll
  for (int p = 0; p < kSmemP; ++p) {
    float l, d;
    const bool bad = logits(p, l, d);
    ld[p] = f32x2{l, l};
    fl |= (c == 0 && kbase + p * kBcastThreads < K && bad) ? MI_FLAG_PARAM : 0u;
  }

  // ---- sum_i x_i l_k: element pairs from SGPRs against duplicated particle logits --------------
  double acc[kSmemP];
#pragma unroll
  for (int p = 0; p < kSmemP; ++p) acc[p] = 0.0;
  smem_float* xs = (smem_float*)(xg + i0);
  auto flush = [&](const f32x2 (&in)[2][kSmemP]) {
#pragma unroll
    for (int p = 0; p < kSmemP; ++p)
      acc[p] += (double)((in[0][p].x + in[0][p].y) + (in[1][p].x + in[1][p].y));
  };
  // Whole 256-element blocks in groups of 32 (two s_load_dwordx16): the next group's loads are in
  // flight during this group's packed FMAs (scalar loads return out of order, so every use waits
  // for all of them: one group of lookahead). Even and odd element pairs go to separate
  // accumulators, 2 kSmemP independent chains of 64 terms per block.
  constexpr int kGroup = 32, kBlock = 256;
  const int nfull = SUFF ? 0 : len & ~(kBlock - 1);
  int j = 0;
  if (nfull > 0) {
    float xc[kGroup];
#pragma unroll
    for (int e = 0; e < kGroup; ++e) xc[e] = xs[e];
    // the first block index of each later quarter of the chunk (no division inside the loop)
    const int q1 = (nfull / 4 + kBlock - 1) & ~(kBlock - 1), q2 = (nfull / 2 + kBlock - 1) & ~(kBlock - 1),
              q3 = (3 * nfull / 4 + kBlock - 1) & ~(kBlock - 1);
    if (balance) __builtin_amdgcn_s_setprio(3);
    for (; j < nfull; j += kBlock) {
      // Progress-balanced priority: a wave drops one priority level per quarter of its chunk, so
      // the SIMD's arbiter (priority, then age) lets the waves behind it catch up; the waves of a
      // SIMD then finish together instead of the oldest first, which would leave the last one
      // issuing alone (at half the VALU rate) through the kernel's tail.
      if (balance) {
        if (j == q1) __builtin_amdgcn_s_setprio(2);
        else if (j == q2) __builtin_amdgcn_s_setprio(1);
        else if (j == q3) __builtin_amdgcn_s_setprio(0);
      }
      f32x2 in[2][kSmemP];
#pragma unroll
      for (int p = 0; p < kSmemP; ++p) in[0][p] = in[1][p] = f32x2{0.0f, 0.0f};
#pragma unroll
      for (int g = 0; g < kBlock; g += kGroup) {
        const int nxt = min(j + g + kGroup, nfull - kGroup);   // in bounds; the last is unused
        float xn[kGroup];
#pragma unroll
        for (int e = 0; e < kGroup; ++e) xn[e] = xs[nxt + e];
#pragma unroll
        for (int e = 0; e < kGroup; e += 2) {
          const f32x2 xv = f32x2{xc[e], xc[e + 1]};
#pragma unroll
          for (int p = 0; p < kSmemP; ++p)
            in[(e >> 1) & 1][p] = __builtin_elementwise_fma(xv, ld[p], in[(e >> 1) & 1][p]);
        }
#pragma unroll
        for (int e = 0; e < kGroup; ++e) xc[e] = xn[e];
      }
      flush(in);
    }
  }
  if (!SUFF && j + kGroup <= len) {   // whole groups of 32 past the last whole block
    f32x2 in[2][kSmemP];
#pragma unroll
    for (int p = 0; p < kSmemP; ++p) in[0][p] = in[1][p] = f32x2{0.0f, 0.0f};
    float xc[kGroup];
#pragma unroll
    for (int e = 0; e < kGroup; ++e) xc[e] = xs[j + e];
    for (; j + kGroup <= len; j += kGroup) {
      const int nxt = min(j + kGroup, len - kGroup);   // in bounds; the last is unused
      float xn[kGroup];
#pragma unroll
      for (int e = 0; e < kGroup; ++e) xn[e] = xs[nxt + e];
#pragma unroll
      for (int e = 0; e < kGroup; e += 2) {
        const f32x2 xv = f32x2{xc[e], xc[e + 1]};
#pragma unroll
        for (int p = 0; p < kSmemP; ++p)
          in[(e >> 1) & 1][p] = __builtin_elementwise_fma(xv, ld[p], in[(e >> 1) & 1][p]);
      }
#pragma unroll
      for (int e = 0; e < kGroup; ++e) xc[e] = xn[e];
    }
    flush(in);
  }
  if (!SUFF && j < len) {   // the chunk's tail: element pairs, a zero for an odd last element
    f32x2 in[2][kSmemP];
#pragma unroll
    for (int p = 0; p < kSmemP; ++p) in[0][p] = in[1][p] = f32x2{0.0f, 0.0f};
    for (int e = 0; j < len; j += 2, ++e) {
      const f32x2 xv = f32x2{xs[j], j + 1 < len ? xs[j + 1] : 0.0f};
#pragma unroll
      for (int p = 0; p < kSmemP; ++p)
        in[e & 1][p] = __builtin_elementwise_fma(xv, ld[p], in[e & 1][p]);
    }
    flush(in);
  }

  // ---- chunk sum and support flags (vector loads, L2-resident by now) --------------------------
  // Each lane takes kSmemMaxChunk / kBcastThreads consecutive elements (those within the chunk)
  // with all its loads in flight at once (a strided loop waits for one L2 round trip per element
  // group, at the end of every wave).
  constexpr int kPerLane = kSmemMaxChunk / kBcastThreads;
  static_assert(kPerLane % 4 == 0, "whole float4 groups per lane");
  float s_a = 0.0f;
  {
    const int e0 = (int)threadIdx.x * kPerLane;
    const float* xl = xg + i0 + e0;
    if (e0 + kPerLane <= len && (reinterpret_cast<uintptr_t>(xl) & 15) == 0) {
      float v[kPerLane];
#pragma unroll
      for (int q = 0; q < kPerLane / 4; ++q) {
        const float4 t = reinterpret_cast<const float4*>(xl)[q];
        v[4 * q] = t.x;
        v[4 * q + 1] = t.y;
        v[4 * q + 2] = t.z;
        v[4 * q + 3] = t.w;
      }
#pragma unroll
      for (int e = 0; e < kPerLane; ++e) {
        fl |= !(v[e] == 0.0f || v[e] == 1.0f) ? MI_FLAG_SUPPORT : 0u;
        s_a += v[e];
      }
    } else {
      for (int e = e0; e < len && e < e0 + kPerLane; ++e) {
        const float v = xg[i0 + e];
        fl |= !(v == 0.0f || v == 1.0f) ? MI_FLAG_SUPPORT : 0u;
        s_a += v;
      }
    }
  }
  s_a = block_sum(s_a, scratch);
  if (SUFF) {
#pragma unroll
    for (int p = 0; p < kSmemP; ++p) acc[p] = (double)ld[p].x * (double)s_a;
  }
  __asm__ volatile("" ::: "memory");   // (the parameters are read again, not held in registers)
  float dl[kSmemP];
#pragma unroll
  for (int p = 0; p < kSmemP; ++p) {
    float l;
    (void)logits(p, l, dl[p]);
  }

  // ---- partials of this chunk, and the particle-constant segment (below) --------------------
  const int o_a = st.operand[0];
  const int slot_a = (G.compute_grads != 0 && o_a >= 0 && G.operands[o_a].grad_mode == MI_GRAD_PARTICLE)
                         ? G.operands[o_a].slot : -1;
  const float w = (float)st.scale;
  const int64_t extra = nseg - 1;
  uint32_t fl_prior = 0u;
  float* slot_part = part + (int64_t)(1 + slot_a) * nseg * K;   // (slot_a >= 0)
  if (rank1 && slot_a >= 0 && kblock == 0 && threadIdx.x == 0) slot_part[c] = s_a;   // u[c]
#pragma unroll
  for (int p = 0; p < kSmemP; ++p) {
    const int64_t k = kbase + p * kBcastThreads;
    if (k >= K) continue;
    part[c * K + k] = (float)acc[p];
    if (slot_a >= 0 && !rank1) slot_part[c * K + k] = w * (s_a * dl[p]);
  }
  // The particle-constant segment: particle slot p of every lane by the chunk-p workgroups (chunk 0
  // takes all of them when the grid has fewer chunks than particles per lane), one particle at a
  // time -- the prior's special functions interleaved over the particles held ~40 registers.
  const bool spread = chunks >= kSmemP;
  if (spread ? c < kSmemP : c == 0) {
    const int p0 = spread ? (int)c : 0, p1 = spread ? (int)c + 1 : kSmemP;
#pragma unroll 1
    for (int p = p0; p < p1; ++p) {
      const int64_t k = kbase + p * kBcastThreads;
      if (k >= K) continue;
      float l, dlp;
      (void)logits(p, l, dlp);
      const float t = expf(-fabsf(l));
      const double softplus = (double)(fmaxf(l, 0.0f) + log1pf(t));
      const double sig = (double)(l >= 0.0f ? 1.0f / (1.0f + t) : t / (1.0f + t));
      const double n = (double)G.N;
      // the folded prior site (mi_prior): log p(a_k) and d/da_k of the per-particle parameter a_k
      float prior_lp = 0.0f, prior_d = 0.0f;
      if (G.prior.present != 0) {
        const float a = role_scalar(G, st, 0, k);
        Elem pe;
        if (G.prior.family == MI_BETA) eval_beta(G.prior.constant[0], G.prior.constant[1], a, pe);
        else if (G.prior.family == MI_NORMAL) eval_normal(G.prior.constant[0], G.prior.constant[1], a, pe);
        else eval_gamma(G.prior.constant[0], G.prior.constant[1], a, pe);
        prior_lp = pe.lp;
        prior_d = pe.d[2];
        fl_prior |= (pe.param_bad ? MI_FLAG_PARAM : 0u) | (pe.support_bad ? MI_FLAG_SUPPORT : 0u);
      }
      part[extra * K + k] = (float)(-n * softplus) + prior_lp;
      if (slot_a >= 0) {
        const float e = w * (float)(-n * sig * (double)dlp) + w * prior_d;
        if (rank1) {
          slot_part[nseg + k] = w * dlp;         // f[k]
          slot_part[nseg + K + k] = e;           // e[k]
        } else {
          slot_part[extra * K + k] = e;
        }
      }
    }
  }
  if (rank1 && slot_a >= 0 && kblock == 0 && threadIdx.x == 0 && c == 0) slot_part[extra] = 0.0f;
  publish_flags(flags, fl);
  if (G.prior.present != 0) publish_flags(G.prior.flags, fl_prior);
  span_end(G.stamps, t0);
}

// -------------------------------------------------------------------------------------------------
// Finalize: fixed-order fp64 reduction of partials over segments.
// -------------------------------------------------------------------------------------------------
struct FinalizeArgs {
  int32_t num_sites;
  int32_t num_slots;
  int32_t rank1;      // bit v: value v in the rank-one layout (mi_reduce.rank1)
  int32_t pad0;
  double scale[MI_MAX_SITES];  // num_sites <= MI_MAX_SITES
  double slot_scale;  // the group's grad_scale: slot gradients are speculative like dense ones
};

// One block per 64 particles; its 1024 threads split the segments 16 ways (fixed assignment), each
// sums its share in fp64 with independent loads in flight, then the 16 shares are combined in a
// fixed order through LDS -- deterministic, and ~16x the memory-level parallelism of a thread-per-
// particle loop.
constexpr int kFinK = 64;
constexpr int kFinG = 16;

// Stage 1 of the two-stage finalize for long segment lists: block (k-block, v, chunk) sums the
// chunk's segments of value v for 64 particles (fixed order) into stage[v][chunk][k] (fp64).
constexpr int64_t kFinChunk = 256;

__global__ __launch_bounds__(kFinK * kFinG) void k_finalize_chunks(const float* __restrict__ part,
                                                                  int64_t nseg, int64_t K,
                                                                  double* __restrict__ stage) {
  __shared__ double red[kFinG][kFinK];
  const int kl = threadIdx.x % kFinK;
  const int gl = threadIdx.x / kFinK;
  const int64_t k = (int64_t)blockIdx.x * kFinK + kl;
  const int64_t kc = k < K ? k : K - 1;
  const int64_t v = blockIdx.y, c = blockIdx.z, nchunk = gridDim.z;
  const int64_t g0 = c * kFinChunk, g1 = min(nseg, g0 + kFinChunk);
  const float* p = part + v * nseg * K + kc;
  double a0 = 0.0, a1 = 0.0;
  int64_t g = g0 + gl;
  for (; g + kFinG < g1; g += 2 * kFinG) {
    a0 += (double)p[g * K];
    a1 += (double)p[(g + kFinG) * K];
  }
  for (; g < g1; g += kFinG) a0 += (double)p[g * K];
  red[gl][kl] = a0 + a1;
  __syncthreads();
  if (gl == 0 && k < K) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < kFinG; ++j) acc += red[j][kl];
    stage[(v * nchunk + c) * K + k] = acc;
  }
}

template <typename T>
__global__ __launch_bounds__(kFinK * kFinG) void k_finalize(const T* __restrict__ part,
                                                           int64_t nseg, int64_t K,
                                                           const FinalizeArgs A,
                                                           float* __restrict__ total,
                                                           double* __restrict__ site_lp,
                                                           float* __restrict__ slot_grad) {
  __shared__ double red[kFinG][kFinK];
  const int kl = threadIdx.x % kFinK;
  const int gl = threadIdx.x / kFinK;
  const int64_t k = (int64_t)blockIdx.x * kFinK + kl;
  const int64_t kc = k < K ? k : K - 1;
  double t = 0.0;
  const int nv = A.num_sites + A.num_slots;
  // With one (combined) site value, blockIdx.y selects the value: many-slot groups (linear sites:
  // one slot per coefficient) reduce in parallel instead of one value after another.
  const bool split = gridDim.y > 1;
  const int v_begin = split ? (int)blockIdx.y : 0;
  const int v_end = split ? v_begin + 1 : nv;
  for (int v = v_begin; v < v_end; ++v) {
    const bool r1 = (A.rank1 >> v) & 1;
    // rank one: the particle-independent u[seg] (stride 1) instead of the per-particle column
    const T* p = part + (int64_t)v * nseg * K + (r1 ? 0 : kc);
    const int64_t stride = r1 ? 1 : K;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int64_t g = gl;
    for (; g + 3 * kFinG < nseg; g += 4 * kFinG) {
      a0 += (double)p[g * stride];
      a1 += (double)p[(g + kFinG) * stride];
      a2 += (double)p[(g + 2 * kFinG) * stride];
      a3 += (double)p[(g + 3 * kFinG) * stride];
    }
    for (; g < nseg; g += kFinG) a0 += (double)p[g * stride];
    __syncthreads();
    red[gl][kl] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (gl == 0 && k < K) {
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < kFinG; ++j) acc += red[j][kl];
      if (r1) {
        const T* q = part + (int64_t)v * nseg * K + nseg;
        acc = (double)q[kc] * acc + (double)q[K + kc];
      }
      if (v < A.num_sites) {
        acc *= A.scale[v];
        if (site_lp != nullptr) site_lp[(int64_t)v * K + k] = acc;
        t += acc;
      } else {
        slot_grad[(int64_t)(v - A.num_sites) * K + k] = (float)(acc * A.slot_scale);
      }
    }
  }
  if (gl == 0 && k < K && v_begin == 0) total[k] = (float)t;
}

// -------------------------------------------------------------------------------------------------
// Fused guide draws: sum the per-K-block dloc / dscale partials (fixed order, fp64).
// -------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_draw_reduce(const float* __restrict__ part, int64_t slices,
                                                     int64_t N, float* __restrict__ dloc,
                                                     float* __restrict__ dscale) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  double a = 0.0, b = 0.0;
  for (int64_t y = 0; y < slices; ++y) {
    a += (double)part[y * N + i];
    b += (double)part[(slices + y) * N + i];
  }
  dloc[i] = (float)a;
  dscale[i] = (float)b;
}

// -------------------------------------------------------------------------------------------------
// Backward rescale of speculative dense gradients.
// -------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_scale_rows(float* __restrict__ x, int64_t sk, int64_t si,
                                                    int64_t K, int64_t N,
                                                    const float* __restrict__ g, float g0,
                                                    int64_t rows_per_block) {
  const int64_t k0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t k1 = min(K, k0 + rows_per_block);
  bool all_same = true;
  for (int64_t k = k0; k < k1; ++k) all_same &= (g[k] == g0);
  if (all_same) return;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  for (int64_t k = k0; k < k1; ++k) {
    const float f = g[k] / g0;
    if (f != 1.0f) x[k * sk + i * si] *= f;
  }
}

// -------------------------------------------------------------------------------------------------
// Categorical: normalisation (categorical.py:74-78, logits - logsumexp) and gather
// (categorical.py:150-156) of one (particle, element) row per lane, lanes along elements. The row's
// C logits are read twice (max, then the exponentials; the second pass hits L1/L2). Gradient with
// respect to the given logits, dense: g * (onehot(v) - softmax) -- exact for raw logits, and for
// already normalised ones (whose logsumexp is 0) the same vector autograd's normalisation backward
// passes through unchanged.
// -------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_categorical(
    const float* __restrict__ logits, int64_t sk, int64_t si, int64_t sc, int64_t K, int64_t N,
    int64_t C, const int64_t* __restrict__ value, int64_t vsk, int64_t vsi,
    const uint8_t* __restrict__ mask, int64_t msi, float gscale, float* __restrict__ dlogits,
    float* __restrict__ part, int64_t nseg, uint32_t* __restrict__ flags) {
  const int lane = threadIdx.x & 63;
  const int64_t seg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t k = blockIdx.y;
  uint32_t fl = 0u;
  if (seg < nseg) {
    float acc = 0.0f;
    for (int e = 0; e < 16; ++e) {
      const int64_t i = seg * 1024 + e * 64 + lane;
      if (i >= N) break;
      const bool obs = mask == nullptr || mask[i * msi] != 0;
      const int64_t v = value[k * vsk + i * vsi];
      const bool ok = v >= 0 && v < C;
      fl |= (obs && !ok) ? MI_FLAG_SUPPORT : 0u;
      const float* row = logits + k * sk + i * si;
      float* drow = dlogits == nullptr ? nullptr : dlogits + k * sk + i * si;
      if (!(obs && ok)) {   // masked lanes: value and gradient 0 (util.py:85-90)
        if (drow != nullptr)
          for (int64_t c = 0; c < C; ++c) drow[c * sc] = 0.0f;
        continue;
      }
      float mx = -INFINITY;
      for (int64_t c = 0; c < C; ++c) mx = fmaxf(mx, row[c * sc]);
      const float shift = isinf(mx) ? 0.0f : mx;   // torch.logsumexp's all--inf guard
      float se = 0.0f;
      for (int64_t c = 0; c < C; ++c) se += expf(row[c * sc] - shift);
      const float lse = logf(se) + shift;
      acc += row[v * sc] - lse;
      if (drow != nullptr) {
        const float inv = 1.0f / se;
        for (int64_t c = 0; c < C; ++c) {
          const float soft = expf(row[c * sc] - shift) * inv;
          drow[c * sc] = gscale * ((c == v ? 1.0f : 0.0f) - soft);
        }
      }
    }
    acc = wave_sum(acc);
    if (lane == 0) part[seg * K + k] = acc;
  }
  publish_flags(flags, fl);
}

__global__ void k_categorical_finalize(const float* __restrict__ part, int64_t nseg, int64_t K,
                                       double scale, float* __restrict__ total) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  double acc = 0.0;
  for (int64_t g = 0; g < nseg; ++g) acc += (double)part[g * K + k];
  total[k] = (float)(acc * scale);
}

}  // namespace mi

// =================================================================================================
// Host side: launch-shape selection and the C ABI.
// =================================================================================================
namespace {

enum Shape { kRow = 0, kCol = 1, kBcast = 2 };

constexpr int kRowElems = 8;
constexpr int kColUnroll = 4;
constexpr int64_t kTargetBlocks = 2048;

int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

bool validate_group(const mi_group* g) {
  if (g == nullptr || g->K < 1 || g->N < 1) return false;
  if (g->num_sites < 1 || g->num_sites > MI_MAX_SITES) return false;
  if (g->num_operands < 0 || g->num_operands > MI_MAX_OPERANDS) return false;
  if (g->num_slots < 0 || g->num_slots > MI_MAX_SLOTS) return false;
  for (int s = 0; s < g->num_sites; ++s) {
    const mi_site& st = g->sites[s];
    if (st.family < MI_NORMAL || st.family > MI_INVERSE_GAMMA) return false;
    if (st.operand[2] < 0) return false;  // the value is always an operand
    for (int q = 0; q < 3; ++q)
      if (st.operand[q] >= g->num_operands) return false;
  }
  const int draw = g->draw.operand - 1;
  if (draw >= g->num_operands || draw < -1) return false;
  if (draw >= 0 && (g->draw.loc == nullptr || g->draw.scale == nullptr ||
                    g->draw.element_offset < 0 || (g->draw.element_offset & 3) != 0 ||
                    (g->compute_grads && !(g->options & MI_GROUP_DRAW_PARTIALS) &&
                     (g->draw.dloc == nullptr || g->draw.dscale == nullptr))))
    return false;
  if (g->side.out != nullptr &&
      (g->side.x == nullptr || g->side.c1 == nullptr || g->side.c0 == nullptr || g->side.K < 1 ||
       g->side.N < 1))
    return false;
  if (g->prior.present != 0 &&
      ((g->prior.family != MI_BETA && g->prior.family != MI_NORMAL && g->prior.family != MI_GAMMA) ||
       g->prior.flags == nullptr || g->sites[0].operand[0] < 0))
    return false;
  const int pdraw = g->pdraw.operand - 1;
  if (pdraw >= g->num_operands || pdraw < -1 || (pdraw >= 0 && pdraw == draw)) return false;
  if (pdraw >= 0 && (g->pdraw.loc == nullptr || g->pdraw.scale == nullptr ||
                     g->pdraw.element_offset < 0 || (g->pdraw.element_offset & 3) != 0 ||
                     g->operands[pdraw].stride_i != 0 || g->operands[pdraw].stride_k == 0))
    return false;
  for (int o = 0; o < g->num_operands; ++o) {
    const mi_operand& op = g->operands[o];
    if (o == draw) continue;  // computed in the kernel
    if (op.data == nullptr) return false;
    if (op.grad_mode == MI_GRAD_DENSE && op.grad == nullptr) return false;
    if (op.grad_mode == MI_GRAD_PARTICLE && (op.slot < 0 || op.slot >= g->num_slots)) return false;
  }
  return true;
}

// A fused guide draw (mi_draw) needs the row layout with whole element quads per lane and plain
// row-major [K, N] companions (see include/mininf_amd.h).
// Largest particle block of a program that makes a per-particle draw (mi_group.pdraw): the
// values live in an LDS table of the program (jit.cpp kPdrawTable).
constexpr int64_t kPdrawMax = 1024;

bool draw_supported(const mi_group* g) {
  const int draw = g->draw.operand - 1;
  if (draw < 0) return true;
  if (g->N % 4 != 0 || g->N < 64 * 8) return false;
  for (int o = 0; o < g->num_operands; ++o) {
    const mi_operand& op = g->operands[o];
    if (o == draw) continue;
    if (op.stride_k != 0 && op.stride_i != 0 && op.stride_i != 1) return false;
    if (op.stride_k == 0 && op.stride_i != 0 && op.stride_i != 1) return false;
  }
  for (int s = 0; s < g->num_sites; ++s) {
    const mi_site& st = g->sites[s];
    if (st.mask != nullptr && st.mask_stride_k != 0) return false;
  }
  return true;
}

bool is_dense(const mi_operand& op) { return op.stride_k != 0 && op.stride_i != 0; }

int env_int(const char* name, int fallback) {
  const char* v = std::getenv(name);
  return v != nullptr ? std::atoi(v) : fallback;
}

bool bcast_eligible(const mi_group* g) {
  if (g->num_sites != 1 || g->N < 1024 || g->K < 64) return false;
  const mi_site& st = g->sites[0];
  if (st.family > MI_BETA) return false;   // BCAST kernels exist for the first four families
  if (st.mask != nullptr && st.mask_stride_k != 0) return false;
  const mi_operand& v = g->operands[st.operand[2]];
  if (v.stride_k != 0 || v.stride_i == 0 || v.grad_mode != MI_GRAD_NONE) return false;
  for (int q = 0; q < 2; ++q) {
    const int o = st.operand[q];
    if (o < 0) continue;
    const mi_operand& op = g->operands[o];
    if (op.stride_i != 0 || op.grad_mode == MI_GRAD_DENSE) return false;
  }
  return true;
}

// Bernoulli BCAST sites over unmasked contiguous data run k_site_bcast_smem.
bool bcast_smem(const mi_group* g) {
  const mi_site& st = g->sites[0];
  return (st.family == MI_BERNOULLI_LOGITS || st.family == MI_BERNOULLI_PROBS) &&
         st.mask == nullptr && g->operands[st.operand[2]].stride_i == 1;
}

// k_site_bcast_smem: particles per lane and chunk length (measured r02: the best of {4, 8} x
// {2048, 4096, 8192}; r06 at 78 VGPR: 8 particles per lane in 1010 workgroups 91.8 us per C2 step
// against 86.2, profiles/r06_ab.json ab14)
constexpr int kSmemP = 4;
// Chunks of at most 4096 elements (measured r02: 4096 against 2048 / 8192), sized so that chunks x
// particle blocks come close to kSmemSlots workgroups: four 4-wave workgroups per CU on 256 CUs, one
// round. (r05 used 4096-element chunks throughout: C2's 245 chunks x 4 particle blocks left 44 of
// the 1024 slots idle; r06: 1280 / 1536 slots at 78 VGPR measured slower, ab14.)
constexpr int64_t kSmemSlots = 1024;

// Grids of 4096-element chunks between half a round and one round of slots are evened out to one
// round; smaller grids keep 4096 (shorter chunks would only add partials for the reduction).
int smem_chunk(int64_t N, int64_t gy) {
  gy = std::max<int64_t>(1, gy);
  const int64_t blocks = ceil_div(N, mi::kSmemMaxChunk) * gy;
  if (blocks < kSmemSlots / 2 || blocks > kSmemSlots) return mi::kSmemMaxChunk;
  const int64_t chunk = (ceil_div(N, kSmemSlots / gy) + 31) / 32 * 32;
  return (int)std::min<int64_t>(mi::kSmemMaxChunk, std::max<int64_t>(2048, chunk));
}

struct Plan {
  Shape shape;
  bool draw = false;       // a fused guide draw (mi_draw)
  int elems;               // ROW: elements per lane per row
  int64_t nseg;
  int64_t rows_per_block;  // ROW
  int64_t seg_len;         // COL
  int kw;                  // COL
  int chunk = 0;           // BCAST (k_site_bcast_smem): elements per chunk
  dim3 grid;
};

Plan make_plan(const mi_group* g) {
  Plan p{};
  const int nv = g->num_sites + g->num_slots;
  (void)nv;
  if (g->draw.operand == 0 && bcast_eligible(g)) {
    p.shape = kBcast;
    const bool smem = bcast_smem(g);
    if (smem) p.chunk = smem_chunk(g->N, ceil_div(g->K, mi::kBcastThreads * kSmemP));
    const int64_t chunks = ceil_div(g->N, smem ? p.chunk : mi::kBcastChunk);
    p.nseg = smem ? chunks + 1 : chunks;   // k_site_bcast_smem: + the particle-constant segment
    const int64_t side = (smem && g->side.out != nullptr)
                             ? ceil_div(2 * g->side.K * g->side.N, mi::kBcastThreads) : 0;
    p.grid = dim3((unsigned)(chunks + side),
                  (unsigned)ceil_div(g->K, mi::kBcastThreads * (smem ? kSmemP : mi::kBcastP)));
    return p;
  }
  int dense = -1;
  for (int o = 0; o < g->num_operands; ++o)
    if (is_dense(g->operands[o])) { dense = o; break; }
  const bool row = dense >= 0 && g->operands[dense].stride_i == 1 && g->operands[dense].stride_k != 1;
  const bool row_fallback = dense >= 0 && g->operands[dense].stride_k != 1 && g->operands[dense].stride_i != 1 &&
                            llabs(g->operands[dense].stride_i) < llabs(g->operands[dense].stride_k);
  // Short element spaces (e.g. a prior over a handful of coefficients) have too few row
  // segments to fill the chip and would loop over all particles serially: lanes go along
  // particles instead.
  const bool short_rows = g->N < 256 && g->draw.operand == 0;
  if ((row || row_fallback) && !short_rows) {
    p.shape = kRow;
    p.draw = g->draw.operand != 0;
    // fused draws: one Philox quad per lane and row keeps the register footprint at 4 waves/SIMD
    p.elems = g->draw.operand != 0 ? 4 : kRowElems;
    p.nseg = ceil_div(g->N, 64 * p.elems);
    const int64_t gx = ceil_div(p.nseg, 4);
    // about two rounds of 4-wave blocks (fused draws: fewer, longer particle blocks write fewer
    // d loc / d scale partial rows for the same balance; r04/r05 sweeps kept this target)
    int64_t gy = std::max<int64_t>(1, std::min<int64_t>(ceil_div(g->K, 64),
                                                        ceil_div(kTargetBlocks, gx)));
    p.rows_per_block = ceil_div(g->K, gy);
    gy = ceil_div(g->K, p.rows_per_block);
    p.grid = dim3((unsigned)gx, (unsigned)gy);
    return p;
  }
  p.shape = kCol;
  int kw = 1;
  while (kw < 64 && kw < g->K) kw <<= 1;
  p.kw = kw;
  const int64_t gy = ceil_div(g->K, kw);
  const int istep = 64 / kw;
  const int64_t waves_per_tile = std::max<int64_t>(1, (kTargetBlocks * 4) / gy);
  int64_t seg_len = ceil_div(g->N, waves_per_tile);
  seg_len = std::max<int64_t>(seg_len, (int64_t)istep * 16);
  seg_len = ceil_div(seg_len, istep) * istep;
  p.seg_len = seg_len;
  p.nseg = ceil_div(g->N, seg_len);
  p.grid = dim3((unsigned)ceil_div(p.nseg, 4), (unsigned)gy);
  return p;
}

PlanInfo plan_info(const Plan& p, bool combined) {
  PlanInfo info{};
  info.combined = combined;
  info.row = p.shape == kRow;
  info.elems = p.shape == kRow ? p.elems : kColUnroll;
  // fused draws: the block's four waves combine their particle sums (a quarter of the partial rows:
  // C5's 3907 segments become 977 rows, within the ELBO forward's fused reduction)
  info.block_rows = info.row && p.draw;
  info.packed = info.row && p.draw;
  info.kw = p.kw;
  info.grid_x = p.grid.x;
  info.grid_y = p.grid.y;
  return info;
}

size_t partial_bytes(const mi_group* g, const Plan& p) {
  const int nv = g->num_sites + g->num_slots;
  return (size_t)nv * (size_t)p.nseg * (size_t)g->K * sizeof(float);
}

// BCAST groups also hold the per-particle constants after the (256-byte aligned) partials.
size_t prep_offset(const mi_group* g, const Plan& p) {
  return (partial_bytes(g, p) + 255) / 256 * 256;
}

// Per-K-block partial dloc / dscale of a fused draw (when the grid splits the particles, or when
// the caller reduces them itself: MI_GROUP_DRAW_PARTIALS).
size_t draw_partial_floats(const mi_group* g, const Plan& p) {
  if (g->draw.operand == 0 || !g->compute_grads) return 0;
  if (p.grid.y <= 1 && !(g->options & MI_GROUP_DRAW_PARTIALS)) return 0;
  return 2 * (size_t)p.grid.y * (size_t)g->N;
}

size_t finalize_offset(const mi_group* g, const Plan& p) {
  const size_t middle = p.shape != kBcast ? draw_partial_floats(g, p) * sizeof(float)
                                          : (size_t)mi::kPrep * (size_t)g->K * sizeof(float);
  return (prep_offset(g, p) + middle + 255) / 256 * 256;
}

// The slot value of a k_site_bcast_smem launch in the rank-one layout (mi_reduce.rank1): one
// slot, and a segment list short enough for the one-launch finalize / the fused reduction.
bool smem_rank1(const mi_group* g, const Plan& p) {
  return g->num_slots == 1 && g->compute_grads && p.nseg >= 3 && p.nseg <= MI_REDUCE_MAX_SEG;
}

template <int FAM>
void launch_smem(const mi_group& G, const Plan& p, float* part, uint32_t* flags, hipStream_t s) {
  const dim3 block(mi::kBcastThreads);
  // p.grid = (chunks + side blocks, particle blocks): the kernel takes them as one XCD-aware
  // dimension (see k_site_bcast_smem)
  const int64_t chunks = p.nseg - 1;
  const int64_t side = (int64_t)p.grid.x - chunks;
  const int gy = (int)p.grid.y;
  const dim3 grid((unsigned)(ceil_div(chunks, 8) * 8 * gy + side));
  const int rank1 = (smem_rank1(&G, p) ? 1 : 0) | 2;   // bit 2: progress-balanced priorities
  // MININF_AMD_BCAST_SUFFSTAT=1: the reducible-floor measurement of bench.py (sum_i x_i l_k as
  // l_k sum_i x_i), never the default
  if (env_int("MININF_AMD_BCAST_SUFFSTAT", 0) != 0)
    hipLaunchKernelGGL((mi::k_site_bcast_smem<FAM, kSmemP, true>), grid, block, 0, s,
                       G, part, p.nseg, gy, rank1, p.chunk, flags);
  else
    hipLaunchKernelGGL((mi::k_site_bcast_smem<FAM, kSmemP>), grid, block, 0, s, G,
                       part, p.nseg, gy, rank1, p.chunk, flags);
}

size_t workspace_bytes(const mi_group* g, const Plan& p) {
  return finalize_offset(g, p) +
         mi_finalize_scratch_bytes(p.nseg, g->K, g->num_sites + g->num_slots);
}

int to_code(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

}  // namespace

size_t mi_finalize_scratch_bytes(int64_t nseg, int64_t K, int nv) {
  if (nseg <= 2 * mi::kFinChunk) return 0;
  return (size_t)nv * (size_t)ceil_div(nseg, mi::kFinChunk) * (size_t)K * sizeof(double);
}

int mi_launch_finalize(const float* part, int64_t nseg, int64_t K, int num_sites, int num_slots,
                       const double* scale, double slot_scale, float* total, double* site_lp,
                       float* slot_grad, double* scratch, hipStream_t stream, int rank1) {
  if (num_sites > MI_MAX_SITES) return MI_EINVAL;
  mi::FinalizeArgs A{};
  A.num_sites = num_sites;
  A.num_slots = num_slots;
  A.rank1 = rank1;
  A.slot_scale = slot_scale;
  for (int i = 0; i < num_sites; ++i) A.scale[i] = scale[i];
  const int nv = num_sites + num_slots;
  const unsigned gx = (unsigned)ceil_div(K, mi::kFinK);
  const unsigned gy = num_sites == 1 ? (unsigned)nv : 1u;
  if (scratch != nullptr && mi_finalize_scratch_bytes(nseg, K, nv) != 0 && rank1 == 0) {
    // long segment lists: chunks of segments in parallel, then the chunk sums
    const int64_t nchunk = ceil_div(nseg, mi::kFinChunk);
    hipLaunchKernelGGL(mi::k_finalize_chunks, dim3(gx, (unsigned)nv, (unsigned)nchunk),
                       dim3(mi::kFinK * mi::kFinG), 0, stream, part, nseg, K, scratch);
    hipLaunchKernelGGL(mi::k_finalize<double>, dim3(gx, gy), dim3(mi::kFinK * mi::kFinG), 0,
                       stream, scratch, nchunk, K, A, total, site_lp, slot_grad);
  } else {
    hipLaunchKernelGGL(mi::k_finalize<float>, dim3(gx, gy), dim3(mi::kFinK * mi::kFinG), 0,
                       stream, part, nseg, K, A, total, site_lp, slot_grad);
  }
  return to_code(hipGetLastError());
}

extern "C" {

int mi_abi_version(char* target, size_t target_bytes) {
  const char name[] = "gfx950";
  if (target != nullptr && target_bytes > 0) {
    size_t n = 0;
    for (; n + 1 < target_bytes && name[n] != '\0'; ++n) target[n] = name[n];
    target[n] = '\0';
  }
  return MI_ABI_VERSION;
}

int mi_wall_clock_khz(int* khz) {
  if (khz == nullptr) return MI_EINVAL;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(khz, hipDeviceAttributeWallClockRate, dev);
  return to_code(e);
}

int mi_struct_sizes(size_t* operand, size_t* site, size_t* group) {
  if (operand == nullptr || site == nullptr || group == nullptr) return MI_EINVAL;
  *operand = sizeof(mi_operand);
  *site = sizeof(mi_site);
  *group = sizeof(mi_group);
  return 0;
}

int mi_group_side_supported(const mi_group* group, int* supported) {
  if (!validate_group(group) || supported == nullptr) return MI_EINVAL;
  const Plan p = make_plan(group);
  *supported = (p.shape == kBcast && bcast_smem(group)) ? 1 : 0;
  return 0;
}

int mi_group_prior_supported(const mi_group* group, int* supported) {
  if (!validate_group(group) || supported == nullptr) return MI_EINVAL;
  const Plan p = make_plan(group);
  // the BCAST kernel's one site, or a fused-draw site program's site 0 (evaluated at its
  // block-row flush); either way on site 0's per-particle parameter, an operand (stride_i == 0)
  const int o = group->sites[0].operand[0];
  const bool host = (p.shape == kBcast && bcast_smem(group) && group->num_sites == 1) ||
                    (p.shape == kRow && p.draw && draw_supported(group) && mi_jit_enabled());
  *supported = (host && o >= 0 && group->operands[o].stride_i == 0 &&
                group->operands[o].stride_k != 0 &&
                group->prior.scale == group->sites[0].scale) ? 1 : 0;
  return 0;
}

int mi_group_pdraw_supported(const mi_group* group, int* supported) {
  if (!validate_group(group) || supported == nullptr) return MI_EINVAL;
  const Plan p = make_plan(group);
  // a fused-draw site program (row shape, block-row partials) whose particle block fits the
  // program's LDS table of per-particle values
  *supported = (p.shape == kRow && p.draw && draw_supported(group) && mi_jit_enabled() &&
                p.rows_per_block <= kPdrawMax) ? 1 : 0;
  return 0;
}

int mi_group_workspace_bytes(const mi_group* group, size_t* bytes) {
  if (!validate_group(group) || bytes == nullptr) return MI_EINVAL;
  const Plan p = make_plan(group);
  *bytes = workspace_bytes(group, p);
  return 0;
}

int mi_group_forward(const mi_group* group, void* workspace, size_t workspace_bytes, float* total,
                     double* site_lp, float* slot_grad, uint32_t* flags, void* stream) {
  return mi_group_forward_deferred(group, workspace, workspace_bytes, total, site_lp, slot_grad,
                                   flags, nullptr, nullptr, stream, nullptr);
}

int mi_group_forward_deferred(const mi_group* group, void* workspace, size_t workspace_bytes,
                              float* total, double* site_lp, float* slot_grad, uint32_t* flags,
                              void* start_event, void* stop_event, void* stream,
                              mi_reduce* reduce) {
  if (reduce != nullptr) *reduce = mi_reduce{};
  if (!validate_group(group) || total == nullptr || flags == nullptr) return MI_EINVAL;
  if (group->num_slots > 0 && slot_grad == nullptr) return MI_EINVAL;
  if (start_event != nullptr || stop_event != nullptr) {   // eager timing only (internal.hpp)
    bool capturing = false;
    const hipError_t ce = mi_stream_capturing(static_cast<hipStream_t>(stream), &capturing);
    if (ce != hipSuccess) return to_code(ce);
    if (capturing) return MI_EUNSUPPORTED;
  }
  const Plan p = make_plan(group);
  if (workspace_bytes < ::workspace_bytes(group, p) || workspace == nullptr) return MI_EWORKSPACE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  float* part = static_cast<float*>(workspace);
  hipError_t e = hipSuccess;
  if (!(group->options & MI_GROUP_FLAGS_ZEROED)) {
    e = hipMemsetAsync(flags, 0, sizeof(uint32_t) * group->num_sites, s);
    if (e == hipSuccess && group->prior.present != 0)
      e = hipMemsetAsync(group->prior.flags, 0, sizeof(uint32_t), s);
    if (e != hipSuccess) return to_code(e);
  }
  const mi_group G = *group;
  // Without a per-site output the specialised kernels reduce one weighted log-joint value per
  // particle instead of one per site.
  const bool combined = site_lp == nullptr;
  int reduced_lp = G.num_sites;
  bool prescaled = false;  // partials already carry the site scales
  int64_t prows = p.nseg;   // partial rows written (fused-draw programs: one per block)
  float* prep = reinterpret_cast<float*>(static_cast<char*>(workspace) + prep_offset(group, p));
  if (group->draw.operand != 0 && (p.shape != kRow || !draw_supported(group))) return MI_EUNSUPPORTED;
  if (group->side.out != nullptr && !(p.shape == kBcast && bcast_smem(group))) return MI_EUNSUPPORTED;
  if (group->prior.present != 0) {
    int ok = 0;
    mi_group_prior_supported(group, &ok);
    if (!ok || (p.shape == kRow && !combined)) return MI_EUNSUPPORTED;
  }
  if (group->pdraw.operand != 0) {
    int ok = 0;
    mi_group_pdraw_supported(group, &ok);
    if (!ok) return MI_EUNSUPPORTED;
  }
  float* draw_partials = draw_partial_floats(group, p) != 0 ? prep : nullptr;
  const bool smem = p.shape == kBcast && bcast_smem(group);
  if (p.shape == kBcast && !smem) {
    const dim3 pg((unsigned)ceil_div(G.K, 256));
    switch (G.sites[0].family) {
      case MI_BERNOULLI_LOGITS:
        hipLaunchKernelGGL((mi::k_bcast_prep<MI_BERNOULLI_LOGITS>), pg, dim3(256), 0, s, G, prep, flags);
        break;
      case MI_BERNOULLI_PROBS:
        hipLaunchKernelGGL((mi::k_bcast_prep<MI_BERNOULLI_PROBS>), pg, dim3(256), 0, s, G, prep, flags);
        break;
      case MI_NORMAL:
        hipLaunchKernelGGL((mi::k_bcast_prep<MI_NORMAL>), pg, dim3(256), 0, s, G, prep, flags);
        break;
      case MI_BETA:
        hipLaunchKernelGGL((mi::k_bcast_prep<MI_BETA>), pg, dim3(256), 0, s, G, prep, flags);
        break;
      default: return MI_EUNSUPPORTED;
    }
  }
  if (start_event != nullptr) {
    e = mi_record_event(start_event, s);
    if (e != hipSuccess) return to_code(e);
  }
  switch (p.shape) {
    case kBcast: {
      const bool masked = G.sites[0].mask != nullptr;
      if (smem) {
        if (G.sites[0].family == MI_BERNOULLI_PROBS)
          launch_smem<MI_BERNOULLI_PROBS>(G, p, part, flags, s);
        else
          launch_smem<MI_BERNOULLI_LOGITS>(G, p, part, flags, s);
        break;
      }
      switch (G.sites[0].family) {
#define MI_LAUNCH_BCAST(FAM)                                                                   \
  case FAM:                                                                                    \
    if (masked)                                                                                \
      hipLaunchKernelGGL((mi::k_site_bcast<FAM, true>), p.grid, dim3(mi::kBcastThreads), 0, s,         \
                         G, prep, part, p.nseg, flags);                                        \
    else                                                                                       \
      hipLaunchKernelGGL((mi::k_site_bcast<FAM, false>), p.grid, dim3(mi::kBcastThreads), 0,             \
                         s, G, prep, part, p.nseg, flags);                                     \
    break;
        MI_LAUNCH_BCAST(MI_BERNOULLI_LOGITS)
        MI_LAUNCH_BCAST(MI_BERNOULLI_PROBS)
        MI_LAUNCH_BCAST(MI_NORMAL)
        MI_LAUNCH_BCAST(MI_BETA)
#undef MI_LAUNCH_BCAST
        default: return MI_EUNSUPPORTED;
      }
      break;
    }
    case kRow:
    case kCol: {
      const PlanInfo info = plan_info(p, combined);
      mi_group GK = G;
      if (draw_partials != nullptr) {  // per-K-block partials, summed below
        GK.draw.dloc = draw_partials;
        GK.draw.dscale = draw_partials + (size_t)p.grid.y * G.N;
      }
      const int rc = mi_jit_launch(GK, info, part, p.nseg,
                                   p.shape == kRow ? p.rows_per_block : p.seg_len, flags, s);
      if (rc < 0) return -rc;
      if (rc == 0) {
        prescaled = combined;
        reduced_lp = combined ? 1 : G.num_sites;
        if (info.block_rows) prows = (int64_t)p.grid.x;
        break;
      }
      if (G.draw.operand != 0) return MI_EUNSUPPORTED;  // fused draws need the specialised kernel
      if (p.shape == kRow) {
        const int e = p.elems;
        if (e == 4)
          hipLaunchKernelGGL((mi::k_group_row<4>), p.grid, dim3(256), 0, s, G, part, p.nseg,
                             p.rows_per_block, flags);
        else if (e == 16)
          hipLaunchKernelGGL((mi::k_group_row<16>), p.grid, dim3(256), 0, s, G, part, p.nseg,
                             p.rows_per_block, flags);
        else
          hipLaunchKernelGGL((mi::k_group_row<8>), p.grid, dim3(256), 0, s, G, part, p.nseg,
                             p.rows_per_block, flags);
      } else
        hipLaunchKernelGGL(mi::k_group_col, p.grid, dim3(256), 0, s, G, part, p.nseg, p.seg_len,
                           p.kw, flags);
      break;
    }
  }
  e = hipGetLastError();
  if (e != hipSuccess) return to_code(e);
  if (stop_event != nullptr) {
    e = mi_record_event(stop_event, s);
    if (e != hipSuccess) return to_code(e);
  }
  if (draw_partials != nullptr && !(G.options & MI_GROUP_DRAW_PARTIALS)) {
    hipLaunchKernelGGL(mi::k_draw_reduce, dim3((unsigned)ceil_div(G.N, 256)), dim3(256), 0, s,
                       draw_partials, (int64_t)p.grid.y, G.N, G.draw.dloc, G.draw.dscale);
    e = hipGetLastError();
    if (e != hipSuccess) return to_code(e);
  }
  double scales[MI_MAX_SITES];
  for (int i = 0; i < reduced_lp; ++i) scales[i] = prescaled ? 1.0 : G.sites[i].scale;
  // values in the rank-one layout: the slot of a k_site_bcast_smem launch (after the site value)
  const int rank1_mask = (smem && smem_rank1(group, p)) ? (1 << reduced_lp) : 0;
  if (reduce != nullptr && prows <= MI_REDUCE_MAX_SEG) {   // the caller runs the finalize
    reduce->part = part;
    reduce->nseg = prows;
    reduce->K = G.K;
    reduce->num_sites = reduced_lp;
    reduce->num_slots = G.num_slots;
    reduce->rank1 = rank1_mask;
    for (int i = 0; i < reduced_lp; ++i) reduce->scale[i] = scales[i];
    reduce->slot_scale = (double)G.grad_scale;
    reduce->total = total;
    reduce->site_lp = site_lp;
    reduce->slot_grad = slot_grad;
    return 0;
  }
  double* scratch = reinterpret_cast<double*>(static_cast<char*>(workspace) +
                                              finalize_offset(group, p));
  return mi_launch_finalize(part, prows, G.K, reduced_lp, G.num_slots, scales,
                            (double)G.grad_scale, total, site_lp, slot_grad, scratch, s,
                            rank1_mask);
}

int mi_reduce_launch(const mi_reduce* r, void* stream) {
  if (r == nullptr || r->part == nullptr || r->nseg < 1 || r->K < 1 || r->total == nullptr ||
      r->num_sites < 1 || r->num_sites > MI_MAX_SITES || r->num_slots < 0 ||
      (r->num_slots > 0 && r->slot_grad == nullptr) || r->nseg > MI_REDUCE_MAX_SEG)
    return MI_EINVAL;
  // nseg <= MI_REDUCE_MAX_SEG: the one-launch finalize (no chunk scratch)
  return mi_launch_finalize(r->part, r->nseg, r->K, r->num_sites, r->num_slots, r->scale,
                            r->slot_scale, r->total, r->site_lp, r->slot_grad, nullptr,
                            static_cast<hipStream_t>(stream), r->rank1);
}

int mi_group_draw_partials(const mi_group* group, size_t* offset_bytes, int64_t* rows) {
  if (!validate_group(group) || offset_bytes == nullptr || rows == nullptr) return MI_EINVAL;
  if (!(group->options & MI_GROUP_DRAW_PARTIALS)) return MI_EINVAL;
  const Plan p = make_plan(group);
  if (draw_partial_floats(group, p) == 0) return MI_EINVAL;
  *offset_bytes = prep_offset(group, p);
  *rows = (int64_t)p.grid.y;
  return 0;
}

int mi_group_source(const mi_group* group, char* out, size_t out_bytes, size_t* needed) {
  if (!validate_group(group)) return MI_EINVAL;
  const Plan p = make_plan(group);
  std::string text;
  if (p.shape == kBcast) text = "// BCAST shape: precompiled k_site_bcast\n";
  else text = mi_jit_source(*group, plan_info(p, true));
  if (needed != nullptr) *needed = text.size() + 1;
  if (out != nullptr && out_bytes > 0) {
    const size_t n = std::min(out_bytes - 1, text.size());
    std::memcpy(out, text.data(), n);
    out[n] = '\0';
  }
  return 0;
}

int mi_group_compile_check(const mi_group* group, char* log, size_t log_bytes) {
  if (!validate_group(group)) return MI_EINVAL;
  const Plan p = make_plan(group);
  if (p.shape == kBcast) return 0;
  std::string text;
  const bool ok = mi_jit_compile_check(*group, plan_info(p, true), &text) &&
                  mi_jit_compile_check(*group, plan_info(p, false), &text);
  if (log != nullptr && log_bytes > 0) {
    const size_t n = std::min(log_bytes - 1, text.size());
    std::memcpy(log, text.data(), n);
    log[n] = '\0';
  }
  return ok ? 0 : MI_EUNSUPPORTED;
}

int mi_scale_rows(float* x, int64_t stride_k, int64_t stride_i, int64_t K, int64_t N,
                  const float* g, float g0, void* stream) {
  if (x == nullptr || g == nullptr || K < 1 || N < 1 || g0 == 0.0f) return MI_EINVAL;
  const int64_t rows = 64;
  dim3 grid((unsigned)ceil_div(N, 256), (unsigned)ceil_div(K, rows));
  hipLaunchKernelGGL(mi::k_scale_rows, grid, dim3(256), 0, static_cast<hipStream_t>(stream), x,
                     stride_k, stride_i, K, N, g, g0, rows);
  return to_code(hipGetLastError());
}

int mi_categorical_workspace_bytes(int64_t K, int64_t N, size_t* bytes) {
  if (K < 1 || N < 1 || bytes == nullptr) return MI_EINVAL;
  *bytes = (size_t)ceil_div(N, 1024) * (size_t)K * sizeof(float);
  return 0;
}

int mi_categorical_forward(const float* logits, int64_t stride_k, int64_t stride_i,
                           int64_t stride_c, int64_t K, int64_t N, int64_t C,
                           const int64_t* value, int64_t value_stride_k, int64_t value_stride_i,
                           const uint8_t* mask, int64_t mask_stride_i, double scale, float g0,
                           float* dlogits, void* workspace, size_t workspace_bytes, float* total,
                           uint32_t* flags, void* stream) {
  if (logits == nullptr || value == nullptr || total == nullptr || flags == nullptr || K < 1 ||
      N < 1 || C < 1)
    return MI_EINVAL;
  size_t need = 0;
  mi_categorical_workspace_bytes(K, N, &need);
  if (workspace == nullptr || workspace_bytes < need) return MI_EWORKSPACE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e = hipMemsetAsync(flags, 0, sizeof(uint32_t), s);
  if (e != hipSuccess) return to_code(e);
  const int64_t nseg = ceil_div(N, 1024);
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(mi::k_categorical, dim3((unsigned)ceil_div(nseg, 4), (unsigned)K), dim3(256),
                     0, s, logits, stride_k, stride_i, stride_c, K, N, C, value, value_stride_k,
                     value_stride_i, mask, mask_stride_i, (float)(g0 * scale), dlogits, part, nseg,
                     flags);
  e = hipGetLastError();
  if (e != hipSuccess) return to_code(e);
  hipLaunchKernelGGL(mi::k_categorical_finalize, dim3((unsigned)ceil_div(K, 256)), dim3(256), 0, s,
                     part, nseg, K, scale, total);
  return to_code(hipGetLastError());
}

}  // extern "C"
