// Reparameterised guide sampling and its backward, for the mean-field Normal and Beta guide factors.
//
// Replaces FactorizedDistribution.rsample (mininf/nn.py:133-145) for those families, i.e.
// torch Normal.rsample (torch/distributions/normal.py:83-86: loc + eps * scale) and Beta.rsample
// (beta.py:85-86 -> dirichlet.py:23-36, 85-88: normalised gamma draws), plus the gradients autograd
// would compute through them (Normal: d/dloc, d/dscale; Beta: the implicit reparameterisation
// gradient torch._dirichlet_grad, ATen/native/Distributions.h dirichlet_grad_one).
//
// Layout: draws are written row-major z[k, i] (particles x elements) so that the site kernels read
// them with unit stride along elements. eps is never stored: the backward regenerates it from the
// Philox counter (seed, step, stream, global particle, element quad).
#include "beta_grad.hpp"

#include <algorithm>

namespace mi {

constexpr int kGuideThreads = 256;

// -------------------------------------------------------------------------------------------------
// Normal
// -------------------------------------------------------------------------------------------------
// EXP: `scale` holds the unconstrained parameter; the scale is expf of it (as
// k_transform_params) and the first row block writes it to scale_out (same strides).
template <bool EXP>
__global__ __launch_bounds__(kGuideThreads) void k_normal_rsample(
    const float* __restrict__ loc, int64_t loc_s, const float* __restrict__ scale, int64_t scale_s,
    int64_t K, int64_t N, uint64_t seed, uint64_t step, const uint64_t* __restrict__ step_dev,
    uint32_t stream_id, int64_t poff, int64_t qoff, const float* __restrict__ eps_in,
    float* __restrict__ z, int64_t rows_per_block, float* __restrict__ scale_out) {
  if (step_dev != nullptr) step += *step_dev;
  const int64_t quad = (int64_t)blockIdx.x * kGuideThreads + threadIdx.x;
  const int64_t i0 = quad * 4;
  if (i0 >= N) return;
  const int64_t k0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t k1 = min(K, k0 + rows_per_block);
  float m[4], sd[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t i = min(i0 + j, N - 1);
    m[j] = loc[i * loc_s];
    sd[j] = EXP ? expf(scale[i * scale_s]) : scale[i * scale_s];
    if (EXP && blockIdx.y == 0 && i0 + j < N) scale_out[(i0 + j) * scale_s] = sd[j];
  }
  const bool full = (i0 + 4 <= N) && ((N & 3) == 0);
  for (int64_t k = k0; k < k1; ++k) {
    float e[4];
    if (eps_in != nullptr) {
#pragma unroll
      for (int j = 0; j < 4; ++j) e[j] = (i0 + j < N) ? eps_in[k * N + i0 + j] : 0.0f;
    } else {
      guide_normals(seed, step, stream_id, (uint64_t)(qoff + quad), (uint64_t)(poff + k), e);
    }
    float out[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) out[j] = fmaf(e[j], sd[j], m[j]);
    if (full) {
      *reinterpret_cast<float4*>(z + k * N + i0) = make_float4(out[0], out[1], out[2], out[3]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (i0 + j < N) z[k * N + i0 + j] = out[j];
    }
  }
}

// Backward of the Normal draw, reduced over particles. A block is TI quad-lanes x TK particle-lanes
// (TI * TK = 256, TI = min(64, quads)): coalesced along elements for large N, and still 256-wide for
// N = 1 (a scalar guide factor with thousands of particles). Each block covers one slice of the
// particles; per-block sums are combined in a fixed order through LDS and written per slice.
__global__ __launch_bounds__(kGuideThreads) void k_normal_rsample_bwd(
    const float* __restrict__ dz, int64_t dz_sk, int64_t dz_si, int64_t K, int64_t N,
    uint64_t seed, uint64_t step, const uint64_t* __restrict__ step_dev, uint32_t stream_id,
    int64_t poff, int64_t qoff, const float* __restrict__ eps_in, float* __restrict__ out_loc,
    float* __restrict__ out_scale, int64_t out_stride, int64_t rows_per_block, int ti) {
  if (step_dev != nullptr) step += *step_dev;
  __shared__ float red[kGuideThreads][8];
  const int tx = threadIdx.x % ti, ty = threadIdx.x / ti, tk = kGuideThreads / ti;
  const int64_t quad = (int64_t)blockIdx.x * ti + tx;
  const int64_t i0 = quad * 4;
  const int64_t k0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t k1 = min(K, k0 + rows_per_block);
  float sl[4] = {0.f, 0.f, 0.f, 0.f}, ss[4] = {0.f, 0.f, 0.f, 0.f};
  if (i0 < N) {
    const bool vec = (dz_si == 1) && (i0 + 4 <= N) && ((N & 3) == 0) && ((dz_sk & 3) == 0) &&
                     ((reinterpret_cast<uintptr_t>(dz) & 15) == 0);
    for (int64_t k = k0 + ty; k < k1; k += tk) {
      float g[4];
      if (vec) {
        const float4 v = *reinterpret_cast<const float4*>(dz + k * dz_sk + i0);
        g[0] = v.x; g[1] = v.y; g[2] = v.z; g[3] = v.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) g[j] = (i0 + j < N) ? dz[k * dz_sk + (i0 + j) * dz_si] : 0.0f;
      }
      float e[4];
      if (eps_in != nullptr) {
#pragma unroll
        for (int j = 0; j < 4; ++j) e[j] = (i0 + j < N) ? eps_in[k * N + i0 + j] : 0.0f;
      } else {
        guide_normals(seed, step, stream_id, (uint64_t)(qoff + quad), (uint64_t)(poff + k), e);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sl[j] += g[j];
        ss[j] = fmaf(g[j], e[j], ss[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[threadIdx.x][j] = sl[j];
    red[threadIdx.x][4 + j] = ss[j];
  }
  __syncthreads();
  if (ty == 0 && i0 < N) {
    float tl[4] = {0.f, 0.f, 0.f, 0.f}, ts[4] = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < tk; ++r) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        tl[j] += red[r * ti + tx][j];
        ts[j] += red[r * ti + tx][4 + j];
      }
    }
    const int64_t slice = blockIdx.y;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (i0 + j < N) {
        out_loc[slice * out_stride + i0 + j] = tl[j];
        out_scale[slice * out_stride + i0 + j] = ts[j];
      }
    }
  }
}

// Sum the `slices` rows of two [slices, N] partial arrays (fixed order, fp64) into out_a[i * sa]
// and out_b[i * sb].
__global__ __launch_bounds__(kGuideThreads) void k_sum_slices(const float* __restrict__ part_a,
                                                              const float* __restrict__ part_b,
                                                              int64_t slices, int64_t N,
                                                              float* __restrict__ out_a, int64_t sa,
                                                              float* __restrict__ out_b,
                                                              int64_t sb) {
  const int64_t i = (int64_t)blockIdx.x * kGuideThreads + threadIdx.x;
  if (i >= N) return;
  double a = 0.0, b = 0.0;
  for (int64_t s = 0; s < slices; ++s) {
    a += (double)part_a[s * N + i];
    b += (double)part_b[s * N + i];
  }
  out_a[i * sa] = (float)a;
  out_b[i * sb] = (float)b;
}

// -------------------------------------------------------------------------------------------------
// Beta via two Marsaglia-Tsang gamma variates (G. Marsaglia, W. W. Tsang, "A simple method for
// generating gamma variables", ACM TOMS 26(3), 2000), with the alpha < 1 boost
// G(alpha) = G(alpha + 1) * U^(1/alpha).
// -------------------------------------------------------------------------------------------------
struct Stream {
  uint64_t seed, step;
  uint32_t stream_id, sub;
  uint64_t elem, particle;
  uint32_t block = 0;
  U4 bits{};
  int used = 4;
  MI_DEV uint32_t next() {
    if (used == 4) {
      U4 c{(uint32_t)elem, (uint32_t)particle, (uint32_t)step ^ (uint32_t)(step >> 32),
           (stream_id << 8) | (sub << 6) | (block & 63u)};
      bits = philox4x32<kGuideRounds>(c, (uint32_t)seed, (uint32_t)(seed >> 32));
      ++block;
      used = 0;
    }
    const uint32_t out = used == 0 ? bits.x : used == 1 ? bits.y : used == 2 ? bits.z : bits.w;
    ++used;
    return out;
  }
  MI_DEV float uniform() { return u01(next()); }
  MI_DEV float normal() {
    float a, b;
    box_muller(next(), next(), a, b);
    return a;
  }
};

MI_DEV float sample_gamma(float alpha, Stream& rng) {
  float boost = 1.0f;
  if (!(alpha > 0.0f)) return 0.0f;
  if (alpha < 1.0f) {
    boost = powf(rng.uniform(), 1.0f / alpha);
    alpha += 1.0f;
  }
  const float d = alpha - 1.0f / 3.0f;
  const float c = 1.0f / sqrtf(9.0f * d);
  for (int attempt = 0; attempt < 64; ++attempt) {
    float x, y;
    int tries = 0;
    do {
      x = rng.normal();
      y = 1.0f + c * x;
    } while (y <= 0.0f && ++tries < 16);
    if (y <= 0.0f) continue;
    const float v = y * y * y;
    const float u = rng.uniform();
    const float xx = x * x;
    if (u < 1.0f - 0.0331f * xx * xx) return boost * d * v;
    if (logf(u) < 0.5f * xx + d * (1.0f - v + logf(v))) return boost * d * v;
  }
  return boost * d;  // not reached in practice (acceptance > 95 % per attempt)
}

// EXP: c1 / c0 hold the unconstrained parameters; the concentrations are expf of them (as
// k_transform_params) and the k = 0 threads write them to conc[i, 0..1].
// Two lanes per draw: the even lane samples g1 (sub-stream 0), the odd lane g0 (sub-stream 1) --
// the two rejection loops run side by side instead of one after the other (the draw is a short
// latency-bound launch); the pair exchanges its variates and the even lane writes x = g1 / (g1 + g0).
template <bool EXP>
__global__ __launch_bounds__(kGuideThreads) void k_beta_rsample(
    const float* __restrict__ c1, int64_t c1_s, const float* __restrict__ c0, int64_t c0_s,
    int64_t K, int64_t N, uint64_t seed, uint64_t step, const uint64_t* __restrict__ step_dev,
    uint32_t stream_id, int64_t poff, const float* __restrict__ x_in, float* __restrict__ x,
    float* __restrict__ conc) {
  const int64_t t = (int64_t)blockIdx.x * kGuideThreads + threadIdx.x;
  if (t >= 2 * K * N) return;   // (whole pairs: the bound is even)
  const int64_t d = t >> 1;
  const uint32_t side = (uint32_t)(t & 1);
  const int64_t k = d / N, i = d - k * N;
  const float a = EXP ? expf(c1[i * c1_s]) : c1[i * c1_s];
  const float b = EXP ? expf(c0[i * c0_s]) : c0[i * c0_s];
  if (EXP && k == 0 && side == 0) {
    conc[2 * i] = a;
    conc[2 * i + 1] = b;
  }
  if (x_in != nullptr) {
    if (side == 0) x[d] = x_in[d];
    return;
  }
  if (step_dev != nullptr) step += *step_dev;
  Stream rng{seed, step, stream_id, side, (uint64_t)i, (uint64_t)(poff + k)};
  const float g = sample_gamma(side == 0 ? a : b, rng);
  const float other = __shfl_xor(g, 1, kWave);
  if (side == 0) {
    const float g1 = g, g0 = other;
    const float s = g1 + g0;
    x[d] = s > 0.0f ? g1 / s : (a >= b ? 1.0f : 0.0f);
  }
}

__global__ __launch_bounds__(kGuideThreads) void k_beta_rsample_bwd(
    const float* __restrict__ dx, int64_t dx_sk, int64_t dx_si, const float* __restrict__ x,
    const float* __restrict__ c1, int64_t c1_s, const float* __restrict__ c0, int64_t c0_s,
    int64_t K, int64_t N, float* __restrict__ out1, int64_t o1_s, float* __restrict__ out0,
    int64_t o0_s, int64_t out_stride, int64_t rows_per_block, int ti) {
  __shared__ double red[kGuideThreads][2];
  const int tx = threadIdx.x % ti, ty = threadIdx.x / ti, tk = kGuideThreads / ti;
  const int64_t i = (int64_t)blockIdx.x * ti + tx;
  const int64_t k0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t k1 = min(K, k0 + rows_per_block);
  double s1 = 0.0, s0 = 0.0;
  if (i < N) {
    const float a = c1[i * c1_s], b = c0[i * c0_s];
    const float tot = a + b;  // concentration.sum(-1) in fp32, dirichlet.py:18
    const double psi_a = digamma((double)a), psi_b = digamma((double)b);
    const double psi_t = digamma((double)tot);
    for (int64_t k = k0 + ty; k < k1; k += tk) {
      const float g = dx[k * dx_sk + i * dx_si];
      if (g == 0.0f) continue;
      const float xv = x[k * N + i];
      const float xw = 1.0f - xv;
      // _Dirichlet_backward: grad_j * (go_j - sum(x * go)) with go = (g, 0)
      s1 += dirichlet_grad(xv, a, tot, psi_a, psi_t) * (double)g * (double)(1.0f - xv);
      s0 -= dirichlet_grad(xw, b, tot, psi_b, psi_t) * (double)g * (double)xv;
    }
  }
  red[threadIdx.x][0] = s1;
  red[threadIdx.x][1] = s0;
  __syncthreads();
  if (ty == 0 && i < N) {
    double t1 = 0.0, t0 = 0.0;
    for (int r = 0; r < tk; ++r) {
      t1 += red[r * ti + tx][0];
      t0 += red[r * ti + tx][1];
    }
    out1[blockIdx.y * out_stride + i * o1_s] = (float)t1;
    out0[blockIdx.y * out_stride + i * o0_s] = (float)t0;
  }
}

// Gamma(concentration, rate) draws (gamma.py:80-88): x = standard_gamma(concentration) / rate,
// clamped below at the smallest normal float as torch does. The standard draws g are kept for the
// backward (torch saves them as _standard_gamma's result). Injected g (parity mode) replaces the
// generator.
__global__ __launch_bounds__(kGuideThreads) void k_gamma_rsample(
    const float* __restrict__ conc, int64_t conc_s, const float* __restrict__ rate, int64_t rate_s,
    int64_t K, int64_t N, uint64_t seed, uint64_t step, const uint64_t* __restrict__ step_dev,
    uint32_t stream_id, int64_t poff, const float* __restrict__ g_in, float* __restrict__ g_out,
    float* __restrict__ x) {
  const int64_t t = (int64_t)blockIdx.x * kGuideThreads + threadIdx.x;
  if (t >= K * N) return;
  const int64_t k = t / N, i = t - k * N;
  float g;
  if (g_in != nullptr) {
    g = g_in[t];
  } else {
    if (step_dev != nullptr) step += *step_dev;
    Stream r{seed, step, stream_id, 2u, (uint64_t)i, (uint64_t)(poff + k)};
    g = sample_gamma(conc[i * conc_s], r);
  }
  g_out[t] = g;
  x[t] = fmaxf(g / rate[i * rate_s], 1.17549435e-38f);
}

// Backward of k_gamma_rsample for upstream dx, reduced over particle rows [k0, k1) per element:
//   d concentration = sum_k (dx / rate) * standard_gamma_grad(concentration, g)
//   d rate          = sum_k -dx * g / rate^2
// (autograd of `_standard_gamma(c) / r`: div backward, then _standard_gamma's backward).
__global__ __launch_bounds__(kGuideThreads) void k_gamma_rsample_bwd(
    const float* __restrict__ dx, int64_t dx_sk, int64_t dx_si, const float* __restrict__ g,
    const float* __restrict__ conc, int64_t conc_s, const float* __restrict__ rate,
    int64_t rate_s, int64_t K, int64_t N, float* __restrict__ out_c, int64_t oc_s,
    float* __restrict__ out_r, int64_t or_s, int64_t out_stride, int64_t rows_per_block, int ti) {
  __shared__ double red[kGuideThreads][2];
  const int tx = threadIdx.x % ti, ty = threadIdx.x / ti, tk = kGuideThreads / ti;
  const int64_t i = (int64_t)blockIdx.x * ti + tx;
  const int64_t k0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t k1 = min(K, k0 + rows_per_block);
  double sc = 0.0, sr = 0.0;
  if (i < N) {
    const float a = conc[i * conc_s], r = rate[i * rate_s];
    for (int64_t k = k0 + ty; k < k1; k += tk) {
      const float d = dx[k * dx_sk + i * dx_si];
      if (d == 0.0f) continue;
      const float gv = g[k * N + i];
      const float dg = d / r;                       // grad of the standard draw (fp32, as torch)
      sc += (double)(dg * (float)standard_gamma_grad((double)a, (double)gv));
      sr += (double)(-d * gv / (r * r));
    }
  }
  red[threadIdx.x][0] = sc;
  red[threadIdx.x][1] = sr;
  __syncthreads();
  if (ty == 0 && i < N) {
    double tc = 0.0, tr = 0.0;
    for (int q = 0; q < tk; ++q) {
      tc += red[q * ti + tx][0];
      tr += red[q * ti + tx][1];
    }
    out_c[blockIdx.y * out_stride + i * oc_s] = (float)tc;
    out_r[blockIdx.y * out_stride + i * or_s] = (float)tr;
  }
}

// Per-draw implicit-gradient factors of Beta draws, independent of the upstream gradient:
//   out[(k N + i) 2 + 0] =  dgrad(x, a, a+b) (1 - x),  out[... + 1] = -dgrad(1 - x, b, a+b) x
// so that sum_k dx[k,i] out[k,i,j] is mi_beta_rsample_backward's dc1 / dc0. One thread per
// (draw, component): the fp64 chains (digammas, dirichlet_grad) are the whole cost, and they depend
// only on the draw, so this launch can run beside the site kernels that produce dx.
__global__ __launch_bounds__(kGuideThreads) void k_beta_dgrad(
    const float* __restrict__ x, const float* __restrict__ c1, int64_t c1_s,
    const float* __restrict__ c0, int64_t c0_s, int64_t K, int64_t N, double* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * kGuideThreads + threadIdx.x;
  if (t >= 2 * K * N) return;
  const int j = (int)(t & 1);
  const int64_t e = t >> 1, i = e % N;
  const float a = c1[i * c1_s], b = c0[i * c0_s];
  const float tot = a + b;  // concentration.sum(-1) in fp32, dirichlet.py:18
  const double psi_t = digamma((double)tot);
  const float xv = x[e];
  if (j == 0) {
    out[t] = dirichlet_grad(xv, a, tot, digamma((double)a), psi_t) * (double)(1.0f - xv);
  } else {
    out[t] = -dirichlet_grad(1.0f - xv, b, tot, digamma((double)b), psi_t) * (double)xv;
  }
}

// Start of an ELBO step in one launch: snapshot[0] = counter[0] (the step the draws of this call use,
// read again by the backward's eps regeneration), counter[0] += 1 (the next call draws anew, also
// when replayed from a captured graph), flags[0 .. nflags) = 0 (the step's validation words).
__global__ __launch_bounds__(kGuideThreads) void k_step_begin(uint64_t* __restrict__ counter,
                                                              uint64_t* __restrict__ snapshot,
                                                              uint32_t* __restrict__ flags,
                                                              int64_t nflags) {
  const int64_t t = (int64_t)blockIdx.x * kGuideThreads + threadIdx.x;
  if (t == 0) {
    const uint64_t c = *counter;
    *snapshot = c;
    *counter = c + 1u;
  }
  if (t < nflags) flags[t] = 0u;
}

// Constrained guide parameters of one factor, interleaved: out[i * m + j] = T_j(u_j[i * stride_j])
// with T_j = exp (transform_to(positive), constraint_registry.py:184-189) or the identity.
__global__ __launch_bounds__(kGuideThreads) void k_transform_params(const mi_params P,
                                                                    float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * kGuideThreads + threadIdx.x;
  if (t >= P.n * P.m) return;
  const int64_t i = t / P.m;
  const int j = (int)(t - i * P.m);
  float u = 0.0f;
  int tr = MI_TRANSFORM_NONE;
#pragma unroll
  for (int q = 0; q < MI_MAX_PARAMS; ++q)
    if (q == j) {
      u = P.u[q][i * P.stride[q]];
      tr = P.transform[q];
    }
  out[t] = tr == MI_TRANSFORM_EXP ? expf(u) : u;
}

// Raw generator access for tests.
__global__ void k_philox_normal(int64_t K, int64_t N, uint64_t seed, uint64_t step,
                                uint32_t stream_id, int64_t poff, float* __restrict__ out) {
  const int64_t quad = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t k = blockIdx.y;
  if (quad * 4 >= N) return;
  float e[4];
  guide_normals(seed, step, stream_id, (uint64_t)quad, (uint64_t)(poff + k), e);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (quad * 4 + j < N) out[k * N + quad * 4 + j] = e[j];
}

__global__ void k_philox_raw(const uint32_t* __restrict__ ctr, int64_t count, uint32_t k0,
                             uint32_t k1, uint32_t* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= count) return;
  const U4 r = philox4x32_10(U4{ctr[4 * j], ctr[4 * j + 1], ctr[4 * j + 2], ctr[4 * j + 3]}, k0, k1);
  out[4 * j] = r.x;
  out[4 * j + 1] = r.y;
  out[4 * j + 2] = r.z;
  out[4 * j + 3] = r.w;
}

}  // namespace mi

namespace {

int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
int to_code(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

// Launch geometry of the particle-reducing backward kernels: `lanes` element lanes per block
// (TI), 256 / TI particle lanes, and enough particle slices to fill the chip.
struct BwdGeometry {
  int ti;
  int64_t gx, slices, rows;
};

BwdGeometry bwd_geometry(int64_t K, int64_t units) {
  BwdGeometry g{};
  int ti = 1;
  while (ti < 64 && ti < units) ti <<= 1;
  g.ti = ti;
  const int tk = 256 / ti;
  g.gx = ceil_div(units, ti);
  int64_t slices = ceil_div(1024, g.gx);
  slices = std::min<int64_t>(slices, ceil_div(K, (int64_t)tk * 2));
  slices = std::max<int64_t>(1, slices);
  g.rows = ceil_div(K, slices);
  g.slices = ceil_div(K, g.rows);
  return g;
}

}  // namespace

extern "C" {

int mi_normal_rsample(const float* loc, int64_t loc_stride, const float* scale, int64_t scale_stride,
                      int64_t K, int64_t N, uint64_t seed, uint64_t step,
                      const uint64_t* step_device, uint32_t stream_id, int64_t particle_offset,
                      int64_t element_offset, const float* eps, float* z, void* stream) {
  if (loc == nullptr || scale == nullptr || z == nullptr || K < 1 || N < 1 || stream_id > 0xFFFFFFu ||
      element_offset < 0 || (element_offset & 3) != 0)
    return MI_EINVAL;
  const int64_t gx = ceil_div(N, 4 * mi::kGuideThreads);
  const int64_t gy = std::max<int64_t>(1, std::min<int64_t>(K, ceil_div(2048, gx)));
  const int64_t rows = ceil_div(K, gy);
  hipLaunchKernelGGL(mi::k_normal_rsample<false>, dim3((unsigned)gx, (unsigned)ceil_div(K, rows)),
                     dim3(mi::kGuideThreads), 0, static_cast<hipStream_t>(stream), loc, loc_stride,
                     scale, scale_stride, K, N, seed, step, step_device, stream_id, particle_offset,
                     element_offset >> 2, eps, z, rows, nullptr);
  return to_code(hipGetLastError());
}

int mi_normal_rsample_exp(const float* loc, int64_t loc_stride, const float* u, int64_t u_stride,
                          float* scale_out, int64_t K, int64_t N, uint64_t seed, uint64_t step,
                          const uint64_t* step_device, uint32_t stream_id, int64_t particle_offset,
                          int64_t element_offset, const float* eps, float* z, void* stream) {
  if (loc == nullptr || u == nullptr || scale_out == nullptr || z == nullptr || K < 1 || N < 1 ||
      stream_id > 0xFFFFFFu || element_offset < 0 || (element_offset & 3) != 0)
    return MI_EINVAL;
  const int64_t gx = ceil_div(N, 4 * mi::kGuideThreads);
  const int64_t gy = std::max<int64_t>(1, std::min<int64_t>(K, ceil_div(2048, gx)));
  const int64_t rows = ceil_div(K, gy);
  hipLaunchKernelGGL(mi::k_normal_rsample<true>, dim3((unsigned)gx, (unsigned)ceil_div(K, rows)),
                     dim3(mi::kGuideThreads), 0, static_cast<hipStream_t>(stream), loc, loc_stride,
                     u, u_stride, K, N, seed, step, step_device, stream_id, particle_offset,
                     element_offset >> 2, eps, z, rows, scale_out);
  return to_code(hipGetLastError());
}

int mi_normal_rsample_backward_workspace_bytes(int64_t K, int64_t N, size_t* bytes) {
  if (K < 1 || N < 1 || bytes == nullptr) return MI_EINVAL;
  const BwdGeometry geo = bwd_geometry(K, ceil_div(N, 4));
  *bytes = geo.slices > 1 ? (size_t)geo.slices * 2 * (size_t)N * sizeof(float) : 0;
  return 0;
}

int mi_normal_rsample_backward(const float* dz, int64_t dz_stride_k, int64_t dz_stride_i,
                               int64_t K, int64_t N, uint64_t seed, uint64_t step,
                               const uint64_t* step_device, uint32_t stream_id,
                               int64_t particle_offset, int64_t element_offset, const float* eps,
                               void* workspace, size_t workspace_bytes, float* dloc, float* dscale,
                               void* stream) {
  if (dz == nullptr || dloc == nullptr || dscale == nullptr || K < 1 || N < 1 ||
      element_offset < 0 || (element_offset & 3) != 0)
    return MI_EINVAL;
  size_t need = 0;
  mi_normal_rsample_backward_workspace_bytes(K, N, &need);
  if (need > 0 && (workspace == nullptr || workspace_bytes < need)) return MI_EWORKSPACE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const BwdGeometry geo = bwd_geometry(K, ceil_div(N, 4));
  const int64_t rows = geo.rows, gy = geo.slices, gx = geo.gx;
  float* out_loc = dloc;
  float* out_scale = dscale;
  if (gy > 1) {
    out_loc = static_cast<float*>(workspace);
    out_scale = out_loc + gy * N;
  }
  hipLaunchKernelGGL(mi::k_normal_rsample_bwd, dim3((unsigned)gx, (unsigned)gy),
                     dim3(mi::kGuideThreads), 0, s, dz, dz_stride_k, dz_stride_i, K, N, seed, step,
                     step_device, stream_id, particle_offset, element_offset >> 2, eps, out_loc,
                     out_scale, N, rows, geo.ti);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || gy == 1) return to_code(e);
  const unsigned g = (unsigned)ceil_div(N, mi::kGuideThreads);
  hipLaunchKernelGGL(mi::k_sum_slices, dim3(g), dim3(mi::kGuideThreads), 0, s, out_loc, out_scale,
                     gy, N, dloc, (int64_t)1, dscale, (int64_t)1);
  return to_code(hipGetLastError());
}

int mi_beta_rsample(const float* c1, int64_t c1_stride, const float* c0, int64_t c0_stride,
                    int64_t K, int64_t N, uint64_t seed, uint64_t step,
                    const uint64_t* step_device, uint32_t stream_id, int64_t particle_offset,
                    const float* x_in, float* x, void* stream) {
  if (c1 == nullptr || c0 == nullptr || x == nullptr || K < 1 || N < 1 || stream_id > 0xFFFFFFu)
    return MI_EINVAL;
  hipLaunchKernelGGL(mi::k_beta_rsample<false>, dim3((unsigned)ceil_div(2 * K * N, mi::kGuideThreads)),
                     dim3(mi::kGuideThreads), 0, static_cast<hipStream_t>(stream), c1, c1_stride,
                     c0, c0_stride, K, N, seed, step, step_device, stream_id, particle_offset, x_in,
                     x, nullptr);
  return to_code(hipGetLastError());
}

int mi_beta_rsample_exp(const float* u1, int64_t u1_stride, const float* u0, int64_t u0_stride,
                        float* conc, int64_t K, int64_t N, uint64_t seed, uint64_t step,
                        const uint64_t* step_device, uint32_t stream_id, int64_t particle_offset,
                        const float* x_in, float* x, void* stream) {
  if (u1 == nullptr || u0 == nullptr || conc == nullptr || x == nullptr || K < 1 || N < 1 ||
      stream_id > 0xFFFFFFu)
    return MI_EINVAL;
  hipLaunchKernelGGL(mi::k_beta_rsample<true>, dim3((unsigned)ceil_div(2 * K * N, mi::kGuideThreads)),
                     dim3(mi::kGuideThreads), 0, static_cast<hipStream_t>(stream), u1, u1_stride,
                     u0, u0_stride, K, N, seed, step, step_device, stream_id, particle_offset, x_in,
                     x, conc);
  return to_code(hipGetLastError());
}

int mi_beta_rsample_backward_workspace_bytes(int64_t K, int64_t N, size_t* bytes) {
  if (K < 1 || N < 1 || bytes == nullptr) return MI_EINVAL;
  const BwdGeometry geo = bwd_geometry(K, N);
  *bytes = geo.slices > 1 ? (size_t)geo.slices * 2 * (size_t)N * sizeof(float) : 0;
  return 0;
}

int mi_beta_rsample_backward(const float* dx, int64_t dx_stride_k, int64_t dx_stride_i,
                             const float* x, const float* c1, int64_t c1_stride, const float* c0,
                             int64_t c0_stride, int64_t K, int64_t N, void* workspace,
                             size_t workspace_bytes, float* dc1, int64_t dc1_stride, float* dc0,
                             int64_t dc0_stride, void* stream) {
  if (dx == nullptr || x == nullptr || c1 == nullptr || c0 == nullptr || dc1 == nullptr ||
      dc0 == nullptr || K < 1 || N < 1)
    return MI_EINVAL;
  size_t need = 0;
  mi_beta_rsample_backward_workspace_bytes(K, N, &need);
  if (need > 0 && (workspace == nullptr || workspace_bytes < need)) return MI_EWORKSPACE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const BwdGeometry geo = bwd_geometry(K, N);
  const int64_t rows = geo.rows, gy = geo.slices;
  float* o1 = dc1;
  float* o0 = dc0;
  int64_t s1 = dc1_stride, s0 = dc0_stride;
  if (gy > 1) {
    o1 = static_cast<float*>(workspace);
    o0 = o1 + gy * N;
    s1 = s0 = 1;
  }
  hipLaunchKernelGGL(mi::k_beta_rsample_bwd, dim3((unsigned)geo.gx, (unsigned)gy),
                     dim3(mi::kGuideThreads), 0, s, dx, dx_stride_k, dx_stride_i, x, c1, c1_stride,
                     c0, c0_stride, K, N, o1, s1, o0, s0, N, rows, geo.ti);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || gy == 1) return to_code(e);
  const unsigned g = (unsigned)ceil_div(N, mi::kGuideThreads);
  hipLaunchKernelGGL(mi::k_sum_slices, dim3(g), dim3(mi::kGuideThreads), 0, s, o1, o0, gy, N, dc1,
                     dc1_stride, dc0, dc0_stride);
  return to_code(hipGetLastError());
}

int mi_gamma_rsample(const float* concentration, int64_t concentration_stride, const float* rate,
                     int64_t rate_stride, int64_t K, int64_t N, uint64_t seed, uint64_t step,
                     const uint64_t* step_device, uint32_t stream_id, int64_t particle_offset,
                     const float* g_in, float* g, float* x, void* stream) {
  if (concentration == nullptr || rate == nullptr || g == nullptr || x == nullptr || K < 1 ||
      N < 1 || stream_id > 0xFFFFFFu)
    return MI_EINVAL;
  hipLaunchKernelGGL(mi::k_gamma_rsample, dim3((unsigned)ceil_div(K * N, mi::kGuideThreads)),
                     dim3(mi::kGuideThreads), 0, static_cast<hipStream_t>(stream), concentration,
                     concentration_stride, rate, rate_stride, K, N, seed, step, step_device,
                     stream_id, particle_offset, g_in, g, x);
  return to_code(hipGetLastError());
}

int mi_gamma_rsample_backward_workspace_bytes(int64_t K, int64_t N, size_t* bytes) {
  return mi_beta_rsample_backward_workspace_bytes(K, N, bytes);   // same geometry
}

int mi_gamma_rsample_backward(const float* dx, int64_t dx_stride_k, int64_t dx_stride_i,
                              const float* g, const float* concentration,
                              int64_t concentration_stride, const float* rate,
                              int64_t rate_stride, int64_t K, int64_t N, void* workspace,
                              size_t workspace_bytes, float* dconcentration,
                              int64_t dconcentration_stride, float* drate, int64_t drate_stride,
                              void* stream) {
  if (dx == nullptr || g == nullptr || concentration == nullptr || rate == nullptr ||
      dconcentration == nullptr || drate == nullptr || K < 1 || N < 1)
    return MI_EINVAL;
  size_t need = 0;
  mi_gamma_rsample_backward_workspace_bytes(K, N, &need);
  if (need > 0 && (workspace == nullptr || workspace_bytes < need)) return MI_EWORKSPACE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const BwdGeometry geo = bwd_geometry(K, N);
  const int64_t rows = geo.rows, gy = geo.slices;
  float* oc = dconcentration;
  float* orr = drate;
  int64_t sc = dconcentration_stride, sr = drate_stride;
  if (gy > 1) {
    oc = static_cast<float*>(workspace);
    orr = oc + gy * N;
    sc = sr = 1;
  }
  hipLaunchKernelGGL(mi::k_gamma_rsample_bwd, dim3((unsigned)geo.gx, (unsigned)gy),
                     dim3(mi::kGuideThreads), 0, s, dx, dx_stride_k, dx_stride_i, g, concentration,
                     concentration_stride, rate, rate_stride, K, N, oc, sc, orr, sr, N, rows,
                     geo.ti);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || gy == 1) return to_code(e);
  const unsigned grid = (unsigned)ceil_div(N, mi::kGuideThreads);
  hipLaunchKernelGGL(mi::k_sum_slices, dim3(grid), dim3(mi::kGuideThreads), 0, s, oc, orr, gy, N,
                     dconcentration, dconcentration_stride, drate, drate_stride);
  return to_code(hipGetLastError());
}

int mi_beta_dgrad(const float* x, const float* c1, int64_t c1_stride, const float* c0,
                  int64_t c0_stride, int64_t K, int64_t N, double* out, void* stream) {
  if (x == nullptr || c1 == nullptr || c0 == nullptr || out == nullptr || K < 1 || N < 1)
    return MI_EINVAL;
  hipLaunchKernelGGL(mi::k_beta_dgrad, dim3((unsigned)ceil_div(2 * K * N, mi::kGuideThreads)),
                     dim3(mi::kGuideThreads), 0, static_cast<hipStream_t>(stream), x, c1,
                     c1_stride, c0, c0_stride, K, N, out);
  return to_code(hipGetLastError());
}

int mi_capture_abandon(void* stream, int* was_capturing) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipStreamCaptureStatus status = hipStreamCaptureStatusNone;
  hipError_t err = hipStreamIsCapturing(s, &status);
  int capturing = err == hipSuccess && status != hipStreamCaptureStatusNone;
  if (was_capturing != nullptr) *was_capturing = capturing;
  if (capturing) {
    hipGraph_t graph = nullptr;
    err = hipStreamEndCapture(s, &graph);   // ends an invalidated capture too (graph stays NULL)
    if (graph != nullptr) (void)hipGraphDestroy(graph);
  }
  (void)hipGetLastError();
  hipStreamCaptureStatus after = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &after) == hipSuccess && after != hipStreamCaptureStatusNone)
    return to_code(err == hipSuccess ? hipErrorStreamCaptureInvalidated : err);
  (void)hipGetLastError();
  return 0;
}

int mi_step_begin(uint64_t* counter, uint64_t* snapshot, uint32_t* flags, int64_t nflags,
                  void* stream) {
  if (counter == nullptr || snapshot == nullptr || nflags < 0 || (nflags > 0 && flags == nullptr))
    return MI_EINVAL;
  const int64_t threads = std::max<int64_t>(1, nflags);
  hipLaunchKernelGGL(mi::k_step_begin, dim3((unsigned)ceil_div(threads, mi::kGuideThreads)),
                     dim3(mi::kGuideThreads), 0, static_cast<hipStream_t>(stream), counter,
                     snapshot, flags, nflags);
  return to_code(hipGetLastError());
}

int mi_transform_params(const mi_params* params, float* out, void* stream) {
  if (params == nullptr || out == nullptr || params->m < 1 || params->m > MI_MAX_PARAMS ||
      params->n < 1)
    return MI_EINVAL;
  for (int j = 0; j < params->m; ++j)
    if (params->u[j] == nullptr ||
        (params->transform[j] != MI_TRANSFORM_NONE && params->transform[j] != MI_TRANSFORM_EXP))
      return MI_EINVAL;
  hipLaunchKernelGGL(mi::k_transform_params,
                     dim3((unsigned)ceil_div(params->n * params->m, mi::kGuideThreads)),
                     dim3(mi::kGuideThreads), 0, static_cast<hipStream_t>(stream), *params, out);
  return to_code(hipGetLastError());
}

int mi_philox_normal(int64_t K, int64_t N, uint64_t seed, uint64_t step, uint32_t stream_id,
                     int64_t particle_offset, float* out, void* stream) {
  if (out == nullptr || K < 1 || N < 1 || K > 65535) return MI_EINVAL;
  hipLaunchKernelGGL(mi::k_philox_normal, dim3((unsigned)ceil_div(N, 4 * 256), (unsigned)K),
                     dim3(256), 0, static_cast<hipStream_t>(stream), K, N, seed, step, stream_id,
                     particle_offset, out);
  return to_code(hipGetLastError());
}

int mi_philox4x32(const uint32_t* ctr, int64_t count, uint32_t key0, uint32_t key1, uint32_t* out,
                  void* stream) {
  if (ctr == nullptr || out == nullptr || count < 1) return MI_EINVAL;
  hipLaunchKernelGGL(mi::k_philox_raw, dim3((unsigned)ceil_div(count, 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), ctr, count, key0, key1, out);
  return to_code(hipGetLastError());
}

}  // extern "C"
