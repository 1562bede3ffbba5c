// The ELBO's scalar tail in two launches: forward reduces every per-particle log joint and the
// guide's entropy into the loss, backward writes the entropy gradients, hands the upstream gradient
// back to the site groups and rescales their speculative gradients only if it is not 1.
//
// Replaces, in the reference's EvidenceLowerBoundLoss.forward (mininf/nn.py:210-228):
//   `elbo = log_prob.total + approximation.entropy()` (nn.py:224-226) and `return -elbo`, where
//   FactorizedDistribution.entropy (nn.py:121-131) sums torch Normal.entropy (normal.py:112-113)
//   and Beta.entropy (beta.py:101-102 -> dirichlet.py:122-130) over factors and elements,
// plus every autograd kernel of those expressions (~50 small launches per step for a Beta guide),
// and -- for guide factors whose draws feed only the site kernels (mi_factor draw_kind) -- the
// draws' own backward (mi_normal_rsample_backward / mi_beta_rsample_backward), autograd's
// accumulation of the factor gradients and ParameterizedDistribution's transform backward.
//
// Reductions are deterministic: fixed grids, fp64 per-block partial sums, and the last block to
// finish (device-scope counter, reset by that block) adds the partials in a fixed order.
#include <cmath>
#include "beta_grad.hpp"
#include "adam_math.hpp"
#include "entropy.hpp"

#include <algorithm>
#include <cstdlib>

namespace mi {

constexpr int kElboThreads = 256;
constexpr int kElboMaxBlocks = 1024;

// Entropy of element i of a factor (fp32 terms, as torch evaluates them; sums are carried in
// fp64 by the callers).
MI_DEV double factor_entropy(const mi_factor& f, int64_t i) {
  if (f.family == MI_NORMAL) {  // 0.5 + 0.5 log(2 pi) + log(scale)  (normal.py:112-113)
    return (double)(1.4189385332046727f + logf(f.param[1][i * f.stride[1]]));
  }
  if (f.family == MI_GAMMA) {   // a - log(r) + lgamma(a) + (1 - a) psi(a)  (gamma.py:101-107)
    const float a = f.param[0][i * f.stride[0]], r = f.param[1][i * f.stride[1]];
    return (double)(a - logf(r)) + (double)lgammaf(a) + (double)((1.0f - a) * digammaf(a));
  }
  // Beta(a, b) = Dirichlet([a, b]) (dirichlet.py:122-130 with k = 2, a0 = a + b):
  //   lgamma(a) + lgamma(b) - lgamma(a0) - (2 - a0) psi(a0) - (a - 1) psi(a) - (b - 1) psi(b)
  const float a = f.param[0][i * f.stride[0]], b = f.param[1][i * f.stride[1]];
  const float t = a + b;  // concentration.sum(-1)
  return (double)(lgammaf(a) + lgammaf(b) - lgammaf(t)) -
         (double)((2.0f - t) * digammaf(t)) - (double)((a - 1.0f) * digammaf(a)) -
         (double)((b - 1.0f) * digammaf(b));
}

// The element's two parameters, loaded together up front (a missing one reads as 1): the entropy
// derivatives and the exp-transform chain rule below then wait for one round trip, not three.
struct Params2 {
  float p0, p1;
};
MI_DEV Params2 load_params(const mi_factor& f, int64_t i) {
  // (a Normal's loc only feeds its exp transform)
  const bool has0 = f.param[0] != nullptr &&
                    (f.family != MI_NORMAL || f.transform[0] == MI_TRANSFORM_EXP);
  const float* a = has0 ? f.param[0] + i * f.stride[0] : f.param[1] + i * f.stride[1];
  const float v0 = *a, v1 = f.param[1][i * f.stride[1]];
  return Params2{has0 ? v0 : 1.0f, v1};
}

// entropy_grad from loaded parameters
MI_DEV void entropy_grad_of(const mi_factor& f, const Params2& q, double& d0, double& d1) {
  if (f.family == MI_NORMAL) {
    d0 = 0.0;
    d1 = (double)(1.0f / q.p1);
    return;
  }
  if (f.family == MI_GAMMA) {
    d0 = (double)(1.0f + (1.0f - q.p0) * trigammaf(q.p0));
    d1 = (double)(-1.0f / q.p1);
    return;
  }
  const float t = q.p0 + q.p1;
  const float tt = (t - 2.0f) * trigammaf(t);
  d0 = (double)(tt - (q.p0 - 1.0f) * trigammaf(q.p0));
  d1 = (double)(tt - (q.p1 - 1.0f) * trigammaf(q.p1));
}

// write_grad from loaded parameters
MI_DEV void write_grad_of(const mi_factor& F, int j, int64_t i, double g, const Params2& q) {
  if (F.grad[j] == nullptr) return;
  if (F.transform[j] == MI_TRANSFORM_EXP) g *= (double)(j == 0 ? q.p0 : q.p1);
  F.grad[j][i * F.grad_stride[j]] = (float)g;
}

// dH(i) / dparam_j. Normal: (0, 1 / scale); Beta: (a0 - 2) psi'(a0) - (a - 1) psi'(a) and the
// same with b.
MI_DEV void entropy_grad(const mi_factor& f, int64_t i, double& d0, double& d1) {
  if (f.family == MI_NORMAL) {
    d0 = 0.0;
    d1 = (double)(1.0f / f.param[1][i * f.stride[1]]);
    return;
  }
  if (f.family == MI_GAMMA) {   // (1 + (1 - a) psi'(a), -1 / r)
    const float a = f.param[0][i * f.stride[0]], r = f.param[1][i * f.stride[1]];
    d0 = (double)(1.0f + (1.0f - a) * trigammaf(a));
    d1 = (double)(-1.0f / r);
    return;
  }
  const float a = f.param[0][i * f.stride[0]], b = f.param[1][i * f.stride[1]];
  const float t = a + b;
  const float tt = (t - 2.0f) * trigammaf(t);
  d0 = (double)(tt - (a - 1.0f) * trigammaf(a));
  d1 = (double)(tt - (b - 1.0f) * trigammaf(b));
}

// ---- absorbed guide draws -------------------------------------------------------------------
// Blocks [lead_blocks, lead_blocks + first[num]) of a launch work on absorbed factors: factor a
// gets a [slices x gx] grid (gx columns of ti elements, slices of the particle rows), whose
// per-slice sums the last block of each column combines in a fixed order. Beta factors are
// reduced in the forward launch (their fp64 implicit-gradient chains then overlap the entropy
// reduction) and leave pre[i] = {S0, S1, dH0, dH1} for the backward; the other absorbed draws are
// reduced in the backward launch.
struct AbsorbPlan {
  int lead_blocks;
  int num;
  int index[MI_MAX_FACTORS];
  int first[MI_MAX_FACTORS + 1];
  int ti[MI_MAX_FACTORS];
  int gx[MI_MAX_FACTORS];
  int slices[MI_MAX_FACTORS];
  int pad0;
  int64_t rows_per_slice[MI_MAX_FACTORS];
  int64_t counter[MI_MAX_FACTORS];   // first completion counter of the factor's columns
  int64_t partial[MI_MAX_FACTORS];   // offset (doubles) of its [slices, n, 2] partial sums
  int32_t pre[MI_MAX_FACTORS];       // 1: a Beta factor whose [n, 4] forward sums are in F.saved
  int32_t epl[MI_MAX_FACTORS];       // elements per lane (4: a backward over a few partial rows)
};

// Block-dependent selections from the by-value kernel descriptors, written as unrolled
// constant-index selects: indexing a by-value kernel parameter with a run-time index makes the
// compiler copy the whole parameter to scratch memory, and reading it through a generic pointer
// turns every descriptor field into a dependent vector-memory load.
template <typename T, int N>
MI_DEV T pick(const T (&arr)[N], int a) {
  T v = arr[0];
#pragma unroll
  for (int q = 1; q < N; ++q)
    if (a == q) v = arr[q];
  return v;
}

MI_DEV mi_factor factor_at(const mi_elbo& E, int f) {
  switch (f) {
    case 1: return E.factors[1];
    case 2: return E.factors[2];
    case 3: return E.factors[3];
    case 4: return E.factors[4];
    case 5: return E.factors[5];
    case 6: return E.factors[6];
    case 7: return E.factors[7];
    default: return E.factors[0];
  }
}

// d loss / d param_j (or d loss / d u_j for param_j = exp(u_j)) of element i.
MI_DEV void write_grad(const mi_factor& F, int j, int64_t i, double g) {
  if (F.grad[j] == nullptr) return;
  if (F.transform[j] == MI_TRANSFORM_EXP) g *= (double)F.param[j][i * F.stride[j]];
  F.grad[j][i * F.grad_stride[j]] = (float)g;
}

// d T / d z[k, i] summed over the sources (fp32, as autograd accumulates the groups' gradients).
// Branch-free: every slot reads (source 0 stands in for the unused ones) and the unused terms are
// +0 -- the loads of several rows can then be in flight together.
MI_DEV float source_sum(const mi_factor& F, int64_t k, int64_t i) {
  float g = 0.0f;
#pragma unroll
  for (int s = 0; s < MI_MAX_SOURCES; ++s) {
    const mi_source& S = F.source[s < F.num_sources ? s : 0];
    g += keep_if(S.ptr[k * S.stride_k + i * S.stride_i], s < F.num_sources);
  }
  return g;
}

// Sums of one absorbed draw's backward over particle rows r0, r0 + tk, ... < r1 for element i:
//   Normal: s0 = sum_k dz, s1 = sum_k dz * eps  (mi_normal_rsample_backward)
//   Beta:   s0 = sum_k dx * dgrad(x, a, a+b) * (1 - x), s1 = -sum_k dx * dgrad(1-x, b, a+b) * x
//           (mi_beta_rsample_backward / torch _Dirichlet_backward with grad (dx, 0))
// BETA: the forward launch's Beta draws; otherwise the backward's Normal draws.
template <bool BETA>
MI_DEV void draw_sums(const mi_factor& F, int64_t i, int64_t r0, int64_t r1, int tk,
                      double& s0, double& s1) {
  const int64_t n = F.n;
  if ((BETA || F.family == MI_BETA) && F.dgrad != nullptr) {   // factors precomputed (mi_side,
                                                               // mi_beta_dgrad)
    // eight rows' loads in flight per lane, then the sums in row order
    constexpr int kU = 8;
    for (int64_t k0 = r0; k0 < r1; k0 += kU * (int64_t)tk) {
      float g[kU];
      double2 d[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t k = k0 + (int64_t)u * tk;
        const int64_t kc = k < r1 ? k : r1 - 1;
        g[u] = keep_if(source_sum(F, kc, i), k < r1);
        d[u] = *reinterpret_cast<const double2*>(F.dgrad + 2 * (kc * n + i));
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (g[u] == 0.0f) continue;   // as the evaluating branch: a zero upstream never meets
                                      // the factor
        s0 += (double)g[u] * d[u].x;
        s1 += (double)g[u] * d[u].y;
      }
    }
  } else if (BETA) {
    const float a = F.param[0][i * F.stride[0]], b = F.param[1][i * F.stride[1]];
    const float tot = a + b;  // concentration.sum(-1) in fp32, dirichlet.py:18
    const double psi_a = digamma((double)a), psi_b = digamma((double)b);
    const double psi_t = digamma((double)tot);
    for (int64_t k = r0; k < r1; k += tk) {
      const float g = source_sum(F, k, i);
      if (g == 0.0f) continue;
      const float xv = F.draws[k * n + i];
      const float xw = 1.0f - xv;
      s0 += dirichlet_grad(xv, a, tot, psi_a, psi_t) * (double)g * (double)(1.0f - xv);
      s1 -= dirichlet_grad(xw, b, tot, psi_b, psi_t) * (double)g * (double)xv;
    }
  } else if (F.draw_kind == MI_DRAW_PARTIALS) {
    for (int64_t r = r0; r < r1; r += tk) {
      s0 += (double)F.partial[0][r * n + i];
      s1 += (double)F.partial[1][r * n + i];
    }
  } else if (F.family == MI_NORMAL) {
    uint64_t step = F.step;
    if (F.step_device != nullptr) step += *F.step_device;
    // four rows' loads (sources, eps) in flight per lane, then the sums in row order
    constexpr int kU = 4;
    for (int64_t k0 = r0; k0 < r1; k0 += kU * (int64_t)tk) {
      float g[kU], e[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t k = k0 + (int64_t)u * tk;
        const int64_t kc = k < r1 ? k : r1 - 1;
        g[u] = keep_if(source_sum(F, kc, i), k < r1);
        if (F.eps != nullptr) {
          e[u] = F.eps[kc * n + i];
        } else {
          float q[4];
          guide_normals(F.seed, step, F.stream_id, (uint64_t)((F.element_offset + i) >> 2),
                        (uint64_t)(F.particle_offset + kc), q);
          e[u] = q[i & 3];
        }
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (k0 + (int64_t)u * tk >= r1) break;
        s0 += (double)g[u];
        s1 += (double)g[u] * (double)e[u];
      }
    }
  }
}

// Backward of a draw whose particle sums arrive as a few partial rows (MI_DRAW_PARTIALS): lane
// elements base + e * ti, e < 4 -- every load of the four elements (partial rows, the parameters
// for the entropy and exp-transform terms) in flight before the first gradient is stored.
MI_DEV void partial_lane_elements(const mi_factor& F, int64_t base, int ti, int64_t rows, float u,
                                  double w) {
  constexpr int kE = 4;
  double g[kE][2];
  bool ok[kE];
  int64_t ic[kE];
  double s0[kE], s1[kE];
  float pm[kE][2];
#pragma unroll
  for (int e = 0; e < kE; ++e) {
    const int64_t i = base + (int64_t)e * ti;
    ok[e] = i < F.n;
    ic[e] = ok[e] ? i : 0;
    s0[e] = s1[e] = 0.0;
#pragma unroll
    for (int j = 0; j < 2; ++j)   // only what the exp transforms read (C5's loc is not)
      pm[e][j] = F.transform[j] == MI_TRANSFORM_EXP ? F.param[j][ic[e] * F.stride[j]] : 1.0f;
  }
  // rows outermost: each row's eight loads (four elements, two sums) issue together
  for (int64_t r = 0; r < rows; ++r) {
    float a0[kE], a1[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      a0[e] = F.partial[0][r * F.n + ic[e]];
      a1[e] = F.partial[1][r * F.n + ic[e]];
    }
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      s0[e] += (double)a0[e];
      s1[e] += (double)a1[e];
    }
  }
#pragma unroll
  for (int e = 0; e < kE; ++e) {
    double d0, d1;
    entropy_grad(F, ic[e], d0, d1);
    g[e][0] = (double)u * s0[e] + w * d0;
    g[e][1] = (double)u * s1[e] + w * d1;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (F.transform[j] == MI_TRANSFORM_EXP) g[e][j] *= (double)pm[e][j];
  }
#pragma unroll
  for (int e = 0; e < kE; ++e) {
    if (!ok[e]) continue;
    const int64_t i = base + (int64_t)e * ti;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (F.grad[j] != nullptr) F.grad[j][i * F.grad_stride[j]] = (float)g[e][j];
  }
}

// The same backward with 16-byte accesses (Normal factors, n % 4 == 0, unit strides, aligned --
// checked by the plan): lane quads q = first + p * ti, p < NP, every load of all NP quads in flight
// before the first gradient is computed; the arithmetic and its order are those of
// partial_lane_elements.
template <int NP>
MI_DEV void partial_lane_quads(const mi_factor& F, int64_t first, int ti, int64_t rows, float u,
                               double w) {
  const bool exp0 = F.transform[0] == MI_TRANSFORM_EXP, exp1 = F.transform[1] == MI_TRANSFORM_EXP;
  const int64_t nq = F.n >> 2;
  const float4* __restrict__ sc = reinterpret_cast<const float4*>(F.param[1]);
  const float4* __restrict__ lc = reinterpret_cast<const float4*>(F.param[0]);
  float4 scale[NP], loc[NP];
  double s0[NP][4], s1[NP][4];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int64_t q = min(first + (int64_t)p * ti, nq - 1);
    scale[p] = sc[q];
    loc[p] = exp0 ? lc[q] : make_float4(1.0f, 1.0f, 1.0f, 1.0f);
#pragma unroll
    for (int e = 0; e < 4; ++e) s0[p][e] = s1[p][e] = 0.0;
  }
  for (int64_t r = 0; r < rows; ++r) {
    const float4* __restrict__ r0 = reinterpret_cast<const float4*>(F.partial[0] + r * F.n);
    const float4* __restrict__ r1 = reinterpret_cast<const float4*>(F.partial[1] + r * F.n);
    float4 a0[NP], a1[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int64_t q = min(first + (int64_t)p * ti, nq - 1);
      a0[p] = r0[q];
      a1[p] = r1[q];
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      s0[p][0] += (double)a0[p].x; s0[p][1] += (double)a0[p].y;
      s0[p][2] += (double)a0[p].z; s0[p][3] += (double)a0[p].w;
      s1[p][0] += (double)a1[p].x; s1[p][1] += (double)a1[p].y;
      s1[p][2] += (double)a1[p].z; s1[p][3] += (double)a1[p].w;
    }
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int64_t q = first + (int64_t)p * ti;
    if (q >= nq) continue;
    const float sv[4] = {scale[p].x, scale[p].y, scale[p].z, scale[p].w};
    const float lv[4] = {loc[p].x, loc[p].y, loc[p].z, loc[p].w};
    float g0[4], g1[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      // entropy_grad of a Normal: (0, 1 / scale)
      double d0 = (double)u * s0[p][e] + w * 0.0;
      double d1 = (double)u * s1[p][e] + w * (double)(1.0f / sv[e]);
      if (exp0) d0 *= (double)lv[e];
      if (exp1) d1 *= (double)sv[e];
      g0[e] = (float)d0;
      g1[e] = (float)d1;
    }
    if (F.grad[0] != nullptr)
      reinterpret_cast<float4*>(F.grad[0])[q] = make_float4(g0[0], g0[1], g0[2], g0[3]);
    if (F.grad[1] != nullptr)
      reinterpret_cast<float4*>(F.grad[1])[q] = make_float4(g1[0], g1[1], g1[2], g1[3]);
  }
}

// One block of absorbed-factor work (block `bid` of the absorbed range). FORWARD: Beta factors,
// leaving pre[i] = {S0, S1, dH0, dH1}; backward: everything else, writing the gradients.
template <bool FORWARD>
MI_DEV void absorbed_block(const mi_elbo& E, const AbsorbPlan& P, int bid, float u,
                           unsigned* __restrict__ counters, double* __restrict__ work,
                           double (*red)[2], bool* last) {
  int a = 0;
#pragma unroll
  for (int q = 1; q < MI_MAX_FACTORS; ++q)
    if (q < P.num && bid >= P.first[q]) a = q;
  const mi_factor F = factor_at(E, pick(P.index, a));
  const double w = -(double)u * E.entropy_scale * F.weight;
  const int local = bid - pick(P.first, a);
  const int gx = pick(P.gx, a), ti = pick(P.ti, a), slices = pick(P.slices, a);
  const int64_t rows_per_slice = pick(P.rows_per_slice, a);
  const bool has_pre = pick(P.pre, a) != 0;
  const int col = local % gx, slice = local / gx;
  const int tx = threadIdx.x % ti, ty = threadIdx.x / ti, tk = kElboThreads / ti;
  const int64_t i = (int64_t)col * ti + tx;
  if (!FORWARD && has_pre) {   // Beta: sums and entropy derivatives from the forward
    if (i < F.n) {
      const double* pre = F.saved + 4 * i;
      write_grad(F, 0, i, (double)u * pre[0] + w * pre[2]);
      write_grad(F, 1, i, (double)u * pre[1] + w * pre[3]);
    }
    return;
  }
  const int64_t rows = F.draw_kind == MI_DRAW_PARTIALS ? F.partial_rows : E.K;
  const int64_t r0 = (int64_t)slice * rows_per_slice;
  const int64_t r1 = min(rows, r0 + rows_per_slice);
  double s0 = 0.0, s1 = 0.0;
  if (!FORWARD && pick(P.epl, a) == 4) {   // a fused draw's few partial rows: 4 elements per lane
    partial_lane_elements(F, (int64_t)col * ti * 4 + tx, ti, rows, u, w);
    return;
  }
  if (!FORWARD && pick(P.epl, a) < 0) {   // the same over quads: -epl quads per lane
    const int np = -pick(P.epl, a);
    const int64_t q0 = (int64_t)col * ti * np + tx;
    switch (np) {
      case 2: partial_lane_quads<2>(F, q0, ti, rows, u, w); break;
      case 4: partial_lane_quads<4>(F, q0, ti, rows, u, w); break;
      default: partial_lane_quads<1>(F, q0, ti, rows, u, w); break;
    }
    return;
  }
  if (tk == 1 && slices == 1) {   // a lane per element: no block reduction, and no barrier
                                  // between its loads
    if (i < F.n) {
      const Params2 q = load_params(F, i);   // in flight during the draw sums
      draw_sums<FORWARD>(F, i, r0, r1, 1, s0, s1);
      double d0, d1;
      entropy_grad_of(F, q, d0, d1);
      if (FORWARD) {
        double* pre = F.saved + 4 * i;
        pre[0] = s0;
        pre[1] = s1;
        pre[2] = d0;
        pre[3] = d1;
      } else {
        write_grad_of(F, 0, i, (double)u * s0 + w * d0, q);
        write_grad_of(F, 1, i, (double)u * s1 + w * d1, q);
      }
    }
    return;
  }
  // the element's parameters, in flight during the sums (the lanes that finish the element)
  const Params2 q = load_params(F, i < F.n ? i : F.n - 1);
  if (i < F.n) draw_sums<FORWARD>(F, i, r0 + ty, r1, tk, s0, s1);
  red[threadIdx.x][0] = s0;
  red[threadIdx.x][1] = s1;
  __syncthreads();
  // fixed pairwise tree over the block's particle lanes (log2(tk) steps; a serial sum over 256
  // lanes is a 256-long chain of dependent LDS reads and fp64 adds)
  for (int half = tk >> 1; half > 0; half >>= 1) {
    if (ty < half) {
      red[threadIdx.x][0] += red[threadIdx.x + half * ti][0];
      red[threadIdx.x][1] += red[threadIdx.x + half * ti][1];
    }
    __syncthreads();
  }
  if (ty == 0) {
    s0 = red[tx][0];
    s1 = red[tx][1];
  }
  unsigned* counter = nullptr;
  if (slices > 1) {
    double* part = work + pick(P.partial, a);
    if (ty == 0 && i < F.n) {
      part[((int64_t)slice * F.n + i) * 2] = s0;
      part[((int64_t)slice * F.n + i) * 2 + 1] = s1;
    }
    __syncthreads();
    counter = counters + pick(P.counter, a) + col;
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");   // the block's partials, then the count
      *last = atomicAdd(counter, 1u) == (unsigned)slices - 1u;
    }
    __syncthreads();
    if (!*last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (ty == 0 && i < F.n) {   // the column's last block: slices in a fixed order
      s0 = s1 = 0.0;
      for (int s = 0; s < slices; ++s) {
        s0 += part[((int64_t)s * F.n + i) * 2];
        s1 += part[((int64_t)s * F.n + i) * 2 + 1];
      }
    }
  }
  if (ty == 0 && i < F.n) {
    double d0, d1;
    entropy_grad_of(F, q, d0, d1);
    if (FORWARD) {
      double* pre = F.saved + 4 * i;
      pre[0] = s0;
      pre[1] = s1;
      pre[2] = d0;
      pre[3] = d1;
    } else {
      write_grad_of(F, 0, i, (double)u * s0 + w * d0, q);
      write_grad_of(F, 1, i, (double)u * s1 + w * d1, q);
    }
  }
  if (counter != nullptr && threadIdx.x == 0) *counter = 0u;
}

// Phase timestamps (MI_ELBO_TIMING builds only, tools/elbo_timing.py): wall clock at up to 16
// points of every block of k_elbo_forward (thread 0), into a buffer the timing build allocates.
#ifndef MI_ELBO_TIMING
#define MI_ELBO_TIMING 0
#endif
#if MI_ELBO_TIMING
__device__ unsigned long long* mi_elbo_tbuf;
__shared__ unsigned long long mi_ets[16];
#define MI_ELBO_STAMP(i) do { if (threadIdx.x == 0) mi_ets[i] = wall_clock64(); } while (0)
#define MI_ELBO_FLUSH() do { if (threadIdx.x == 0) { unsigned long long* o = mi_elbo_tbuf + (int64_t)blockIdx.x * 16; \
    for (int q = 0; q < 16; ++q) o[q] = mi_ets[q]; } } while (0)
#else
#define MI_ELBO_STAMP(i) do { } while (0)
#define MI_ELBO_FLUSH() do { } while (0)
#endif

// ---- deferred site finalize reductions (mi_elbo.reduce) ---------------------------------------
// Block (job a, particle block kb, value v) sums part[v][seg][k] over the job's segments for 64
// particles: 4 segment groups of 64 lanes, up to sixteen loads in flight per lane, partial sums in fp64
// combined in a fixed order -- the arithmetic of sites.hip k_finalize, fused into this launch.
// Jobs with one site value split their values over blocks (as k_finalize's split mode).
// Long segment lists use blocks of 32 particles x 8 segment groups (more blocks, fewer serial load
// rounds per lane; MININF_AMD_ELBO_KRED), short ones 64 particles x 4 groups.
constexpr int kRedKWide = 64;

// Completion counting of the forward's share-writing blocks in two levels: blocks count into the
// counter of their group of kGroupBlocks, the last of a group into the launch counter -- a few
// hundred blocks contending for one address would serialise on it.
#ifndef MI_ELBO_RELEASE_FENCE
#define MI_ELBO_RELEASE_FENCE 0
#endif
constexpr int kGroupBlocks = 32;
constexpr int kSingleCount = 160;
constexpr int kGroupCounters = 64;        // groups: at most kGroupCounters * kGroupBlocks blocks
constexpr int kGroupCounterWord = 16;     // first group counter (uint32 word)
constexpr int kGroupCounterStride = 16;   // words between group counters (64 bytes)

// Forward-absorbed Beta factors of one element (a global parameter's K draws, e.g. the coin's
// theta) whose precomputed implicit-gradient factors dgrad[k] this launch sums against their
// upstream g_k = sum_s source_s[k]: by linearity, every block that writes a source row (the slot
// values of the reductions) or reads one written earlier (the lead blocks) adds its particles'
// sum_k g_sk dgrad[k] to its own partial, and the last block adds the partials in a fixed order.
constexpr int kMaxTails = 2;

struct ReducePlan {
  int external;                   // 1: the reductions ran as their own launches; add their totals
  int num;
  int first[MI_MAX_REDUCE + 1];   // first block of each job
  int vblocks[MI_MAX_REDUCE];     // blocks per particle block: num values (split) or 1
  int kred[MI_MAX_REDUCE];        // particles per block
  int tails;                      // tail factors
  int tail_slot[MI_MAX_REDUCE * MI_MAX_SLOTS];   // [a * MI_MAX_SLOTS + j], bit t: job a's slot
                                                 // j is a source of tail t
  int tail_ext[kMaxTails];        // bit s: source s of tail t is read by the lead blocks
  int64_t tail_part;              // offset (doubles) of the [tails][nshare][2] partials
  const double* tail_dgrad[kMaxTails];   // [K, 1, 2]
  const float* tail_src[kMaxTails][MI_MAX_SOURCES];
  int64_t tail_src_stride[kMaxTails][MI_MAX_SOURCES];
  const float* tail_c1[kMaxTails];       // concentrations (n = 1)
  const float* tail_c0[kMaxTails];
  double* tail_saved[kMaxTails];
  // MI_ELBO_FINAL_GRADS: the factor of each tail; its fields are read through factor_field-style
  // selects (a whole mi_factor selected by a run-time index would be copied to scratch memory,
  // and the kernel arguments must stay within 4 KiB)
  int tail_factor[kMaxTails];
  // One small Normal factor -- factor 0 of the launch -- whose draw's only source is consecutive
  // slot rows of one split reduction (the regression's theta under a linear site,
  // mi_linear.draw): with MI_ELBO_FINAL_GRADS the blocks writing those rows also sum dz and
  // dz * eps over their particles, and the last block finishes the factor's gradients.
  int nt_job;                            // -1: none
  int nt_j0;                             // slot of element 0
  int nt_nkb;                            // particle blocks of the job
  int64_t nt_part;                       // offset (doubles) of the [n][nt_nkb][2] partials
  // A one-element Normal factor (the masked hierarchical model's mu) whose sources are slots of
  // any jobs (nt_mask[a] bit j: job a's slot j): every reducing block adds its slots' share, by
  // linearity, into its own partial (nt_nkb = the reducing blocks, indexed by block).
  int nt_single;
  int nt_mask[MI_MAX_REDUCE];
  // offset (doubles) of what block 0 computes early for the last block (early_tail): per tail the
  // three trigammas of its entropy derivatives, then per optimizer slot (s1, bias corrections)
  int64_t early;
};
constexpr int kEarlyDoubles = 3 * kMaxTails + 2 * MI_ELBO_ADAM_SLOTS;

// Fields of factor f of the launch, by constant-index selects (see ReducePlan.tail_factor).
MI_DEV float* factor_grad(const mi_elbo& E, int f, int j) {
  float* g = E.factors[0].grad[j];
#pragma unroll
  for (int c = 1; c < MI_MAX_FACTORS; ++c)
    if (f == c) g = E.factors[c].grad[j];
  return g;
}
MI_DEV bool factor_exp(const mi_elbo& E, int f, int j) {
  int t = E.factors[0].transform[j];
#pragma unroll
  for (int c = 1; c < MI_MAX_FACTORS; ++c)
    if (f == c) t = E.factors[c].transform[j];
  return t == MI_TRANSFORM_EXP;
}
MI_DEV double factor_weight(const mi_elbo& E, int f) {
  double w = E.factors[0].weight;
#pragma unroll
  for (int c = 1; c < MI_MAX_FACTORS; ++c)
    if (f == c) w = E.factors[c].weight;
  return w;
}

// The forward's generator step word of factor 0 (the Normal tail): the forward runs before it
// advances the step counter, so the backward's snapshot word still holds the previous
// evaluation's step and the counter this one's.
MI_DEV uint64_t forward_step0(const mi_elbo& E) {
  const mi_factor& F = E.factors[0];
  const uint64_t* sd = (E.step_counter != nullptr && F.step_device == E.step_snapshot)
                           ? E.step_counter : F.step_device;
  return F.step + (sd != nullptr ? *sd : 0ull);
}

// Fixed-order tree sum over the first `n` (a power of two) entries of lds; result in lds[0].
MI_DEV void lds_tree(double* lds, int n) {
  for (int half = n >> 1; half > 0; half >>= 1) {
    if ((int)threadIdx.x < half) lds[threadIdx.x] += lds[threadIdx.x + half];
    __syncthreads();
  }
}

// Writes job J's outputs for one block's particles (local block `local` of the job) and returns
// g0 * the sum of its (fp32) totals (0 from blocks that do not write totals): the block's share of
// the loss.
MI_DEV double reduce_job(const mi_elbo& E, float g0, const mi_reduce& J, int local, int vb,
                         int kRedK, const ReducePlan& R, int a, double (&c)[kMaxTails][2],
                         double (*red)[2], double (&nt)[2], int& nt_slot) {
  const int kRedG = kElboThreads / kRedK;
  const int nv = J.num_sites + J.num_slots;
  const int64_t kb = local / vb;
  const int v0 = vb > 1 ? local % vb : 0, v1 = vb > 1 ? v0 + 1 : nv;
  // this block's element of the Normal tail (split jobs: one value per block), or -1
  const bool nt_fin = (E.options & MI_ELBO_FINAL_GRADS) && R.nt_job >= 0;
  nt_slot = -1;
  if (nt_fin && R.nt_single) {
    nt_slot = 0;   // every reducing block writes its (possibly zero) share
  } else if (nt_fin && a == R.nt_job && vb > 1) {
    const int j = v0 - J.num_sites;
    const int i = j - R.nt_j0;
    if (j >= 0 && i >= 0 && i < E.factors[0].n) nt_slot = i;
  }
  const int nt_mask = nt_fin && R.nt_single ? pick(R.nt_mask, a) : 0;
  // the Normal tail's generator step, read before the segment loads (its use follows them: read
  // there, it was one more memory round trip after them)
  const uint64_t nt_step = nt_slot >= 0 ? forward_step0(E) : 0ull;
  const int kl = threadIdx.x % kRedK, gl = threadIdx.x / kRedK;
  const int64_t K = J.K;
  const int64_t k = kb * kRedK + kl;
  const int64_t kc = k < K ? k : K - 1;
  double* lds = &red[0][0];   // [kRedG][kRedK] doubles
  double t = 0.0;
  // the tails' factors of this lane's particle, fetched ahead of the reduction that decides whether
  // they are needed (a load behind that test costs a round trip of its own at the end)
  double2 tdg[kMaxTails];
#pragma unroll
  for (int q = 0; q < kMaxTails; ++q)
    tdg[q] = (q < R.tails && gl == 0) ? *reinterpret_cast<const double2*>(pick(R.tail_dgrad, q) + 2 * kc)
                                      : make_double2(0.0, 0.0);
  for (int v = v0; v < v1; ++v) {
    // rank-one values (mi_reduce.rank1): the particle-independent u[seg], then f[k] u + e[k]
    const bool r1 = (J.rank1 >> v) & 1;
    const float* __restrict__ p = J.part + (int64_t)v * J.nseg * K + (r1 ? 0 : kc);
    const int64_t stride = r1 ? 1 : K;
    // the rank-one factors of this lane's particle, fetched with the segments (not after them)
    float r1f = 0.0f, r1e = 0.0f;
    if (r1 && gl == 0) {
      const float* __restrict__ q = J.part + (int64_t)v * J.nseg * K + J.nseg;
      r1f = q[kc];
      r1e = q[K + kc];
    }
    MI_ELBO_STAMP(8);   // (descriptor decoded: the segment loads go out next)
    double acc = 0.0;
    int64_t g = gl;
    // sixteen loads in flight per lane (a C2-sized list, ~250 segments over 8 groups, is two
    // rounds of memory latency instead of four), the last round padded with clamped loads whose
    // values are dropped: a remainder loop waited one round trip per segment
    for (; g + 15 * kRedG < J.nseg; g += 16 * kRedG) {
      float x[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) x[j] = p[(g + j * kRedG) * stride];
#pragma unroll
      for (int j = 0; j < 16; ++j) acc += (double)x[j];
    }
    if (g < J.nseg) {
      float x[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int64_t gj = g + j * kRedG;
        x[j] = keep_if(p[(gj < J.nseg ? gj : J.nseg - 1) * stride], gj < J.nseg);
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) acc += (double)x[j];
    }
    MI_ELBO_STAMP(9);   // (the lane's segments summed)
    __syncthreads();
    lds[gl * kRedK + kl] = acc;
    __syncthreads();
    if (gl == 0 && k < K) {
      double s = 0.0;
      for (int j = 0; j < kRedG; ++j) s += lds[j * kRedK + kl];
      if (r1) s = (double)r1f * s + (double)r1e;
      if (v < J.num_sites) {
        s *= pick(J.scale, v);
        if (J.site_lp != nullptr) J.site_lp[(int64_t)v * K + k] = s;
        t += s;
      } else {
        const int j = v - J.num_sites;
        const float gv = (float)(s * J.slot_scale);
        J.slot_grad[(int64_t)j * K + k] = gv;
        if (nt_slot >= 0 && (!R.nt_single || ((nt_mask >> j) & 1))) {
          // d z[k, i] for the Normal tail, against its regenerated eps
          const mi_factor& F = E.factors[0];
          const uint64_t step = nt_step;
          const int64_t i = nt_slot;
          float q[4];
          guide_normals(F.seed, step, F.stream_id, (uint64_t)((F.element_offset + i) >> 2),
                        (uint64_t)(F.particle_offset + k), q);
          nt[0] += (double)gv;
          nt[1] += (double)gv * (double)q[i & 3];
        }
        const int mask = j < MI_MAX_SLOTS ? pick(R.tail_slot, a * MI_MAX_SLOTS + j) : 0;
#pragma unroll
        for (int q = 0; q < kMaxTails; ++q)
          if (((mask >> q) & 1) && gv != 0.0f) {   // a zero upstream never meets the factor
            c[q][0] += (double)gv * tdg[q].x;
            c[q][1] += (double)gv * tdg[q].y;
          }
      }
    }
  }
  double share = 0.0;
  if (v0 == 0 && gl == 0 && k < K) {
    const float tf = (float)t;
    J.total[k] = tf;
    share = (double)tf;
  }
  return (double)g0 * share;
}

MI_DEV double reduce_block(const mi_elbo& E, const ReducePlan& R, int bid,
                           double (&c)[kMaxTails][2], double (*red)[2], double (&nt)[2],
                           int& nt_slot, int& nt_kb) {
  int a = 0;
#pragma unroll
  for (int q = 1; q < MI_MAX_REDUCE; ++q)
    if (q < R.num && bid >= R.first[q]) a = q;
  const int local = bid - pick(R.first, a);
  const int vb = pick(R.vblocks, a);
  const int kred = pick(R.kred, a);
  double share;
  // constant descriptor indices (a run-time index into the by-value kernel argument would copy
  // it to scratch memory)
  nt_kb = R.nt_single ? bid : local / vb;
  switch (a) {
    case 1: share = reduce_job(E, E.g0, E.reduce[1], local, vb, kred, R, 1, c, red, nt, nt_slot); break;
    case 2: share = reduce_job(E, E.g0, E.reduce[2], local, vb, kred, R, 2, c, red, nt, nt_slot); break;
    case 3: share = reduce_job(E, E.g0, E.reduce[3], local, vb, kred, R, 3, c, red, nt, nt_slot); break;
    default: share = reduce_job(E, E.g0, E.reduce[0], local, vb, kred, R, 0, c, red, nt, nt_slot); break;
  }
  return share;
}



// ---- what the last block needs that is known at the launch's start ---------------------------
// Block 0 computes, while its own reduction's loads are in flight, the values the last block's
// tail would otherwise compute on its critical path: the trigammas of each Beta tail's entropy
// derivatives (the concentrations are written by the launch before) and each optimizer slot's
// bias corrections (two fp64 pow per tensor). Device-coherent stores, complete before block 0's
// completion count, so the last block reads them with its first loads.
// whether factor f's final gradients are written by the launch's fused-draw blocks (P: the
// launch's final-gradient plan; its optimizer slots are updated there, fin_adam)
MI_DEV bool fin_factor(const AbsorbPlan& P, int f) {
  bool hit = false;
#pragma unroll
  for (int a = 0; a < MI_MAX_FACTORS; ++a) hit |= a < P.num && P.index[a] == f;
  return hit;
}

MI_DEV void early_tail(const mi_elbo& E, const ReducePlan& R, const AbsorbPlan& P,
                       const mi_elbo_adam* __restrict__ adam, double* __restrict__ work) {
  const int t = threadIdx.x;
  double* out = work + R.early;
  if (t < 3 * kMaxTails) {
    const int q = t / 3, which = t % 3;
    if (q < R.tails) {
      const float a = *pick(R.tail_c1, q), b = *pick(R.tail_c0, q);
      const float x = which == 0 ? a + b : which == 1 ? a : b;
      __hip_atomic_store(out + t, (double)trigammaf(x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else if (adam != nullptr && t >= kWave && t < kWave + MI_ELBO_ADAM_SLOTS) {
    const int q = t - kWave;
    if (q < adam->num && !fin_factor(P, adam->slots[q].factor)) {
      const float s1 = *adam->slots[q].step + 1.0f;
      const AdamCoef c = adam_coef(*adam, s1);
      // (s1, bc1) and (bc2_sqrt, step_size) as two doubles of float pairs
      const float v[4] = {s1, c.bc1, c.bc2_sqrt, c.step_size};
      double d[2];
      __builtin_memcpy(d, v, sizeof(d));
      double* o = out + 3 * kMaxTails + 2 * q;
      __hip_atomic_store(o, d[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o + 1, d[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---- forward --------------------------------------------------------------------------------
// HAS_BETA = false: only Normal factors (log of the scale), which keeps the register footprint
// of the common large-factor case small; true: any Beta or Gamma factor (generic entropy path).
// ABSORB: the launch has forward-absorbed Beta blocks (absorbed_block<true>, inline fp64 implicit
// gradients: a large register footprint the other variants do not pay for).
template <bool HAS_BETA, bool ABSORB>
__global__ __launch_bounds__(kElboThreads) void k_elbo_forward(const mi_elbo E,
                                                               const AbsorbPlan P,
                                                               const ReducePlan R,
                                                               double* __restrict__ work,
                                                               unsigned* __restrict__ counters,
                                                               float* __restrict__ loss,
                                                               const mi_elbo_adam* __restrict__ adam) {
  __shared__ double red[kElboThreads][2];
  __shared__ bool last;
#if MI_ELBO_TIMING
  if (threadIdx.x < 16) mi_ets[threadIdx.x] = 0;
#endif
  MI_ELBO_STAMP(0);
  kernarg_prefetch<(int)(sizeof(mi_elbo) + sizeof(AbsorbPlan) + sizeof(ReducePlan))>();
  const int nred = R.first[R.num];
  const int nloss = P.lead_blocks;
  const int nshare = nred + nloss;   // blocks that write a loss share
  if (ABSORB && (int)blockIdx.x >= nshare) {
    absorbed_block<true>(E, P, (int)blockIdx.x - nshare, 1.0f, counters, work, red, &last);
    return;
  }
  if (!ABSORB && (int)blockIdx.x >= nshare) {
    // MI_ELBO_FINAL_GRADS: the gradients of the fused-draw factors (MI_DRAW_PARTIALS) for an
    // upstream of 1 -- k_elbo_backward's absorbed blocks, run here (P: their plan); they read only
    // the site launches' partial rows, so they run beside the reductions
    absorbed_block<false>(E, P, (int)blockIdx.x - nshare, 1.0f, counters, work, red, &last);
    return;
  }
  if (!ABSORB && blockIdx.x == 0 && (R.tails > 0 || adam != nullptr))
    early_tail(E, R, P, adam, work);
  double* rsum = &red[0][0];
  double share;
  double c[kMaxTails][2] = {};   // this lane's tail contributions
  double nt[2] = {0.0, 0.0};     // this lane's Normal-tail sums (R.nt_job), element nt_slot
  int nt_slot = -1, nt_kb = 0;
  if (!ABSORB && (int)blockIdx.x < nred) {   // (ABSORB launches have no deferred reductions)
    share = reduce_block(E, R, (int)blockIdx.x, c, red, nt, nt_slot, nt_kb);
    __syncthreads();
  } else {
    const int64_t lead = (int64_t)blockIdx.x - nred;
    const int64_t stride = (int64_t)nloss * kElboThreads;
    const int64_t first = lead * kElboThreads + threadIdx.x;
    double lp = 0.0, h = 0.0;
    for (int t = 0; t < E.num_terms; ++t)
      for (int64_t k = first; k < E.K; k += stride) lp += (double)E.terms[t][k];
    if (R.external) {
#pragma unroll
      for (int a = 0; a < MI_MAX_REDUCE; ++a)
        if (a < R.num)
          for (int64_t k = first; k < E.K; k += stride) lp += (double)E.reduce[a].total[k];
    }
    for (int f = 0; f < E.num_factors; ++f) {
      const mi_factor& F = E.factors[f];
      if (!HAS_BETA || F.family == MI_NORMAL) {
        // sum_i (0.5 + 0.5 log(2 pi) + log scale_i): the constant once, the logs per element
        const float* __restrict__ sc = F.param[1];
        const int64_t ss = F.stride[1];
        float hf = 0.0f;   // per-thread partial of a few terms, then fp64
        int64_t head = 0;
        if (ss == 1 && (reinterpret_cast<uintptr_t>(sc) & 15) == 0) {
          // 16-byte loads, all issued before the logs
          const int64_t nq = F.n >> 2;
          const float4* __restrict__ sq = reinterpret_cast<const float4*>(sc);
          int64_t q = first;
          // eight quads' loads in flight per round, then four (a lead block covers ~32 elements
          // per lane: one memory round trip, not two); quads summed in order either way
          for (; q + 7 * stride < nq; q += 8 * stride) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = sq[q + u * stride];
#pragma unroll
            for (int u = 0; u < 8; ++u)
              hf += (logf(v[u].x) + logf(v[u].y)) + (logf(v[u].z) + logf(v[u].w));
          }
          for (; q + 3 * stride < nq; q += 4 * stride) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = sq[q + u * stride];
#pragma unroll
            for (int u = 0; u < 4; ++u)
              hf += (logf(v[u].x) + logf(v[u].y)) + (logf(v[u].z) + logf(v[u].w));
          }
          for (; q < nq; q += stride) {
            const float4 v = sq[q];
            hf += (logf(v.x) + logf(v.y)) + (logf(v.z) + logf(v.w));
          }
          head = nq << 2;
        }
        for (int64_t i = head + first; i < F.n; i += stride) hf += logf(sc[i * ss]);
        double hn = (double)hf;
        if (first == 0) hn += 1.4189385332046727 * (double)F.n;
        h += F.weight * hn;
      } else {
        double hb = 0.0;
        for (int64_t i = first; i < F.n; i += stride) hb += factor_entropy(F, i);
        h += F.weight * hb;
      }
    }
    share = (double)E.g0 * lp - E.entropy_scale * h;
    if (!ABSORB) {   // tail sources written by earlier launches
#pragma unroll
      for (int q = 0; q < kMaxTails; ++q) {
        const int mask = q < R.tails ? R.tail_ext[q] : 0;
        if (mask == 0) continue;
        // every source slot and the factor read unconditionally (an unused slot reads the first
        // used one and adds +0): one memory round trip instead of one per load
        const int on0 = __builtin_ctz((unsigned)mask);
        for (int64_t k = first; k < E.K; k += stride) {
          float g = 0.0f;
#pragma unroll
          for (int src = 0; src < MI_MAX_SOURCES; ++src) {
            const bool on = (mask >> src) & 1;
            const int sc = on ? src : on0;
            g += keep_if(R.tail_src[q][sc][k * R.tail_src_stride[q][sc]], on);
          }
          const double2 d = *reinterpret_cast<const double2*>(R.tail_dgrad[q] + 2 * k);
          if (g == 0.0f) continue;   // a zero upstream never meets the factor
          c[q][0] += (double)g * d.x;
          c[q][1] += (double)g * d.y;
        }
      }
    }
  }
  MI_ELBO_STAMP(1);
  // the block's share and its tail partials in one pass: wave sums, then the waves in order
  // through LDS, one barrier (thread 0 stores the tail partials and returns the share)
  double s;
  {
    constexpr int kWaves = kElboThreads / kWave;
    constexpr int kVals = 1 + 2 * kMaxTails;
    __shared__ double wsum[kVals][kWaves];
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
    const double v0 = wave_sum(share);
    if (lane == 0) wsum[0][wave] = v0;
    const int tails = ABSORB ? 0 : R.tails;
    // the Normal tail's sums live on the particle lanes (the first kRedK <= 64 threads: wave 0)
    double nts0 = 0.0, nts1 = 0.0;
    if (!ABSORB && nt_slot >= 0 && wave == 0) {
      nts0 = wave_sum(nt[0]);
      nts1 = wave_sum(nt[1]);
    }
#pragma unroll
    for (int t = 0; t < kMaxTails; ++t)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (t < tails) {
          const double v = wave_sum(c[t][q]);
          if (lane == 0) wsum[1 + 2 * t + q][wave] = v;
        }
    __syncthreads();
    s = 0.0;
    if (threadIdx.x == 0) {
      for (int w = 0; w < kWaves; ++w) s += wsum[0][w];
      for (int t = 0; t < tails; ++t)
        for (int q = 0; q < 2; ++q) {
          double v = 0.0;
          for (int w = 0; w < kWaves; ++w) v += wsum[1 + 2 * t + q][w];
          __hip_atomic_store(&work[R.tail_part + ((int64_t)t * nshare + blockIdx.x) * 2 + q], v,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      if (!ABSORB && nt_slot >= 0) {
        double* w2 = &work[R.nt_part + ((int64_t)nt_slot * R.nt_nkb + nt_kb) * 2];
        __hip_atomic_store(w2, nts0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(w2 + 1, nts1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  MI_ELBO_STAMP(2);
  // mi_elbo_forward_adam: every share-writing block fetches the optimizer's descriptor (240 B, an
  // L2 hit after the first) into LDS while its completion count is in flight, so the last block
  // can issue the optimised tensors' loads with its first loads
  __shared__ mi_elbo_adam sad;
  const bool has_adam = !ABSORB && adam != nullptr;
  if (has_adam) {
    constexpr int kWords = (int)(sizeof(mi_elbo_adam) / sizeof(uint32_t));
    static_assert(kWords <= kElboThreads, "one descriptor word per thread");
    if ((int)threadIdx.x < kWords)
      reinterpret_cast<uint32_t*>(&sad)[threadIdx.x] =
          reinterpret_cast<const uint32_t*>(adam)[threadIdx.x];
  }
  if (threadIdx.x == 0) {
    // The shares (and the slot gradients the tail reads) are device-coherent stores, complete
    // (s_waitcnt) before the barrier / the counter update: no per-block L2 write-back fence,
    // which serialises over a few hundred reducing blocks.
    __hip_atomic_store(&work[blockIdx.x], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (MI_ELBO_RELEASE_FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_s_waitcnt(0);
    const int group = (int)blockIdx.x / kGroupBlocks;
    // (one level up to kSingleCount blocks: their arrivals at one address cost less than the
    // second level's round trip)
    const int ngroups = nshare <= kSingleCount ? 1 : (nshare + kGroupBlocks - 1) / kGroupBlocks;
    const unsigned in_group = (unsigned)min(kGroupBlocks, nshare - group * kGroupBlocks);
    unsigned* gc = counters + kGroupCounterWord + group * kGroupCounterStride;
    bool done = true;
    if (ngroups > 1) {
      done = atomicAdd(gc, 1u) == in_group - 1u;
      if (done) *gc = 0u;   // reset for the next launch (no other block of the group is left)
    }
    last = done && atomicAdd(counters, 1u) == (unsigned)(ngroups > 1 ? ngroups : nshare) - 1u;
  }
  MI_ELBO_STAMP(3);
  __syncthreads();
  if (!last) {
    MI_ELBO_FLUSH();
    return;
  }
  // the last block adds the shares: each thread a fixed strided subset, then a fixed-order block
  // sum -- deterministic, and no serial chain of dependent loads. Every load of this phase (shares,
  // the tails' partials and concentrations, the validation words, the generator step) is issued
  // before the first sum: one memory round trip instead of one per stage.
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  MI_ELBO_STAMP(10);
  // the optimised tensors' elements this thread updates (element threadIdx.x of every slot) and
  // their moments: loaded now, used when the gradient is written below. Lane q computes slot q's
  // bias corrections (fp64 pow: a long dependent chain) meanwhile, into LDS.
  float av[MI_ELBO_ADAM_SLOTS], am[MI_ELBO_ADAM_SLOTS], aq[MI_ELBO_ADAM_SLOTS];
  __shared__ AdamCoef sco[MI_ELBO_ADAM_SLOTS];
  __shared__ float sstep1[MI_ELBO_ADAM_SLOTS];
#pragma unroll
  for (int q = 0; q < MI_ELBO_ADAM_SLOTS; ++q) {
    av[q] = am[q] = aq[q] = 0.0f;
    if (has_adam && q < sad.num && (int64_t)threadIdx.x < sad.slots[q].numel &&
        !fin_factor(P, sad.slots[q].factor)) {
      const mi_elbo_adam_slot& A = sad.slots[q];
      av[q] = A.value[threadIdx.x];
      am[q] = A.exp_avg[threadIdx.x];
      aq[q] = A.exp_avg_sq[threadIdx.x];
    }
  }
  if (has_adam && (int)threadIdx.x < sad.num) {   // block 0's (visible after the sums' barrier below)
    const double* o = work + R.early + 3 * kMaxTails + 2 * threadIdx.x;
    const double d[2] = {__hip_atomic_load(o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                         __hip_atomic_load(o + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)};
    float v[4];
    __builtin_memcpy(v, d, sizeof(v));
    sstep1[threadIdx.x] = v[0];
    sco[threadIdx.x] = AdamCoef{v[1], v[2], v[3]};
  }
  // block 0's trigammas of the Beta tails (lane 3 q + which), loaded with the shares
  float tg_early = 0.0f;
  if (!ABSORB && (int)threadIdx.x < 3 * R.tails)
    tg_early = (float)__hip_atomic_load(work + R.early + threadIdx.x, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
  // the Beta tails' argument words, read here and pinned after the share loads below: lanes 0 / 1
  // read them after the tails' barrier otherwise, a dependent chain of scalar-cache misses there
  double hw[kMaxTails] = {};
  float* hout[kMaxTails][2] = {};
  int hexp[kMaxTails] = {};
  double* hpre[kMaxTails] = {};
  if (!ABSORB) {
#pragma unroll
    for (int q = 0; q < kMaxTails; ++q)
      if (q < R.tails) {
        const int f = R.tail_factor[q];
        hw[q] = -(double)1.0f * E.entropy_scale * factor_weight(E, f);
        hout[q][0] = factor_grad(E, f, 0);
        hout[q][1] = factor_grad(E, f, 1);
        hexp[q] = (factor_exp(E, f, 0) ? 1 : 0) | (factor_exp(E, f, 1) ? 2 : 0);
        hpre[q] = R.tail_saved[q];
      }
  }
  // the same for the Normal tail (factor 0)
  float* ngrad[2] = {E.factors[0].grad[0], E.factors[0].grad[1]};
  int64_t nstride[2] = {E.factors[0].grad_stride[0], E.factors[0].grad_stride[1]};
  int nexp = (E.factors[0].transform[0] == MI_TRANSFORM_EXP ? 1 : 0) |
             (E.factors[0].transform[1] == MI_TRANSFORM_EXP ? 2 : 0);
  double nw = -(double)1.0f * E.entropy_scale * E.factors[0].weight;
  double t = 0.0;
  double acc[kMaxTails][2] = {};
  auto ld = [](const double* w) {
    return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // kSU shares per lane per round, each load under its own (uniform per round) guard and all of
  // them issued before the first add: a loop of one share per iteration waited a memory round trip
  // per iteration (C2's 257 shares are two); the adds run in share order, as before
  constexpr int kSU = 2;
  for (int b0 = threadIdx.x; b0 < nshare; b0 += kSU * kElboThreads) {
    double x[kSU], y[kMaxTails][2][kSU];
#pragma unroll
    for (int u = 0; u < kSU; ++u) {
      const int b = b0 + u * kElboThreads;
      x[u] = 0.0;
#pragma unroll
      for (int q = 0; q < kMaxTails; ++q) y[q][0][u] = y[q][1][u] = 0.0;
      if (b < nshare) {
        x[u] = ld(&work[b]);
        if (!ABSORB) {
#pragma unroll
          for (int q = 0; q < kMaxTails; ++q)
            if (q < R.tails) {
              const double* w2 = &work[R.tail_part + ((int64_t)q * nshare + b) * 2];
              y[q][0][u] = ld(w2);
              y[q][1][u] = ld(w2 + 1);
            }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kSU; ++u) {
      t += x[u];
#pragma unroll
      for (int q = 0; q < kMaxTails; ++q) {
        acc[q][0] += y[q][0][u];
        acc[q][1] += y[q][1][u];
      }
    }
  }
  float tc1[kMaxTails] = {}, tc0[kMaxTails] = {};
  if (!ABSORB) {
    // (in vector registers: the values come out of selects and fp64 arithmetic)
    auto vpin = [](auto& v) { asm("" : "+v"(v)); };
#pragma unroll
    for (int q = 0; q < MI_ELBO_ADAM_SLOTS; ++q) {   // (the optimised elements' loads, too)
      vpin(av[q]);
      vpin(am[q]);
      vpin(aq[q]);
    }
    if (R.nt_job >= 0) {
      vpin(ngrad[0]);
      vpin(ngrad[1]);
      vpin(nstride[0]);
      vpin(nstride[1]);
      vpin(nexp);
      vpin(nw);
    }
#pragma unroll
    for (int q = 0; q < kMaxTails; ++q) {
      vpin(hw[q]);
      vpin(hout[q][0]);
      vpin(hout[q][1]);
      vpin(hexp[q]);
      vpin(hpre[q]);
    }
#pragma unroll
    for (int q = 0; q < kMaxTails; ++q)
      if (q < R.tails) {
        tc1[q] = *R.tail_c1[q];
        tc0[q] = *R.tail_c0[q];
      }
  }
  // the Normal tail's partial sums and parameters, fetched with the shares (one round trip)
  const bool nt_fin = !ABSORB && R.nt_job >= 0 && (E.options & MI_ELBO_FINAL_GRADS) &&
                      (int64_t)threadIdx.x < E.factors[0].n;
  double nt_s0 = 0.0, nt_s1 = 0.0;
  float nt_p0 = 1.0f, nt_p1 = 1.0f;
  // the one-element tail (nt_single: one partial per reducing block, hundreds of them) is summed by
  // every lane over a strided subset, then in a fixed order through LDS: a single lane's loop over
  // the blocks was a long chain at the end of the launch
  const bool nt_wide = !ABSORB && R.nt_job >= 0 && R.nt_single &&
                       (E.options & MI_ELBO_FINAL_GRADS);
  if (nt_fin) {
    const mi_factor& F = E.factors[0];
    const int64_t i = threadIdx.x;
    nt_p0 = F.param[0][i * F.stride[0]];
    nt_p1 = F.param[1][i * F.stride[1]];
    if (!nt_wide)   // (the particle blocks' partials: four per round, guarded, added in order)
      for (int kb0 = 0; kb0 < R.nt_nkb; kb0 += 4) {
        double x0[4], x1[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          x0[u] = x1[u] = 0.0;
          if (kb0 + u < R.nt_nkb) {
            const double* w2 = &work[R.nt_part + (i * R.nt_nkb + kb0 + u) * 2];
            x0[u] = ld(w2);
            x1[u] = ld(w2 + 1);
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          nt_s0 += x0[u];
          nt_s1 += x1[u];
        }
      }
  }
  if (nt_wide) {   // (element 0 of factor 0; the whole block, uniform branch)
    double q0 = 0.0, q1 = 0.0;
    for (int kb = threadIdx.x; kb < R.nt_nkb; kb += kElboThreads) {
      const double* w2 = &work[R.nt_part + (int64_t)kb * 2];
      q0 += __hip_atomic_load(w2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      q1 += __hip_atomic_load(w2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    q0 = wave_sum(q0);
    q1 = wave_sum(q1);
    __shared__ double ntw[2][kElboThreads / kWave];
    if ((threadIdx.x & (kWave - 1)) == 0) {
      ntw[0][threadIdx.x / kWave] = q0;
      ntw[1][threadIdx.x / kWave] = q1;
    }
    __syncthreads();
    if (threadIdx.x == 0)
      for (int w = 0; w < kElboThreads / kWave; ++w) {
        nt_s0 += ntw[0][w];
        nt_s1 += ntw[1][w];
      }
  }
  const uint32_t fw0 = (int64_t)threadIdx.x < E.nflags ? E.flags[threadIdx.x] : 0u;
  const uint64_t step0 = (threadIdx.x == 0 && E.step_counter != nullptr) ? *E.step_counter : 0ull;
  // the loss sum and the Beta tails' two sums through one barrier: wave sums, then the waves in a
  // fixed order (the loss's tree as before: each wave's lane-0 sum, waves 0..3 on thread 0); the tails' trigammas (block 0's, lanes 3 q .. 3 q + 2)
  // into LDS before it too
  __shared__ double tws[kMaxTails][2][kElboThreads / kWave];
  __shared__ float tg_all[3 * kMaxTails];
  double total = 0.0;
  {
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
    double* lred = rsum + kElboThreads / kWave;
    const double tw = wave_sum(t);
    if (lane == 0) lred[wave] = tw;
    if (!ABSORB) {
#pragma unroll
      for (int q = 0; q < kMaxTails; ++q) {
        if (q >= R.tails) break;
        const double w0 = wave_sum(acc[q][0]), w1 = wave_sum(acc[q][1]);
        if (lane == 0) {
          tws[q][0][wave] = w0;
          tws[q][1][wave] = w1;
        }
      }
      if ((int)threadIdx.x < 3 * R.tails) tg_all[threadIdx.x] = tg_early;
    }
    __syncthreads();
    if (threadIdx.x == 0)
      for (int w = 0; w < kElboThreads / kWave; ++w) total += lred[w];
  }
  MI_ELBO_STAMP(4);
  // the Adam update of element i of the tensor behind (factor f, parameter j), gradient g
  // (xv / xm / xq: the element's value and moments, av / am / aq unless a lane updates another
  // lane's element)
  auto adam_step_of = [&](int f, int j, int64_t i, float g, const float* xv, const float* xm,
                          const float* xq) {
    if (!has_adam) return;
    // the slot of (f, j) picked first, then one update: lanes of one wave with different (f, j)
    // (the split tails below) share the update's instructions instead of running one per slot
    int qs = -1;
    float pv = 0.0f, mv = 0.0f, vv = 0.0f;
#pragma unroll
    for (int q = 0; q < MI_ELBO_ADAM_SLOTS; ++q)
      if (q < sad.num && sad.slots[q].factor == f && sad.slots[q].param == j) {
        qs = q;
        pv = xv[q];
        mv = xm[q];
        vv = xq[q];
      }
    if (qs < 0) return;
    adam_update(sad, sco[qs], pv, g, mv, vv);
    const mi_elbo_adam_slot& A = sad.slots[qs];
    A.value[i] = pv;
    A.exp_avg[i] = mv;
    A.exp_avg_sq[i] = vv;
  };
  if (threadIdx.x == 0) {
    *loss = (float)total;
    *counters = 0u;
  }
  if (!ABSORB) {
#pragma unroll
    for (int q = 0; q < kMaxTails; ++q) {
      if (q >= R.tails) break;
      // (the sums and trigammas are in LDS, above; no barrier between the tails: each has its own
      // words)
      const float a = tc1[q], b = tc0[q];
      const float tsum = a + b;
      const float* tgs = tg_all + 3 * q;
      // element 0's value and moments on lane 1 too (lane j writes parameter j's gradient)
      float zv[MI_ELBO_ADAM_SLOTS], zm[MI_ELBO_ADAM_SLOTS], zq[MI_ELBO_ADAM_SLOTS];
#pragma unroll
      for (int s = 0; s < MI_ELBO_ADAM_SLOTS; ++s) {
        zv[s] = __shfl(av[s], 0);
        zm[s] = __shfl(am[s], 0);
        zq[s] = __shfl(aq[s], 0);
      }
      MI_ELBO_STAMP(11);
      if (threadIdx.x < 2) {   // pre = {sum dz dgrad0, sum dz dgrad1, dH/da, dH/db} (n = 1)
        const int j = threadIdx.x;
        double s0 = 0.0, s1 = 0.0;
        for (int w = 0; w < kElboThreads / kWave; ++w) {
          s0 += tws[q][0][w];
          s1 += tws[q][1][w];
        }
        const float tt = (tsum - 2.0f) * tgs[0];
        const double h0 = (double)(tt - (a - 1.0f) * tgs[1]);
        const double h1 = (double)(tt - (b - 1.0f) * tgs[2]);
        if (j == 0) {
          double* pre = hpre[q];
          pre[0] = s0;
          pre[1] = s1;
          pre[2] = h0;
          pre[3] = h1;
        }
        if (E.options & MI_ELBO_FINAL_GRADS) {
          // the gradients k_elbo_backward writes from `pre` for an upstream of 1 (same
          // arithmetic as write_grad: u * pre + w * dH with u = 1, w = -entropy_scale * weight,
          // times the parameter under an exp transform)
          const int f = R.tail_factor[q];
          const double w = hw[q];
          double g = j == 0 ? (double)1.0f * s0 + w * h0 : (double)1.0f * s1 + w * h1;
          // (j differs between the lanes: both parameters' words picked)
          float* out = j == 0 ? hout[q][0] : hout[q][1];
          if (out != nullptr) {
            if (hexp[q] & (1 << j)) g *= (double)(j == 0 ? a : b);
            out[0] = (float)g;
            adam_step_of(f, j, 0, (float)g, zv, zm, zq);
          }
        }
        MI_ELBO_STAMP(12);
      }
    }
  }
  MI_ELBO_STAMP(6);
  if (!ABSORB && R.nt_job >= 0 && (E.options & MI_ELBO_FINAL_GRADS)) {
    // the Normal tail's gradients for an upstream of 1: its blocks' sums in a fixed order, then
    // what k_elbo_backward's absorbed blocks write (u * s + w * dH, the exp chain rule)
    const mi_factor& F = E.factors[0];
    // up to 32 elements: lane i (parameter 0) and lane 32 + i (parameter 1) of wave 0 each write
    // one gradient and its Adam update, lane 32 + i with lane i's sums, parameters and moments
    // (shuffled while the whole wave is here); more elements: one thread each, both parameters
    const bool split = F.n <= kWave / 2;
    const int src = split ? (int)(threadIdx.x & (kWave / 2 - 1)) : (int)(threadIdx.x & (kWave - 1));
    float p0 = nt_p0, p1 = nt_p1;
    double s0 = nt_s0, s1 = nt_s1;
    float xv[MI_ELBO_ADAM_SLOTS], xm[MI_ELBO_ADAM_SLOTS], xq[MI_ELBO_ADAM_SLOTS];
#pragma unroll
    for (int s = 0; s < MI_ELBO_ADAM_SLOTS; ++s) {
      xv[s] = av[s];
      xm[s] = am[s];
      xq[s] = aq[s];
    }
    if (split) {
      p0 = __shfl(p0, src);
      p1 = __shfl(p1, src);
      s0 = __shfl(s0, src);
      s1 = __shfl(s1, src);
#pragma unroll
      for (int s = 0; s < MI_ELBO_ADAM_SLOTS; ++s) {
        xv[s] = __shfl(xv[s], src);
        xm[s] = __shfl(xm[s], src);
        xq[s] = __shfl(xq[s], src);
      }
    }
    const int64_t i = split ? src : (int64_t)threadIdx.x;
    // entropy_grad_of / write_grad_of of a Normal factor: dH = (0, 1 / scale)
    auto write = [&](int j, double g, float pv) {
      float* out = j == 0 ? ngrad[0] : ngrad[1];
      if (out == nullptr) return;
      if (nexp & (1 << j)) g *= (double)pv;
      out[i * (j == 0 ? nstride[0] : nstride[1])] = (float)g;
      adam_step_of(0, j, i, (float)g, xv, xm, xq);
    };
    const double w = nw;
    if (split) {
      if (threadIdx.x < kWave && i < F.n) {   // (one path for both halves: selects, not branches)
        const int j = threadIdx.x < kWave / 2 ? 0 : 1;
        const double g0 = (double)1.0f * s0 + w * 0.0, g1 = (double)1.0f * s1 + w * (double)(1.0f / p1);
        write(j, j == 0 ? g0 : g1, j == 0 ? p0 : p1);
      }
    } else if (nt_fin) {
      write(0, (double)1.0f * s0 + w * 0.0, p0);
      write(1, (double)1.0f * s1 + w * (double)(1.0f / p1), p1);
    }
  }
  MI_ELBO_STAMP(7);
  static_assert(sizeof(mi_elbo) + sizeof(AbsorbPlan) + sizeof(ReducePlan) + 4 * sizeof(void*) <= 4096,
                "k_elbo_forward's arguments exceed 4 KiB");
  static_assert(kGroupCounterWord + kGroupCounters * kGroupCounterStride <=
                    MI_ELBO_COUNTER_BYTES / sizeof(unsigned), "counter area");
  if ((int64_t)threadIdx.x < E.nflags) E.flags_mirror[threadIdx.x] = fw0;
  for (int64_t i = threadIdx.x + kElboThreads; i < E.nflags; i += kElboThreads)
    E.flags_mirror[i] = E.flags[i];
  if (threadIdx.x == 0 && E.step_counter != nullptr) {
    *E.step_snapshot = step0;
    *E.step_counter = step0 + 1;
  }
  // (lane q alone read slot q's count; a fused-draw factor's last reader advances its own)
  if (has_adam && (int)threadIdx.x < sad.num && !fin_factor(P, sad.slots[threadIdx.x].factor))
    *sad.slots[threadIdx.x].step = sstep1[threadIdx.x];
  MI_ELBO_STAMP(5);
  MI_ELBO_FLUSH();
}

// ---- backward -------------------------------------------------------------------------------
// Blocks [0, lead_blocks) write dterm, the entropy gradients of factors without an absorbed draw
// and rescale the speculative buffers; the blocks after them finish the absorbed factors.
__global__ __launch_bounds__(kElboThreads) void k_elbo_backward(const mi_elbo E,
                                                                const AbsorbPlan P,
                                                                const float* __restrict__ upstream,
                                                                float* __restrict__ dterm,
                                                                unsigned* __restrict__ counters,
                                                                double* __restrict__ work) {
  __shared__ double red[kElboThreads][2];
  __shared__ bool last;
  const float u = *upstream;
  if ((int)blockIdx.x >= P.lead_blocks) {
    absorbed_block<false>(E, P, (int)blockIdx.x - P.lead_blocks, u, counters, work, red, &last);
    return;
  }
  // d loss / d param = -u * entropy_scale * dH / d param
  const double w = -(double)u * E.entropy_scale;
  const int64_t stride = (int64_t)P.lead_blocks * kElboThreads;
  const int64_t first = (int64_t)blockIdx.x * kElboThreads + threadIdx.x;
  if (first == 0) dterm[0] = u * E.g0;
  for (int f = 0; f < E.num_factors; ++f) {
    const mi_factor& F = E.factors[f];
    if (F.draw_kind != MI_DRAW_NONE) continue;
    for (int64_t i = first; i < F.n; i += stride) {
      const Params2 q = load_params(F, i);
      double d0, d1;
      entropy_grad_of(F, q, d0, d1);
      write_grad_of(F, 0, i, w * F.weight * d0, q);
      write_grad_of(F, 1, i, w * F.weight * d1, q);
    }
  }
  if (u == 1.0f) return;  // the site groups' gradients were computed for exactly this upstream
  for (int b = 0; b < E.num_buffers; ++b) {
    float* x = E.buffers[b];
    const int64_t n = E.buffer_len[b];
    for (int64_t v = first; v < n; v += stride) x[v] *= u;
  }
}

}  // namespace mi

namespace {

int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

bool valid_factor(const mi_factor& F) {
  if (!(F.weight > 0.0) || !std::isfinite(F.weight) || F.element_offset < 0 ||
      (F.element_offset & 3) != 0)
    return false;
  if (F.n < 1 || (F.family != MI_NORMAL && F.family != MI_BETA && F.family != MI_GAMMA) ||
      F.param[1] == nullptr || ((F.family == MI_BETA || F.family == MI_GAMMA) && F.param[0] == nullptr) ||
      (F.family == MI_GAMMA && F.draw_kind != MI_DRAW_NONE))
    return false;
  for (int j = 0; j < 2; ++j) {
    if (F.transform[j] != MI_TRANSFORM_NONE && F.transform[j] != MI_TRANSFORM_EXP) return false;
    if (F.grad[j] != nullptr && F.n > 1 && F.grad_stride[j] == 0) return false;
    if (F.grad[j] != nullptr && F.transform[j] == MI_TRANSFORM_EXP && F.param[j] == nullptr)
      return false;
  }
  switch (F.draw_kind) {
    case MI_DRAW_NONE: return true;
    case MI_DRAW_SOURCES:
      if (F.num_sources < 0 || F.num_sources > MI_MAX_SOURCES) return false;
      for (int s = 0; s < F.num_sources; ++s)
        if (F.source[s].ptr == nullptr) return false;
      if (F.family == MI_BETA) return F.draws != nullptr;
      return F.param[0] != nullptr;
    case MI_DRAW_PARTIALS:
      return F.family == MI_NORMAL && F.partial[0] != nullptr && F.partial[1] != nullptr &&
             F.partial_rows >= 1;
    default: return false;
  }
}

bool forward_absorbed(const mi_factor& F) {
  return F.family == MI_BETA && F.draw_kind == MI_DRAW_SOURCES;
}

bool valid_reduce(const mi_elbo* e, const mi_reduce& r) {
  return r.part != nullptr && r.total != nullptr && r.K == e->K && r.nseg >= 1 &&
         r.nseg <= MI_REDUCE_MAX_SEG && r.num_sites >= 1 && r.num_sites <= MI_MAX_SITES &&
         r.num_slots >= 0 && (r.num_slots == 0 || r.slot_grad != nullptr);
}

bool valid(const mi_elbo* e) {
  if (e == nullptr || e->K < 1 || e->num_terms < 0 || e->num_terms > MI_MAX_TERMS ||
      e->num_factors < 0 || e->num_factors > MI_MAX_FACTORS || e->num_buffers < 0 ||
      e->num_buffers > MI_MAX_BUFFERS || e->num_reduce < 0 || e->num_reduce > MI_MAX_REDUCE ||
      e->nflags < 0 || (e->nflags > 0 && (e->flags == nullptr || e->flags_mirror == nullptr)) ||
      ((e->step_counter == nullptr) != (e->step_snapshot == nullptr)))
    return false;
  for (int r = 0; r < e->num_reduce; ++r)
    if (!valid_reduce(e, e->reduce[r])) return false;
  for (int t = 0; t < e->num_terms; ++t)
    if (e->terms[t] == nullptr) return false;
  for (int f = 0; f < e->num_factors; ++f)
    if (!valid_factor(e->factors[f])) return false;
  for (int b = 0; b < e->num_buffers; ++b)
    if (e->buffers[b] == nullptr || e->buffer_len[b] < 0) return false;
  for (int f = 0; f < e->num_factors; ++f)
    if (forward_absorbed(e->factors[f]) && e->factors[f].saved == nullptr) return false;
  return true;
}

// Enough blocks that each thread handles about four elements of the longest term or factor.
unsigned blocks_for(int64_t longest, int64_t cap) {
  return (unsigned)std::max<int64_t>(
      1, std::min<int64_t>(cap, ceil_div(longest, 4 * mi::kElboThreads)));
}

int64_t longest_factor(const mi_elbo* e) {
  int64_t n = 1;
  for (int f = 0; f < e->num_factors; ++f) n = std::max(n, e->factors[f].n);
  return n;
}


// Counter words (uint32) of the workspace: [0] the forward loss counter, absorbed-draw columns
// from kCounterFirst on; the forward's group counters (kGroupCounters words, 64 bytes apart) in
// between.
constexpr int64_t kCounterFirst = mi::kGroupCounterWord + mi::kGroupCounters * mi::kGroupCounterStride;
constexpr int64_t kMaxCounters = MI_ELBO_COUNTER_BYTES / sizeof(unsigned);

// Launch plans of both kernels and the layout of the fp64 work area that follows the counters:
// [loss partials | forward absorbed partials | backward absorbed partials]. All of it is scratch
// of one launch; what the backward needs from the forward lives in the caller's mi_factor.saved.
struct Layout {
  mi::AbsorbPlan fwd, bwd;
  // MI_ELBO_FINAL_GRADS: the fused-draw factors' backward blocks, run by the forward launch
  // (lead_blocks: the forward's)
  mi::AbsorbPlan fin;
  mi::ReducePlan red;
  int64_t doubles;
};

// quads per lane of partial_lane_quads (measured on C5, two partial rows of 1e6: step 0.2427 ms
// with 2, 0.2457-0.2484 without)
constexpr int kQuads = 2;

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// partial_lane_quads' layout: a Normal factor of whole quads, unit strides, 16-byte aligned rows
bool quad_layout(const mi_factor& F) {
  if (F.family != MI_NORMAL || (F.n & 3) != 0 || F.stride[1] != 1 || !aligned16(F.param[1]) ||
      !aligned16(F.partial[0]) || !aligned16(F.partial[1]))
    return false;
  if (F.transform[0] == MI_TRANSFORM_EXP && (F.stride[0] != 1 || !aligned16(F.param[0])))
    return false;
  for (int j = 0; j < 2; ++j)
    if (F.grad[j] != nullptr && (F.grad_stride[j] != 1 || !aligned16(F.grad[j]))) return false;
  return true;
}

// finish: the backward only combines the sums the forward left in F.saved
void add_absorbed(const mi_elbo* e, int f, bool forward, bool finish, mi::AbsorbPlan& P,
                  int64_t& counters, int64_t& doubles, int& blocks) {
  const mi_factor& F = e->factors[f];
  const int a = P.num++;
  P.index[a] = f;
  P.first[a] = blocks;
  P.pre[a] = 0;
  if (!forward && finish) {   // finish only: one element per thread
    P.pre[a] = 1;
    P.epl[a] = 1;
    P.ti[a] = mi::kElboThreads;
    P.gx[a] = (int)ceil_div(F.n, mi::kElboThreads);
    P.slices[a] = 1;
    P.rows_per_slice[a] = 1;
    blocks += P.gx[a];
    return;
  }
  const int64_t rows = F.draw_kind == MI_DRAW_PARTIALS ? F.partial_rows : e->K;
  // rows per particle lane: one Beta gradient per thread (long fp64 chains) unless they were
  // precomputed (then 16: a column's sums usually fit one block, no cross-block completion)
  const int64_t per_lane = !forward_absorbed(F) ? 4 : (F.dgrad == nullptr ? 1 : 16);
  // lanes along the rows: enough for per_lane rows each (few rows, e.g. a fused draw's
  // per-particle-block partials: one lane, 256 elements per block); the rest along the elements
  int tk = 1;
  while (tk < mi::kElboThreads && tk < ceil_div(rows, per_lane)) tk <<= 1;
  int ti = mi::kElboThreads / tk;
  int ti_need = 1;
  while (ti_need < ti && ti_need < F.n) ti_need <<= 1;
  if (ti_need < ti) {   // fewer elements than lanes: more lanes along the rows
    ti = ti_need;
    tk = mi::kElboThreads / ti;
  }
  const int64_t gx = ceil_div(F.n, ti);
  int64_t slices = ceil_div(rows, (int64_t)tk * per_lane);
  slices = std::max<int64_t>(1, std::min<int64_t>(slices, ceil_div(2048, gx)));
  if (slices > 1 && counters + gx > kMaxCounters) slices = 1;
  const int64_t rps = ceil_div(rows, slices);
  slices = ceil_div(rows, rps);
  // a backward over a few partial rows, one lane per element: four elements per lane instead
  P.epl[a] = (!forward && F.draw_kind == MI_DRAW_PARTIALS && tk == 1 && slices == 1) ? 4 : 1;
  // ... as 16-byte quads when the layout allows
  if (P.epl[a] == 4 && quad_layout(F)) P.epl[a] = -kQuads;
  P.ti[a] = ti;
  P.gx[a] = (int)(P.epl[a] == 4    ? ceil_div(F.n, (int64_t)ti * 4)
                  : P.epl[a] < 0 ? ceil_div(F.n >> 2, (int64_t)ti * -P.epl[a])
                                 : gx);
  P.slices[a] = (int)slices;
  P.rows_per_slice[a] = rps;
  P.counter[a] = counters;
  P.partial[a] = doubles;
  if (slices > 1) {
    counters += gx;
    doubles += slices * F.n * 2;
  }
  blocks += (int)(P.gx[a] * slices);
}

// particles per reducing block for long segment lists (measured on MI355X, C2: 16 / 32 / 64)
constexpr int kKred = 32;
// particles per reducing block for very long segment lists over few particles (8 or 16)
constexpr int kKredLong = 16;
// lead blocks (measured on MI355X, C5, steady clocks: 32 -> 0.2077-0.2079 ms, 16 -> 0.2091-0.2093)
constexpr int kLead = 32;

Layout make_layout(const mi_elbo* e) {
  Layout L{};
  // about 32 elements per lane of the longest term or factor (a lane's quads loaded four at a
  // time): C5's 1e6-element scale entropy in 123 lead blocks instead of 977 -- the launch's
  // 223-VGPR blocks fit two per CU, so a larger grid runs in several rounds
  L.fwd.lead_blocks = (int)std::max<int64_t>(
      1, std::min<int64_t>(mi::kElboMaxBlocks,
                           ceil_div(std::max(e->K, longest_factor(e)), kLead * mi::kElboThreads)));
  int64_t longest = 1;
  for (int f = 0; f < e->num_factors; ++f)
    if (e->factors[f].draw_kind == MI_DRAW_NONE) longest = std::max(longest, e->factors[f].n);
  for (int b = 0; b < e->num_buffers; ++b) longest = std::max(longest, e->buffer_len[b]);
  L.bwd.lead_blocks = (int)blocks_for(longest, 2048);
  int nred = 0;
  L.red.num = e->num_reduce;
  for (int r = 0; r < e->num_reduce; ++r) {
    const mi_reduce& J = e->reduce[r];
    L.red.first[r] = nred;
    L.red.vblocks[r] = J.num_sites == 1 ? J.num_sites + J.num_slots : 1;
    // long lists over few particles (a fused draw's block rows: ~1000 segments, K = 128): 16
    // particles x 16 segment groups per block, for more blocks and fewer serial loads per lane
    // (very long lists, C5's 977 block rows: 8 particles per block, two rounds of loads per lane
    // instead of four -- 0.3 us per C5 step, tools/gpurun_r05/t29.sh; C4's 513 keep 16: 8 was
    // 1.1 us slower there in r04)
    L.red.kred[r] = (J.nseg >= 768 && J.K < 2048)                       ? 8
                    : (J.nseg >= 512 && J.K < 2048)                     ? kKredLong
                    : (J.nseg >= 64 && kKred != mi::kRedKWide) ? kKred
                                                                     : mi::kRedKWide;
    nred += (int)ceil_div(J.K, L.red.kred[r]) * L.red.vblocks[r];
  }
  L.red.first[L.red.num] = nred;
  if (nred + L.fwd.lead_blocks > mi::kGroupCounters * mi::kGroupBlocks) {
    // too many blocks for the completion counters: mi_elbo_forward launches the reductions on
    // their own first and the lead blocks add the totals
    L.red.external = 1;
    for (int r = 0; r <= L.red.num; ++r) L.red.first[r] = 0;
    nred = 0;
  }
  // With deferred reductions, forward-absorbed Beta factors (which read slot gradients the
  // reductions write) are summed in this launch when they are tails (one element, dgrad
  // precomputed), else in the backward launch (mi_elbo_forward checked that they have dgrad).
  const bool deferred = e->num_reduce > 0;
  const int nshare = nred + L.fwd.lead_blocks;
  bool tail[MI_MAX_FACTORS] = {};
  if (deferred)
    for (int f = 0; f < e->num_factors; ++f) {
      const mi_factor& F = e->factors[f];
      if (!forward_absorbed(F) || F.dgrad == nullptr || F.n != 1 || L.red.tails >= mi::kMaxTails)
        continue;
      const int t = L.red.tails++;
      tail[f] = true;
      L.red.tail_dgrad[t] = F.dgrad;
      L.red.tail_c1[t] = F.param[0];
      L.red.tail_c0[t] = F.param[1];
      L.red.tail_saved[t] = F.saved;
      L.red.tail_factor[t] = f;
      for (int src = 0; src < F.num_sources; ++src) {
        const mi_source& S = F.source[src];
        bool matched = false;
        for (int r = 0; r < e->num_reduce && !L.red.external && S.stride_k == 1; ++r) {
          const mi_reduce& J = e->reduce[r];
          for (int j = 0; j < J.num_slots && j < MI_MAX_SLOTS; ++j)
            if (S.ptr == J.slot_grad + (int64_t)j * J.K) {
              L.red.tail_slot[r * MI_MAX_SLOTS + j] |= 1 << t;
              matched = true;
            }
        }
        if (!matched) {
          L.red.tail_ext[t] |= 1 << src;
          L.red.tail_src[t][src] = S.ptr;
          L.red.tail_src_stride[t][src] = S.stride_k;
        }
      }
    }
  L.red.nt_job = -1;
  if (deferred && !L.red.external)
    for (int f = 0; f < 1 && f < e->num_factors; ++f) {   // factor 0 only (ReducePlan.nt_job)
      const mi_factor& F = e->factors[f];
      if (tail[f] || F.family != MI_NORMAL || F.draw_kind != MI_DRAW_SOURCES ||
          F.n > mi::kElboThreads || F.eps != nullptr)
        continue;
      if (F.n == 1 && F.num_sources >= 1) {
        // one element, sources anywhere among the jobs' slots
        int mask[MI_MAX_REDUCE] = {};
        int matched = 0;
        for (int src = 0; src < F.num_sources; ++src) {
          const mi_source& S = F.source[src];
          for (int r = 0; r < e->num_reduce && S.stride_k == 1; ++r) {
            const mi_reduce& J = e->reduce[r];
            const int64_t off = S.ptr - J.slot_grad;
            if (J.slot_grad == nullptr || off < 0 || off % J.K != 0 || off / J.K >= J.num_slots ||
                off / J.K >= 31)
              continue;
            mask[r] |= 1 << (int)(off / J.K);
            ++matched;
            break;
          }
        }
        if (matched == F.num_sources) {
          L.red.nt_single = 1;
          for (int r = 0; r < MI_MAX_REDUCE; ++r) L.red.nt_mask[r] = mask[r];
          L.red.nt_job = 0;
          L.red.nt_j0 = 0;
          L.red.nt_nkb = nred;
          tail[f] = true;
        }
        continue;
      }
      if (F.num_sources != 1) continue;
      const mi_source& S = F.source[0];
      for (int r = 0; r < e->num_reduce; ++r) {
        const mi_reduce& J = e->reduce[r];
        if (J.num_sites != 1 || J.num_slots < 1 || S.stride_k != 1 || S.stride_i != J.K) continue;
        const int64_t off = S.ptr - J.slot_grad;
        if (off < 0 || off % J.K != 0 || off / J.K + F.n > J.num_slots) continue;
        L.red.nt_job = r;
        L.red.nt_j0 = (int)(off / J.K);
        L.red.nt_nkb = (int)ceil_div(J.K, L.red.kred[r]);
        tail[f] = true;
        break;
      }
    }
  int64_t counters = kCounterFirst;
  int64_t doubles = (nshare + 31) / 32 * 32;
  L.red.tail_part = doubles;
  doubles += (int64_t)L.red.tails * nshare * 2;
  L.red.nt_part = doubles;
  if (L.red.nt_job >= 0) doubles += e->factors[0].n * (int64_t)L.red.nt_nkb * 2;
  L.red.early = doubles;
  doubles += mi::kEarlyDoubles;
  int blocks = 0;
  for (int f = 0; f < e->num_factors; ++f)
    if (forward_absorbed(e->factors[f]) && !deferred)
      add_absorbed(e, f, true, false, L.fwd, counters, doubles, blocks);
  L.fwd.first[L.fwd.num] = blocks;
  for (int a = 0; a < L.fwd.num; ++a) L.fwd.pre[a] = 1;   // writes F.saved
  blocks = 0;
  for (int f = 0; f < e->num_factors; ++f)
    if (e->factors[f].draw_kind != MI_DRAW_NONE) {
      // the forward left the sums in F.saved: its absorbed blocks (no deferred reductions) or
      // its tail partials
      const bool finish = forward_absorbed(e->factors[f]) && (!deferred || tail[f]) &&
                          e->factors[f].family == MI_BETA;
      add_absorbed(e, f, false, finish, L.bwd, counters, doubles, blocks);
    }
  L.bwd.first[L.bwd.num] = blocks;
  L.fin.lead_blocks = L.fwd.lead_blocks;
  blocks = 0;
  if (!L.red.external)
    for (int f = 0; f < e->num_factors; ++f)
      if (e->factors[f].draw_kind == MI_DRAW_PARTIALS)
        add_absorbed(e, f, false, false, L.fin, counters, doubles, blocks);
  L.fin.first[L.fin.num] = blocks;
  L.doubles = doubles;
  return L;
}

// With MI_ELBO_FINAL_GRADS the forward finishes every factor: one-element Beta tails, the Normal
// tail (nt_job) and the fused-draw factors (Layout.fin) -- nothing left for the backward at an
// upstream of 1.
bool final_complete(const mi_elbo* e, const Layout& L) {
  const int finished = L.red.tails + (L.red.nt_job >= 0 ? 1 : 0) + L.fin.num;
  return e->num_factors > 0 && finished == e->num_factors && !L.red.external && L.fwd.num == 0;
}

size_t workspace_need(const mi_elbo* e) {
  return MI_ELBO_COUNTER_BYTES + sizeof(double) * (size_t)make_layout(e).doubles;
}

int to_code(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

}  // namespace

#if MI_ELBO_TIMING
static unsigned long long* mi_elbo_timing_last = nullptr;
#endif

extern "C" {

#if MI_ELBO_TIMING
// Copy the stamps of the last k_elbo_forward (16 per block) to the host (timing builds only).
int mi_elbo_timing_read(void* host, size_t bytes) {
  if (mi_elbo_timing_last == nullptr) return MI_EINVAL;
  return hipMemcpy(host, mi_elbo_timing_last, bytes < (8u << 20) ? bytes : (8u << 20),
                   hipMemcpyDeviceToHost) == hipSuccess ? 0 : MI_EINVAL;
}
#endif

int mi_elbo_struct_sizes(size_t* factor, size_t* elbo) {
  if (factor == nullptr || elbo == nullptr) return MI_EINVAL;
  *factor = sizeof(mi_factor);
  *elbo = sizeof(mi_elbo);
  return 0;
}

int mi_elbo_final_grads(const mi_elbo* elbo, int* complete) {
  if (!valid(elbo) || complete == nullptr) return MI_EINVAL;
  const Layout L = make_layout(elbo);
  *complete = final_complete(elbo, L) ? 1 : 0;
  return 0;
}

int mi_elbo_workspace_bytes(const mi_elbo* elbo, size_t* bytes) {
  if (!valid(elbo) || bytes == nullptr) return MI_EINVAL;
  *bytes = workspace_need(elbo);
  return 0;
}

int mi_elbo_workspace_init(void* workspace, size_t workspace_bytes, void* stream) {
  if (workspace == nullptr || workspace_bytes < MI_ELBO_COUNTER_BYTES) return MI_EINVAL;
  return to_code(
      hipMemsetAsync(workspace, 0, MI_ELBO_COUNTER_BYTES, static_cast<hipStream_t>(stream)));
}

int mi_elbo_adam_supported(const mi_elbo* elbo, const mi_elbo_adam* adam, int* supported) {
  if (!valid(elbo) || adam == nullptr || supported == nullptr) return MI_EINVAL;
  *supported = 0;
  if (!(elbo->options & MI_ELBO_FINAL_GRADS) || adam->num < 1 || adam->num > MI_ELBO_ADAM_SLOTS)
    return 0;
  const Layout L = make_layout(elbo);
  if (!final_complete(elbo, L) || L.fwd.num != 0) return 0;
  for (int q = 0; q < adam->num; ++q) {
    const mi_elbo_adam_slot& A = adam->slots[q];
    if (A.factor < 0 || A.factor >= elbo->num_factors || A.param < 0 || A.param > 1 ||
        A.value == nullptr || A.exp_avg == nullptr || A.exp_avg_sq == nullptr || A.step == nullptr)
      return MI_EINVAL;
    for (int r = 0; r < q; ++r)
      if (adam->slots[r].factor == A.factor && adam->slots[r].param == A.param) return MI_EINVAL;
    const mi_factor& F = elbo->factors[A.factor];
    if (F.grad[A.param] == nullptr || A.numel != F.n) return 0;
    int fa = -1;
    for (int a = 0; a < L.fin.num; ++a)
      if (L.fin.index[a] == A.factor) fa = a;
    if (fa >= 0) return 0;   // (written by the fused-draw blocks: Adam's own launch streams them)
    bool tail = false;
    for (int t = 0; t < L.red.tails; ++t) tail |= L.red.tail_factor[t] == A.factor;
    const bool nt = L.red.nt_job >= 0 && A.factor == 0;
    // written by the last block: a one-element Beta tail, or the Normal tail's elements (one per
    // thread)
    if (!((tail && F.n == 1) || (nt && F.n <= mi::kElboThreads))) return 0;
  }
  *supported = 1;
  return 0;
}

int mi_elbo_forward(const mi_elbo* elbo, void* workspace, size_t workspace_bytes, float* loss,
                    void* stream) {
  return mi_elbo_forward_adam(elbo, workspace, workspace_bytes, loss, nullptr, stream);
}

int mi_elbo_forward_adam(const mi_elbo* elbo, void* workspace, size_t workspace_bytes,
                         float* loss, const mi_elbo_adam* adam, void* stream) {
  if (!valid(elbo) || loss == nullptr || workspace == nullptr) return MI_EINVAL;
  if (workspace_bytes < workspace_need(elbo)) return MI_EWORKSPACE;
  if (elbo->num_reduce > 0)
    for (int f = 0; f < elbo->num_factors; ++f)
      if (forward_absorbed(elbo->factors[f]) && elbo->factors[f].dgrad == nullptr)
        return MI_EUNSUPPORTED;
  const Layout L = make_layout(elbo);
  auto* counters = static_cast<unsigned*>(workspace);
  auto* work = reinterpret_cast<double*>(static_cast<char*>(workspace) + MI_ELBO_COUNTER_BYTES);
  if (L.red.external)
    for (int r = 0; r < elbo->num_reduce; ++r) {
      const int rc = mi_reduce_launch(&elbo->reduce[r], stream);
      if (rc != 0) return rc;
    }
  bool has_beta = false;
  for (int f = 0; f < elbo->num_factors; ++f) has_beta |= elbo->factors[f].family != MI_NORMAL;
  // the fused-draw factors' final gradients (blocks after the share-writing ones; only launches
  // without forward-absorbed Beta blocks, which use that range)
  const bool fin = (elbo->options & MI_ELBO_FINAL_GRADS) && L.fin.num > 0 && L.fwd.num == 0 &&
                   final_complete(elbo, L);
  const int extra = L.fwd.num > 0 ? L.fwd.first[L.fwd.num] : fin ? L.fin.first[L.fin.num] : 0;
  const dim3 grid((unsigned)(L.red.first[L.red.num] + L.fwd.lead_blocks + extra));
  const mi::AbsorbPlan& plan = fin ? L.fin : L.fwd;
  hipStream_t s = static_cast<hipStream_t>(stream);
#if MI_ELBO_TIMING
  {
    static unsigned long long* tb = nullptr;
    if (tb == nullptr && hipMalloc(&tb, 8 << 20) != hipSuccess) return MI_EWORKSPACE;
    hipMemsetAsync(tb, 0, 8 << 20, s);
    hipMemcpyToSymbolAsync(HIP_SYMBOL(mi::mi_elbo_tbuf), &tb, sizeof(tb), 0, hipMemcpyHostToDevice, s);
    mi_elbo_timing_last = tb;
  }
#endif
  const dim3 block(mi::kElboThreads);
  if (L.fwd.num > 0)
    hipLaunchKernelGGL((mi::k_elbo_forward<true, true>), grid, block, 0, s, *elbo, L.fwd, L.red,
                       work, counters, loss, nullptr);
  else if (has_beta)
    hipLaunchKernelGGL((mi::k_elbo_forward<true, false>), grid, block, 0, s, *elbo, plan, L.red,
                       work, counters, loss, adam);
  else
    hipLaunchKernelGGL((mi::k_elbo_forward<false, false>), grid, block, 0, s, *elbo, plan,
                       L.red, work, counters, loss, adam);
  return to_code(hipGetLastError());
}

int mi_elbo_backward(const mi_elbo* elbo, const float* upstream, float* dterm, void* workspace,
                     size_t workspace_bytes, void* stream) {
  if (!valid(elbo) || upstream == nullptr || dterm == nullptr || workspace == nullptr)
    return MI_EINVAL;
  if (workspace_bytes < workspace_need(elbo)) return MI_EWORKSPACE;
  const Layout L = make_layout(elbo);
  auto* counters = static_cast<unsigned*>(workspace);
  auto* work = reinterpret_cast<double*>(static_cast<char*>(workspace) + MI_ELBO_COUNTER_BYTES);
  const unsigned grid = (unsigned)(L.bwd.lead_blocks + L.bwd.first[L.bwd.num]);
  hipLaunchKernelGGL(mi::k_elbo_backward, dim3(grid), dim3(mi::kElboThreads), 0,
                     static_cast<hipStream_t>(stream), *elbo, L.bwd, upstream, dterm, counters,
                     work);
  return to_code(hipGetLastError());
}

}  // extern "C"
