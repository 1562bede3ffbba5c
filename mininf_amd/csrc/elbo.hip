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
#include "beta_grad.hpp"

#include <algorithm>

namespace mi {

constexpr int kElboThreads = 256;
constexpr int kElboMaxBlocks = 1024;

// fp32 digamma / trigamma for the Beta entropy, evaluated in the guide's dtype as torch does
// (torch.digamma / torch.polygamma(1, .) on float tensors). Recurrence up to x >= 6, then the
// asymptotic series.
MI_DEV float digammaf(float x) {
  float shift = 0.0f;
  while (x < 6.0f) {
    shift -= 1.0f / x;
    x += 1.0f;
  }
  const float r = 1.0f / (x * x);
  const float series = r * (1.0f / 12 - r * (1.0f / 120 - r * (1.0f / 252 - r * (1.0f / 240))));
  return shift + logf(x) - 0.5f / x - series;
}

MI_DEV float trigammaf(float x) {
  float acc = 0.0f;
  while (x < 6.0f) {
    acc += 1.0f / (x * x);
    x += 1.0f;
  }
  const float r = 1.0f / (x * x);
  return acc + 1.0f / x + 0.5f * r +
         r / x * (1.0f / 6 - r * (1.0f / 30 - r * (1.0f / 42 - r * (1.0f / 30))));
}

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

MI_DEV double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < kElboThreads / kWave; ++w) s += red[w];
  return s;
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
MI_DEV float source_sum(const mi_factor& F, int64_t k, int64_t i) {
  float g = 0.0f;
#pragma unroll
  for (int s = 0; s < MI_MAX_SOURCES; ++s)
    if (s < F.num_sources) g += F.source[s].ptr[k * F.source[s].stride_k + i * F.source[s].stride_i];
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
  if (BETA && F.dgrad != nullptr) {   // factors precomputed by mi_beta_dgrad
    for (int64_t k = r0; k < r1; k += tk) {
      const double g = (double)source_sum(F, k, i);
      if (g == 0.0) continue;   // as the evaluating branch: a zero upstream never meets the factor
      s0 += g * F.dgrad[2 * (k * n + i)];
      s1 += g * F.dgrad[2 * (k * n + i) + 1];
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
    for (int64_t k = r0; k < r1; k += tk) {
      const float g = source_sum(F, k, i);
      float e;
      if (F.eps != nullptr) {
        e = F.eps[k * n + i];
      } else {
        float q[4];
        guide_normals(F.seed, step, F.stream_id, (uint64_t)(i >> 2),
                      (uint64_t)(F.particle_offset + k), q);
        e = q[i & 3];
      }
      s0 += (double)g;
      s1 += (double)g * (double)e;
    }
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
  const double w = -(double)u * E.entropy_scale;
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
  if (i < F.n) draw_sums<FORWARD>(F, i, r0 + ty, r1, tk, s0, s1);
  red[threadIdx.x][0] = s0;
  red[threadIdx.x][1] = s1;
  __syncthreads();
  if (ty == 0) {   // fixed-order sum over the block's particle lanes
    s0 = s1 = 0.0;
    for (int r = 0; r < tk; ++r) {
      s0 += red[r * ti + tx][0];
      s1 += red[r * ti + tx][1];
    }
  }
  unsigned* counter = nullptr;
  if (slices > 1) {
    double* part = work + pick(P.partial, a);
    if (ty == 0 && i < F.n) {
      part[((int64_t)slice * F.n + i) * 2] = s0;
      part[((int64_t)slice * F.n + i) * 2 + 1] = s1;
    }
    __threadfence();
    __syncthreads();
    counter = counters + pick(P.counter, a) + col;
    if (threadIdx.x == 0) *last = atomicAdd(counter, 1u) == (unsigned)slices - 1u;
    __syncthreads();
    if (!*last) return;
    __threadfence();
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
    entropy_grad(F, i, d0, d1);
    if (FORWARD) {
      double* pre = F.saved + 4 * i;
      pre[0] = s0;
      pre[1] = s1;
      pre[2] = d0;
      pre[3] = d1;
    } else {
      write_grad(F, 0, i, (double)u * s0 + w * d0);
      write_grad(F, 1, i, (double)u * s1 + w * d1);
    }
  }
  if (counter != nullptr && threadIdx.x == 0) *counter = 0u;
}

// ---- forward --------------------------------------------------------------------------------
// HAS_BETA = false: only Normal factors (log of the scale), which keeps the register footprint
// of the common large-factor case small; true: any Beta or Gamma factor (generic entropy path).
template <bool HAS_BETA>
__global__ __launch_bounds__(kElboThreads) void k_elbo_forward(const mi_elbo E,
                                                               const AbsorbPlan P,
                                                               double* __restrict__ work,
                                                               unsigned* __restrict__ counters,
                                                               float* __restrict__ loss) {
  __shared__ double red[kElboThreads][2];
  __shared__ bool last;
  const int nloss = P.lead_blocks;
  if (HAS_BETA && (int)blockIdx.x >= nloss) {
    absorbed_block<true>(E, P, (int)blockIdx.x - nloss, 1.0f, counters, work, red, &last);
    return;
  }
  double* rsum = &red[0][0];
  const int64_t stride = (int64_t)nloss * kElboThreads;
  const int64_t first = (int64_t)blockIdx.x * kElboThreads + threadIdx.x;
  double lp = 0.0, h = 0.0;
  for (int t = 0; t < E.num_terms; ++t)
    for (int64_t k = first; k < E.K; k += stride) lp += (double)E.terms[t][k];
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
        for (int64_t q = first; q < nq; q += stride) {
          const float4 v = sq[q];
          hf += (logf(v.x) + logf(v.y)) + (logf(v.z) + logf(v.w));
        }
        head = nq << 2;
      }
      for (int64_t i = head + first; i < F.n; i += stride) hf += logf(sc[i * ss]);
      h += (double)hf;
      if (first == 0) h += 1.4189385332046727 * (double)F.n;
    } else {
      for (int64_t i = first; i < F.n; i += stride) h += factor_entropy(F, i);
    }
  }
  const double s = block_sum((double)E.g0 * lp - E.entropy_scale * h, rsum);
  if (threadIdx.x == 0) {
    work[blockIdx.x] = s;
    __threadfence();
    last = atomicAdd(counters, 1u) == (unsigned)nloss - 1u;
  }
  __syncthreads();
  if (last) {
    // the last block adds the partials: each thread a fixed strided subset, then a fixed-order
    // block sum -- deterministic, and no serial chain of dependent loads
    __threadfence();
    double t = 0.0;
    for (int b = threadIdx.x; b < nloss; b += kElboThreads) t += work[b];
    const double total = block_sum(t, rsum + kElboThreads / kWave);
    if (threadIdx.x == 0) {
      *loss = (float)total;
      *counters = 0u;
    }
  }
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
      double d0, d1;
      entropy_grad(F, i, d0, d1);
      write_grad(F, 0, i, w * d0);
      write_grad(F, 1, i, w * d1);
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

bool valid(const mi_elbo* e) {
  if (e == nullptr || e->K < 1 || e->num_terms < 0 || e->num_terms > MI_MAX_TERMS ||
      e->num_factors < 0 || e->num_factors > MI_MAX_FACTORS || e->num_buffers < 0 ||
      e->num_buffers > MI_MAX_BUFFERS)
    return false;
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
// from kCounterFirst on.
constexpr int64_t kCounterFirst = 64;
constexpr int64_t kMaxCounters = MI_ELBO_COUNTER_BYTES / sizeof(unsigned);

// Launch plans of both kernels and the layout of the fp64 work area that follows the counters:
// [loss partials | forward absorbed partials | backward absorbed partials]. All of it is scratch
// of one launch; what the backward needs from the forward lives in the caller's mi_factor.saved.
struct Layout {
  mi::AbsorbPlan fwd, bwd;
  int64_t doubles;
};

void add_absorbed(const mi_elbo* e, int f, bool forward, mi::AbsorbPlan& P, int64_t& counters,
                  int64_t& doubles, int& blocks) {
  const mi_factor& F = e->factors[f];
  const int a = P.num++;
  P.index[a] = f;
  P.first[a] = blocks;
  P.pre[a] = 0;
  if (!forward && forward_absorbed(F)) {   // finish only: one element per thread
    P.ti[a] = mi::kElboThreads;
    P.gx[a] = (int)ceil_div(F.n, mi::kElboThreads);
    P.slices[a] = 1;
    P.rows_per_slice[a] = 1;
    blocks += P.gx[a];
    return;
  }
  const int64_t rows = F.draw_kind == MI_DRAW_PARTIALS ? F.partial_rows : e->K;
  int ti = 1;
  while (ti < 64 && ti < F.n) ti <<= 1;
  const int tk = mi::kElboThreads / ti;
  const int64_t gx = ceil_div(F.n, ti);
  // rows per particle lane: one Beta gradient per thread (long fp64 chains) unless mi_beta_dgrad
  // precomputed them, a few otherwise
  const int64_t per_lane = (forward_absorbed(F) && F.dgrad == nullptr) ? 1 : 4;
  int64_t slices = ceil_div(rows, (int64_t)tk * per_lane);
  slices = std::max<int64_t>(1, std::min<int64_t>(slices, ceil_div(2048, gx)));
  if (slices > 1 && counters + gx > kMaxCounters) slices = 1;
  const int64_t rps = ceil_div(rows, slices);
  slices = ceil_div(rows, rps);
  P.ti[a] = ti;
  P.gx[a] = (int)gx;
  P.slices[a] = (int)slices;
  P.rows_per_slice[a] = rps;
  P.counter[a] = counters;
  P.partial[a] = doubles;
  if (slices > 1) {
    counters += gx;
    doubles += slices * F.n * 2;
  }
  blocks += (int)(gx * slices);
}

Layout make_layout(const mi_elbo* e) {
  Layout L{};
  L.fwd.lead_blocks = (int)blocks_for(std::max(e->K, longest_factor(e)), mi::kElboMaxBlocks);
  int64_t longest = 1;
  for (int f = 0; f < e->num_factors; ++f)
    if (e->factors[f].draw_kind == MI_DRAW_NONE) longest = std::max(longest, e->factors[f].n);
  for (int b = 0; b < e->num_buffers; ++b) longest = std::max(longest, e->buffer_len[b]);
  L.bwd.lead_blocks = (int)blocks_for(longest, 2048);
  int64_t counters = kCounterFirst;
  int64_t doubles = (L.fwd.lead_blocks + 31) / 32 * 32;
  int blocks = 0;
  for (int f = 0; f < e->num_factors; ++f)
    if (forward_absorbed(e->factors[f]))
      add_absorbed(e, f, true, L.fwd, counters, doubles, blocks);
  L.fwd.first[L.fwd.num] = blocks;
  for (int a = 0; a < L.fwd.num; ++a) L.fwd.pre[a] = 1;   // writes F.saved
  blocks = 0;
  for (int f = 0; f < e->num_factors; ++f)
    if (e->factors[f].draw_kind != MI_DRAW_NONE) {
      add_absorbed(e, f, false, L.bwd, counters, doubles, blocks);
      if (forward_absorbed(e->factors[f]))
        for (int a = 0; a < L.fwd.num; ++a)
          if (L.fwd.index[a] == f) L.bwd.pre[L.bwd.num - 1] = L.fwd.pre[a];
    }
  L.bwd.first[L.bwd.num] = blocks;
  L.doubles = doubles;
  return L;
}

size_t workspace_need(const mi_elbo* e) {
  return MI_ELBO_COUNTER_BYTES + sizeof(double) * (size_t)make_layout(e).doubles;
}

int to_code(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

}  // namespace

extern "C" {

int mi_elbo_struct_sizes(size_t* factor, size_t* elbo) {
  if (factor == nullptr || elbo == nullptr) return MI_EINVAL;
  *factor = sizeof(mi_factor);
  *elbo = sizeof(mi_elbo);
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

int mi_elbo_forward(const mi_elbo* elbo, void* workspace, size_t workspace_bytes, float* loss,
                    void* stream) {
  if (!valid(elbo) || loss == nullptr || workspace == nullptr) return MI_EINVAL;
  if (workspace_bytes < workspace_need(elbo)) return MI_EWORKSPACE;
  const Layout L = make_layout(elbo);
  auto* counters = static_cast<unsigned*>(workspace);
  auto* work = reinterpret_cast<double*>(static_cast<char*>(workspace) + MI_ELBO_COUNTER_BYTES);
  bool has_beta = false;
  for (int f = 0; f < elbo->num_factors; ++f) has_beta |= elbo->factors[f].family != MI_NORMAL;
  const dim3 grid((unsigned)(L.fwd.lead_blocks + L.fwd.first[L.fwd.num]));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (has_beta)
    hipLaunchKernelGGL(mi::k_elbo_forward<true>, grid, dim3(mi::kElboThreads), 0, s, *elbo,
                       L.fwd, work, counters, loss);
  else
    hipLaunchKernelGGL(mi::k_elbo_forward<false>, grid, dim3(mi::kElboThreads), 0, s, *elbo,
                       L.fwd, work, counters, loss);
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
