// The ELBO's scalar tail in two launches: forward reduces every per-particle log joint and the
// guide's entropy into the loss, backward writes the entropy gradients, hands the upstream gradient
// back to the site groups and rescales their speculative gradients only if it is not 1.
//
// Replaces, in the reference's EvidenceLowerBoundLoss.forward (mininf/nn.py:210-228):
//   `elbo = log_prob.total + approximation.entropy()` (nn.py:224-226) and `return -elbo`, where
//   FactorizedDistribution.entropy (nn.py:121-131) sums torch Normal.entropy (normal.py:112-113)
//   and Beta.entropy (beta.py:101-102 -> dirichlet.py:122-130) over factors and elements,
// plus every autograd kernel of those expressions (~50 small launches per step for a Beta guide).
//
// Reductions are deterministic: fixed grid, fp64 per-block partial sums, and the last block to
// finish (device-scope counter, reset by that block) adds the partials in a fixed order.
#include "common.hpp"

#include <algorithm>

namespace mi {

constexpr int kElboThreads = 256;
constexpr int kElboMaxBlocks = 1024;

// Trigamma psi'(x), x > 0: recurrence up to x >= 6, then the asymptotic series
// 1/x + 1/(2x^2) + sum_k B_2k / x^(2k+1).
MI_DEV double trigamma(double x) {
  double acc = 0.0;
  while (x < 6.0) {
    acc += 1.0 / (x * x);
    x += 1.0;
  }
  const double r = 1.0 / (x * x);
  const double series =
      1.0 / x + r / 2.0 +
      r / x * (1.0 / 6 - r * (1.0 / 30 - r * (1.0 / 42 - r * (1.0 / 30 - r * (5.0 / 66)))));
  return acc + series;
}

// Entropy of element i of factor f, and its partial derivatives w.r.t. the factor's parameters.
MI_DEV double factor_entropy(const mi_factor& f, int64_t i, double* d0, double* d1) {
  if (f.family == MI_NORMAL) {
    // 0.5 + 0.5 log(2 pi) + log(scale) in fp32 as torch evaluates it (normal.py:112-113); the
    // sum over elements is carried in fp64.
    const float s = f.param[1][i * f.stride[1]];
    if (d0 != nullptr) {
      *d0 = 0.0;
      *d1 = (double)(1.0f / s);
    }
    return (double)(1.4189385332046727f + logf(s));
  }
  // Beta(a, b) = Dirichlet([a, b]) (dirichlet.py:122-130 with k = 2, a0 = a + b):
  //   lgamma(a) + lgamma(b) - lgamma(a0) - (2 - a0) psi(a0) - (a - 1) psi(a) - (b - 1) psi(b)
  const float af = f.param[0][i * f.stride[0]], bf = f.param[1][i * f.stride[1]];
  const double a = (double)af, b = (double)bf;
  const double t = (double)(af + bf);  // concentration.sum(-1) in fp32
  if (d0 != nullptr) {
    const double tt = (t - 2.0) * trigamma(t);
    *d0 = -(a - 1.0) * trigamma(a) + tt;
    *d1 = -(b - 1.0) * trigamma(b) + tt;
  }
  return lgamma(a) + lgamma(b) - lgamma(t) - (2.0 - t) * digamma(t) - (a - 1.0) * digamma(a) -
         (b - 1.0) * digamma(b);
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

// HAS_BETA = false: only Normal factors (log of the scale), which keeps the register footprint
// of the common large-factor case small (the Beta path carries fp64 lgamma / digamma).
template <bool HAS_BETA>
__global__ __launch_bounds__(kElboThreads) void k_elbo_forward(const mi_elbo E, double* partial,
                                                               unsigned* __restrict__ counter,
                                                               float* __restrict__ loss) {
  __shared__ double red[2 * (kElboThreads / kWave)];
  __shared__ bool last;
  const int64_t stride = (int64_t)gridDim.x * kElboThreads;
  const int64_t first = (int64_t)blockIdx.x * kElboThreads + threadIdx.x;
  double lp = 0.0, h = 0.0;
  for (int t = 0; t < E.num_terms; ++t)
    for (int64_t k = first; k < E.K; k += stride) lp += (double)E.terms[t][k];
  for (int f = 0; f < E.num_factors; ++f) {
    const mi_factor& F = E.factors[f];
    if (!HAS_BETA || F.family == MI_NORMAL) {
      const float* __restrict__ sc = F.param[1];
      const int64_t ss = F.stride[1];
      float hf = 0.0f;   // per-thread partial of <= a few hundred terms, then fp64
      for (int64_t i = first; i < F.n; i += stride) hf += logf(sc[i * ss]);
      h += (double)hf + 1.4189385332046727 * (double)((F.n - first + stride - 1) / stride > 0 ?
                                                        (F.n - first + stride - 1) / stride : 0);
    } else {
      for (int64_t i = first; i < F.n; i += stride) h += factor_entropy(F, i, nullptr, nullptr);
    }
  }
  const double s = block_sum((double)E.g0 * lp - E.entropy_scale * h, red);
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = s;
    __threadfence();
    last = atomicAdd(counter, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (last) {
    // the last block adds the partials: each thread a fixed strided subset, then a fixed-order
    // block sum -- deterministic, and no serial chain of dependent loads
    __threadfence();
    double t = 0.0;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += kElboThreads) t += partial[b];
    const double total = block_sum(t, red + kElboThreads / kWave);
    if (threadIdx.x == 0) {
      *loss = (float)total;
      *counter = 0u;
    }
  }
}

__global__ __launch_bounds__(kElboThreads) void k_elbo_backward(const mi_elbo E,
                                                                const float* __restrict__ upstream,
                                                                float* __restrict__ dterm) {
  const float u = *upstream;
  const int64_t stride = (int64_t)gridDim.x * kElboThreads;
  const int64_t first = (int64_t)blockIdx.x * kElboThreads + threadIdx.x;
  if (first == 0) dterm[0] = u * E.g0;
  // d loss / d param = -u * entropy_scale * dH / d param
  const double w = -(double)u * E.entropy_scale;
  for (int f = 0; f < E.num_factors; ++f) {
    const mi_factor& F = E.factors[f];
    for (int64_t i = first; i < F.n; i += stride) {
      double d0, d1;
      factor_entropy(F, i, &d0, &d1);
      if (F.grad[0] != nullptr) F.grad[0][i * F.stride[0]] = (float)(w * d0);
      if (F.grad[1] != nullptr) F.grad[1][i * F.stride[1]] = (float)(w * d1);
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

bool valid(const mi_elbo* e) {
  if (e == nullptr || e->K < 1 || e->num_terms < 0 || e->num_terms > MI_MAX_TERMS ||
      e->num_factors < 0 || e->num_factors > MI_MAX_FACTORS || e->num_buffers < 0 ||
      e->num_buffers > MI_MAX_BUFFERS)
    return false;
  for (int t = 0; t < e->num_terms; ++t)
    if (e->terms[t] == nullptr) return false;
  for (int f = 0; f < e->num_factors; ++f) {
    const mi_factor& F = e->factors[f];
    if (F.n < 1 || (F.family != MI_NORMAL && F.family != MI_BETA) || F.param[1] == nullptr ||
        (F.family == MI_BETA && F.param[0] == nullptr))
      return false;
  }
  for (int b = 0; b < e->num_buffers; ++b)
    if (e->buffers[b] == nullptr || e->buffer_len[b] < 0) return false;
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

unsigned forward_blocks(const mi_elbo* e) {
  return blocks_for(std::max(e->K, longest_factor(e)), mi::kElboMaxBlocks);
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
  *bytes = 256 + sizeof(double) * (size_t)forward_blocks(elbo);
  return 0;
}

int mi_elbo_workspace_init(void* workspace, size_t workspace_bytes, void* stream) {
  if (workspace == nullptr || workspace_bytes < 256) return MI_EINVAL;
  return to_code(hipMemsetAsync(workspace, 0, 256, static_cast<hipStream_t>(stream)));
}

int mi_elbo_forward(const mi_elbo* elbo, void* workspace, size_t workspace_bytes, float* loss,
                    void* stream) {
  if (!valid(elbo) || loss == nullptr || workspace == nullptr) return MI_EINVAL;
  size_t need = 0;
  mi_elbo_workspace_bytes(elbo, &need);
  if (workspace_bytes < need) return MI_EWORKSPACE;
  auto* counter = static_cast<unsigned*>(workspace);
  auto* partial = reinterpret_cast<double*>(static_cast<char*>(workspace) + 256);
  bool has_beta = false;
  for (int f = 0; f < elbo->num_factors; ++f) has_beta |= elbo->factors[f].family == MI_BETA;
  if (has_beta)
    hipLaunchKernelGGL(mi::k_elbo_forward<true>, dim3(forward_blocks(elbo)),
                       dim3(mi::kElboThreads), 0, static_cast<hipStream_t>(stream), *elbo, partial,
                       counter, loss);
  else
    hipLaunchKernelGGL(mi::k_elbo_forward<false>, dim3(forward_blocks(elbo)),
                       dim3(mi::kElboThreads), 0, static_cast<hipStream_t>(stream), *elbo, partial,
                       counter, loss);
  return to_code(hipGetLastError());
}

int mi_elbo_backward(const mi_elbo* elbo, const float* upstream, float* dterm, void* stream) {
  if (!valid(elbo) || upstream == nullptr || dterm == nullptr) return MI_EINVAL;
  int64_t longest = longest_factor(elbo);
  for (int b = 0; b < elbo->num_buffers; ++b) longest = std::max(longest, elbo->buffer_len[b]);
  hipLaunchKernelGGL(mi::k_elbo_backward, dim3(blocks_for(longest, 2048)),
                     dim3(mi::kElboThreads), 0, static_cast<hipStream_t>(stream), *elbo, upstream,
                     dterm);
  return to_code(hipGetLastError());
}

}  // extern "C"
