// MultivariateNormal site density over a batch of lower-triangular factors: the log_prob of
// torch.distributions.MultivariateNormal (multivariate_normal.py:255-262, _batch_mahalanobis at
// :80-102) for the reference's Gaussian-process sites (examples/missing-observations.md:42),
// evaluated per particle after the covariance is factorised (rocSOLVER, float64, by the caller).
//
// One wave per batch item b (a particle): with r = value - loc,
//   w = L^-1 r        (forward substitution, right-looking: column i of L updates the rest of r)
//   u = L^-T w        (back substitution, row i of L: the gradient direction)
//   log_prob = -0.5 w.w - sum_i log L_ii - n/2 log(2 pi).
// The working vectors live in LDS (n <= MI_MVN_MAX_N); lane j owns elements j, j + 64, ...
// Factors with n <= kMvnLdsMaxN are staged in LDS by one coalesced pass, so each of the 2n
// dependent rounds reads LDS instead of making an L2 round trip; larger ones are read from global
// memory (L2-resident, n^2 doubles per particle). The kernel is latency bound either way.
// float64 throughout: the example's GP covariance (jitter 1e-3) is too ill-conditioned for a
// float32 solve, the reason the host path refactorises in float64 too.
#include "common.hpp"
#include "internal.hpp"

#include <cstdlib>

namespace mi {

constexpr int kMvnThreads = 64;
// factors up to this size are staged in LDS (row stride n + 1: column reads hit distinct banks)
constexpr int kMvnLdsMaxN = 80;   // 51.8 KB + the 8 KB vector: within 64 KB per workgroup

template <bool kLds>
__global__ __launch_bounds__(kMvnThreads) void k_mvn_tril(const double* __restrict__ value,
                                                          const double* __restrict__ loc,
                                                          const double* __restrict__ L, int n,
                                                          double* __restrict__ log_prob,
                                                          double* __restrict__ w_out,
                                                          double* __restrict__ u_out) {
  extern __shared__ double lds[];   // kLds: the factor, [n][n + 1]
  __shared__ double r[MI_MVN_MAX_N];
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const double* Lg = L + b * (int64_t)n * n;
  const int ld = kLds ? n + 1 : n;
  if (kLds) {
    for (int e = lane; e < n * n; e += kMvnThreads) lds[(e / n) * ld + e % n] = Lg[e];
  }
  const double* Lb = kLds ? lds : Lg;
  for (int j = lane; j < n; j += kMvnThreads) r[j] = value[b * n + j] - loc[b * n + j];
  __syncthreads();
  // forward substitution: r becomes w
  for (int i = 0; i < n; ++i) {
    const double wi = r[i] / Lb[i * ld + i];
    __syncthreads();   // every lane has read r[i]
    for (int j = lane; j < n; j += kMvnThreads) {
      if (j == i) r[j] = wi;
      else if (j > i) r[j] = fma(-Lb[j * ld + i], wi, r[j]);
    }
    __syncthreads();
  }
  double quad = 0.0, logdet = 0.0;
  for (int j = lane; j < n; j += kMvnThreads) {
    const double wj = r[j];
    quad = fma(wj, wj, quad);
    logdet += log(Lb[j * ld + j]);
    w_out[b * n + j] = wj;
  }
  for (int off = kMvnThreads / 2; off > 0; off >>= 1) {
    quad += __shfl_xor(quad, off);
    logdet += __shfl_xor(logdet, off);
  }
  if (lane == 0) log_prob[b] = -0.5 * quad - logdet - 0.5 * n * log(2.0 * M_PI);
  // back substitution: L^T u = w, r becomes u
  for (int i = n - 1; i >= 0; --i) {
    const double ui = r[i] / Lb[i * ld + i];
    __syncthreads();
    for (int j = lane; j < n; j += kMvnThreads) {
      if (j == i) r[j] = ui;
      else if (j < i) r[j] = fma(-Lb[i * ld + j], ui, r[j]);
    }
    __syncthreads();
  }
  for (int j = lane; j < n; j += kMvnThreads) u_out[b * n + j] = r[j];
}

// Cholesky factorisation A = L L^T of a batch of symmetric positive-definite matrices, float64
// arithmetic (inputs and outputs float32 or float64): one 256-thread workgroup per matrix,
// right-looking (column j: its diagonal, the column below it scaled, then the trailing lower
// triangle updated by the threads together). The working triangle lives in LDS for
// n <= kMvnLdsMaxN, else in the output buffer itself. info[b] = 0, or j + 1 for the first
// column whose pivot is not positive (torch.linalg.cholesky_ex's convention); the factor is then
// incomplete (NaN from that column on), as rocSOLVER leaves it.
constexpr int kCholThreads = 256;

template <typename TI, typename TO, bool kLds>
__global__ __launch_bounds__(kCholThreads) void k_cholesky(const TI* __restrict__ A, int n,
                                                           TO* __restrict__ Lout,
                                                           int* __restrict__ info) {
  extern __shared__ double wl[];   // kLds: [n][n + 1]
  __shared__ double piv;
  __shared__ int fail;
  const int64_t b = blockIdx.x;
  const int t = threadIdx.x;
  const TI* Ab = A + b * (int64_t)n * n;
  TO* Lb = Lout + b * (int64_t)n * n;
  const int ld = kLds ? n + 1 : n;
  double* W = kLds ? wl : nullptr;
  // the lower triangle of A (the upper one is never read, as in LAPACK's potrf 'L')
  auto at = [&](int i, int k) -> double& { return W[i * ld + k]; };
  if (kLds) {
    for (int e = t; e < n * n; e += kCholThreads) {
      const int i = e / n, k = e - i * n;
      if (k <= i) wl[i * ld + k] = (double)Ab[e];
    }
  }
  if (t == 0) fail = 0;
  __syncthreads();
  if constexpr (kLds) {
    for (int j = 0; j < n; ++j) {
      if (t == 0) {
        const double d = at(j, j);
        if (!(d > 0.0) && fail == 0) fail = j + 1;
        piv = sqrt(d);
        at(j, j) = piv;
      }
      __syncthreads();
      const double inv = 1.0 / piv;
      for (int i = j + 1 + t; i < n; i += kCholThreads) at(i, j) *= inv;
      __syncthreads();
      const int m = n - j - 1;
      for (int e = t; e < m * m; e += kCholThreads) {
        const int i = j + 1 + e / m, k = j + 1 + e % m;
        if (k <= i) at(i, k) = fma(-at(i, j), at(k, j), at(i, k));
      }
      __syncthreads();
    }
    for (int e = t; e < n * n; e += kCholThreads) {
      const int i = e / n, k = e - i * n;
      Lb[e] = k <= i ? (TO)wl[i * ld + k] : (TO)0;
    }
  } else {
    // in place in the output (double precision output only: see mi_cholesky)
    double* G = reinterpret_cast<double*>(Lb);
    for (int e = t; e < n * n; e += kCholThreads) {
      const int i = e / n, k = e - i * n;
      G[e] = k <= i ? (double)Ab[e] : 0.0;
    }
    __syncthreads();
    for (int j = 0; j < n; ++j) {
      if (t == 0) {
        const double d = G[j * n + j];
        if (!(d > 0.0) && fail == 0) fail = j + 1;
        piv = sqrt(d);
        G[j * n + j] = piv;
      }
      __syncthreads();
      const double inv = 1.0 / piv;
      for (int i = j + 1 + t; i < n; i += kCholThreads) G[i * n + j] *= inv;
      __syncthreads();
      const int m = n - j - 1;
      for (int64_t e = t; e < (int64_t)m * m; e += kCholThreads) {
        const int i = j + 1 + (int)(e / m), k = j + 1 + (int)(e % m);
        if (k <= i) G[i * n + k] = fma(-G[i * n + j], G[k * n + j], G[i * n + k]);
      }
      __syncthreads();
    }
  }
  if (t == 0 && info != nullptr) info[b] = fail;
}

}  // namespace mi

extern "C" {

int mi_cholesky(const void* A, int32_t a_bytes, int64_t batch, int64_t n, void* L,
                int32_t l_bytes, int32_t* info, void* stream) {
  if (batch < 0 || n < 1 || n > MI_MVN_MAX_N || batch > 0x7fffffff ||
      (a_bytes != 4 && a_bytes != 8) || (l_bytes != 4 && l_bytes != 8))
    return MI_EINVAL;
  if (batch == 0) return 0;
  if (A == nullptr || L == nullptr) return MI_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)batch), block(mi::kCholThreads);
  if (n <= mi::kMvnLdsMaxN) {
    const size_t bytes = sizeof(double) * (size_t)n * (size_t)(n + 1);
    if (a_bytes == 8 && l_bytes == 8)
      hipLaunchKernelGGL((mi::k_cholesky<double, double, true>), grid, block, bytes, s,
                         static_cast<const double*>(A), (int)n, static_cast<double*>(L), info);
    else if (a_bytes == 4 && l_bytes == 4)
      hipLaunchKernelGGL((mi::k_cholesky<float, float, true>), grid, block, bytes, s,
                         static_cast<const float*>(A), (int)n, static_cast<float*>(L), info);
    else if (a_bytes == 4)
      hipLaunchKernelGGL((mi::k_cholesky<float, double, true>), grid, block, bytes, s,
                         static_cast<const float*>(A), (int)n, static_cast<double*>(L), info);
    else
      hipLaunchKernelGGL((mi::k_cholesky<double, float, true>), grid, block, bytes, s,
                         static_cast<const double*>(A), (int)n, static_cast<float*>(L), info);
  } else {
    if (l_bytes != 8) return MI_EUNSUPPORTED;   // larger factors work in the float64 output
    if (a_bytes == 8)
      hipLaunchKernelGGL((mi::k_cholesky<double, double, false>), grid, block, 0, s,
                         static_cast<const double*>(A), (int)n, static_cast<double*>(L), info);
    else
      hipLaunchKernelGGL((mi::k_cholesky<float, double, false>), grid, block, 0, s,
                         static_cast<const float*>(A), (int)n, static_cast<double*>(L), info);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

int mi_mvn_tril_forward(const double* value, const double* loc, const double* scale_tril,
                        int64_t batch, int64_t n, double* log_prob, double* w, double* u,
                        void* stream) {
  if (batch < 0 || n < 1 || n > MI_MVN_MAX_N || batch > 0x7fffffff)
    return MI_EINVAL;
  if (batch == 0) return 0;
  if (value == nullptr || loc == nullptr || scale_tril == nullptr || log_prob == nullptr ||
      w == nullptr || u == nullptr)
    return MI_EINVAL;
  if (n <= mi::kMvnLdsMaxN) {   // the factor staged in LDS; longer ones read from global memory
    const size_t bytes = sizeof(double) * (size_t)n * (size_t)(n + 1);
    hipLaunchKernelGGL(mi::k_mvn_tril<true>, dim3((unsigned)batch), dim3(mi::kMvnThreads), bytes,
                       static_cast<hipStream_t>(stream), value, loc, scale_tril, (int)n,
                       log_prob, w, u);
  } else {
    hipLaunchKernelGGL(mi::k_mvn_tril<false>, dim3((unsigned)batch), dim3(mi::kMvnThreads), 0,
                       static_cast<hipStream_t>(stream), value, loc, scale_tril, (int)n,
                       log_prob, w, u);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // extern "C"
