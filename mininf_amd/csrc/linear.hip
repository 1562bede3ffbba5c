// Linear-predictor sites: Normal(X @ theta, sigma) and Bernoulli(logits = X @ theta) with the
// product evaluated inside the site kernel.
//
// In the reference's regression models (tests/test_mininf.py:13-18, examples/minibatch.md:24-33)
// the model computes `X @ theta` and hands the result to a Normal site; traced over K particles
// that is a [N, K] predictor written by a GEMM, read by the site kernel, its [N, K] gradient written
// back and reduced by a second GEMM (~4 x 4 B x K x N of HBM traffic, 2.4 ms per C3 step). Here the
// particle tracer defers the product (mininf_amd/linear.py) and this kernel evaluates, per
// (particle k, row i),
//   loc = <X_i, theta_k>,   log p(y_i | loc, sigma_k),   dtheta_k += w * dlogp/dloc * X_i
// so HBM traffic is X and y once (C3: 132 MB) and the work is 2 P FMAs per evaluation.
//
// Layout: lanes along particles (kb = min(256, pow2(K)) per block, 256 / kb row groups), rows of X
// staged through LDS in chunks of 64 and read as wave-wide broadcasts; theta_k and the gradient
// accumulators live in registers. Per-(tile, particle) partials are reduced in fp64 by k_finalize.
#include "common.hpp"
#include "internal.hpp"

#include <algorithm>

namespace mi {

constexpr int kLinThreads = 256;
constexpr int kLinChunk = 64;

template <int FAMILY, int PMAX>
__global__ __launch_bounds__(kLinThreads) void k_linear(const mi_linear L, int kb,
                                                        int64_t rows_per_tile, int64_t ntile,
                                                        float* __restrict__ part,
                                                        uint32_t* __restrict__ flags) {
  __shared__ __attribute__((aligned(16))) float xs[kLinChunk][PMAX];
  __shared__ float ys[kLinChunk];
  __shared__ float ms[kLinChunk];
  __shared__ float red[kLinThreads];
  const int tid = threadIdx.x;
  const int kk = tid & (kb - 1);
  const int g = tid / kb;
  const int G = kLinThreads / kb;
  const int64_t K = L.K, N = L.N;
  const int P = (int)L.P;
  const int64_t k = (int64_t)blockIdx.y * kb + kk;
  const bool kok = k < K;
  const int64_t kc = kok ? k : K - 1;
  const bool per_particle_sigma = FAMILY == MI_NORMAL && L.scale != nullptr;

  float th[PMAX], acc[PMAX];
#pragma unroll
  for (int j = 0; j < PMAX; ++j) {
    th[j] = j < P ? L.theta[kc * L.theta_stride_k + j * L.theta_stride_j] : 0.0f;
    acc[j] = 0.0f;
  }
  uint32_t fl = 0u;
  float inv = 1.0f, cst = 0.0f;
  if (FAMILY == MI_NORMAL) {
    // -(y - loc)^2 / (2 sigma^2) - log(sigma) - log(sqrt(2 pi))   (normal.py:88-103)
    const float sigma = per_particle_sigma ? L.scale[kc * L.scale_stride_k] : L.scale_constant;
    inv = 1.0f / sigma;
    cst = -logf(sigma) - kHalfLog2Pi;
    fl |= (kok && !(sigma > 0.0f)) ? MI_FLAG_PARAM : 0u;
  }
  const float wscale = (float)L.site_scale;
  float lp = 0.0f, ds = 0.0f;

  const int64_t r0 = (int64_t)blockIdx.x * rows_per_tile;
  const int64_t r1 = min(N, r0 + rows_per_tile);
  for (int64_t c0 = r0; c0 < r1; c0 += kLinChunk) {
    const int rows = (int)min((int64_t)kLinChunk, r1 - c0);
    __syncthreads();
    for (int e = tid; e < kLinChunk * PMAX; e += kLinThreads) {
      const int r = e / PMAX, j = e % PMAX;
      xs[r][j] = (r < rows && j < P) ? L.x[(c0 + r) * L.x_stride_i + j * L.x_stride_j] : 0.0f;
    }
    for (int r = tid; r < kLinChunk; r += kLinThreads) {
      float y = 0.0f, m = 0.0f;
      if (r < rows) {
        const int64_t i = c0 + r;
        y = L.value[i * L.value_stride_i];
        m = (L.mask == nullptr || L.mask[i * L.mask_stride_i] != 0) ? 1.0f : 0.0f;
        const bool bad = FAMILY == MI_NORMAL ? (y != y) : !(y == 0.0f || y == 1.0f);
        fl |= (m != 0.0f && bad) ? MI_FLAG_SUPPORT : 0u;
      }
      ys[r] = y;
      ms[r] = m;
    }
    __syncthreads();
    // Rows of the chunk: the whole X row is fetched with 16-byte LDS reads (wave-wide broadcasts)
    // into one of two register sets while the other is used; the dot product runs in four
    // independent partial sums.
    const float4* xq = reinterpret_cast<const float4*>(&xs[0][0]);
    constexpr int Q = PMAX / 4;
    auto row = [&](const float4 (&x)[Q], int r) {
      const float y = ys[r], m = ms[r];
      float l0 = 0.0f, l1 = 0.0f, l2 = 0.0f, l3 = 0.0f;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        l0 = fmaf(th[4 * q + 0], x[q].x, l0);
        l1 = fmaf(th[4 * q + 1], x[q].y, l1);
        l2 = fmaf(th[4 * q + 2], x[q].z, l2);
        l3 = fmaf(th[4 * q + 3], x[q].w, l3);
      }
      const float loc = (l0 + l1) + (l2 + l3);
      float gl;
      if (FAMILY == MI_NORMAL) {
        const float z = (y - loc) * inv;
        lp = fmaf(m, fmaf(-0.5f * z, z, cst), lp);
        gl = z * inv;
        if (per_particle_sigma) ds = fmaf(m * wscale, (z * z - 1.0f) * inv, ds);
        fl |= (loc != loc) ? MI_FLAG_PARAM : 0u;
      } else {
        Elem el;
        eval_bernoulli_logits(loc, y, el);
        lp = fmaf(m, el.lp, lp);
        gl = el.d[0];
        fl |= el.param_bad ? MI_FLAG_PARAM : 0u;
      }
      const float w = m * wscale * gl;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        acc[4 * q + 0] = fmaf(w, x[q].x, acc[4 * q + 0]);
        acc[4 * q + 1] = fmaf(w, x[q].y, acc[4 * q + 1]);
        acc[4 * q + 2] = fmaf(w, x[q].z, acc[4 * q + 2]);
        acc[4 * q + 3] = fmaf(w, x[q].w, acc[4 * q + 3]);
      }
    };
    float4 xa[Q], xb[Q];
    if (g < rows) {
#pragma unroll
      for (int q = 0; q < Q; ++q) xa[q] = xq[g * Q + q];
    }
    for (int r = g; r < rows; r += 2 * G) {
      const bool second = r + G < rows;
      if (second) {
#pragma unroll
        for (int q = 0; q < Q; ++q) xb[q] = xq[(r + G) * Q + q];
      }
      row(xa, r);
      if (!second) break;
      if (r + 2 * G < rows) {
#pragma unroll
        for (int q = 0; q < Q; ++q) xa[q] = xq[(r + 2 * G) * Q + q];
      }
      row(xb, r + G);
    }
  }

  // Sum the row groups' shares of each value in a fixed order and write the tile's partials:
  // v = 0 log p, 1..P dtheta_j, P + 1 dsigma.
  const int nv = 1 + P + (per_particle_sigma ? 1 : 0);
  const int64_t tile = blockIdx.x;
#pragma unroll
  for (int v = 0; v < PMAX + 2; ++v) {
    if (v < nv) {
      const float val = v == 0 ? lp : (v <= PMAX && v - 1 < P ? acc[v - 1 < PMAX ? v - 1 : 0] : ds);
      __syncthreads();
      red[tid] = val;
      __syncthreads();
      if (g == 0 && kok) {
        float s = 0.0f;
        for (int q = 0; q < G; ++q) s += red[q * kb + kk];
        part[((int64_t)v * ntile + tile) * K + k] = s;
      }
    }
  }
  publish_flags(flags, fl);
}

}  // namespace mi

namespace {

int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

bool valid(const mi_linear* L) {
  return L != nullptr && L->K >= 1 && L->N >= 1 && L->P >= 1 && L->P <= MI_LINEAR_MAX_P &&
         (L->family == MI_NORMAL || L->family == MI_BERNOULLI_LOGITS) && L->x != nullptr &&
         L->theta != nullptr && L->value != nullptr;
}

struct Geometry {
  int kb;
  int64_t gy, rows_per_tile, ntile;
  int nv;
};

Geometry geometry(const mi_linear* L) {
  Geometry g{};
  int kb = 1;
  while (kb < 256 && kb < L->K) kb <<= 1;
  g.kb = kb;
  g.gy = ceil_div(L->K, kb);
  // about 768 blocks in total (3 per CU), whole LDS chunks per tile
  const int64_t tiles = std::max<int64_t>(1, 768 / g.gy);
  g.rows_per_tile = std::max<int64_t>(mi::kLinChunk, ceil_div(ceil_div(L->N, tiles), mi::kLinChunk) * mi::kLinChunk);
  g.ntile = ceil_div(L->N, g.rows_per_tile);
  g.nv = 1 + (int)L->P + ((L->family == MI_NORMAL && L->scale != nullptr) ? 1 : 0);
  return g;
}

int to_code(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

// per-(tile, particle) partials, 256-byte aligned so the finalize scratch behind them is too
size_t partial_bytes(const mi_linear* site, const Geometry& g) {
  return ((size_t)g.nv * (size_t)g.ntile * (size_t)site->K * sizeof(float) + 255) / 256 * 256;
}

template <int FAMILY>
void launch(const mi_linear& L, const Geometry& g, float* part, uint32_t* flags, hipStream_t s) {
  const dim3 grid((unsigned)g.ntile, (unsigned)g.gy);
  if (L.P <= 8)
    hipLaunchKernelGGL((mi::k_linear<FAMILY, 8>), grid, dim3(mi::kLinThreads), 0, s, L, g.kb,
                       g.rows_per_tile, g.ntile, part, flags);
  else if (L.P <= 16)
    hipLaunchKernelGGL((mi::k_linear<FAMILY, 16>), grid, dim3(mi::kLinThreads), 0, s, L, g.kb,
                       g.rows_per_tile, g.ntile, part, flags);
  else if (L.P <= 32)
    hipLaunchKernelGGL((mi::k_linear<FAMILY, 32>), grid, dim3(mi::kLinThreads), 0, s, L, g.kb,
                       g.rows_per_tile, g.ntile, part, flags);
  else
    hipLaunchKernelGGL((mi::k_linear<FAMILY, 64>), grid, dim3(mi::kLinThreads), 0, s, L, g.kb,
                       g.rows_per_tile, g.ntile, part, flags);
}

}  // namespace

extern "C" {

int mi_linear_struct_size(size_t* bytes) {
  if (bytes == nullptr) return MI_EINVAL;
  *bytes = sizeof(mi_linear);
  return 0;
}

int mi_linear_workspace_bytes(const mi_linear* site, size_t* bytes) {
  if (!valid(site) || bytes == nullptr) return MI_EINVAL;
  const Geometry g = geometry(site);
  *bytes = partial_bytes(site, g) + mi_finalize_scratch_bytes(g.ntile, site->K, g.nv);
  return 0;
}

int mi_linear_forward_timed(const mi_linear* site, void* workspace, size_t workspace_bytes,
                            float* total, float* dslots, uint32_t* flags, void* start_event,
                            void* stop_event, void* stream) {
  if (!valid(site) || total == nullptr || flags == nullptr ||
      (site->compute_grads && dslots == nullptr))
    return MI_EINVAL;
  size_t need = 0;
  mi_linear_workspace_bytes(site, &need);
  if (workspace == nullptr || workspace_bytes < need) return MI_EWORKSPACE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e;
  if (!(site->options & MI_GROUP_FLAGS_ZEROED)) {
    e = hipMemsetAsync(flags, 0, sizeof(uint32_t), s);
    if (e != hipSuccess) return to_code(e);
  }
  const Geometry g = geometry(site);
  float* part = static_cast<float*>(workspace);
  if (start_event != nullptr && (e = hipEventRecord(static_cast<hipEvent_t>(start_event), s)) != hipSuccess)
    return to_code(e);
  if (site->family == MI_NORMAL)
    launch<MI_NORMAL>(*site, g, part, flags, s);
  else
    launch<MI_BERNOULLI_LOGITS>(*site, g, part, flags, s);
  e = hipGetLastError();
  if (e != hipSuccess) return to_code(e);
  if (stop_event != nullptr && (e = hipEventRecord(static_cast<hipEvent_t>(stop_event), s)) != hipSuccess)
    return to_code(e);
  const double scale = site->site_scale;
  double* scratch = reinterpret_cast<double*>(static_cast<char*>(workspace) + partial_bytes(site, g));
  return mi_launch_finalize(part, g.ntile, site->K, 1, site->compute_grads ? g.nv - 1 : 0, &scale,
                            (double)site->grad_scale, total, nullptr, dslots, scratch, s);
}

int mi_linear_forward(const mi_linear* site, void* workspace, size_t workspace_bytes, float* total,
                      float* dslots, uint32_t* flags, void* stream) {
  return mi_linear_forward_timed(site, workspace, workspace_bytes, total, dslots, flags, nullptr,
                                 nullptr, stream);
}

}  // extern "C"
