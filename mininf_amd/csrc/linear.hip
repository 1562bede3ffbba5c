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
#include "adam_math.hpp"
#include "common.hpp"
#include "internal.hpp"
#include "rows.hpp"

#include <algorithm>
#include <cstdlib>

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
      const int64_t src = (r < rows && L.row_index != nullptr) ? L.row_index[c0 + r] : c0 + r;
      xs[r][j] = (r < rows && j < P) ? L.x[src * L.x_stride_i + j * L.x_stride_j] : 0.0f;
    }
    for (int r = tid; r < kLinChunk; r += kLinThreads) {
      float y = 0.0f, m = 0.0f;
      if (r < rows) {
        const int64_t i = L.row_index != nullptr ? L.row_index[c0 + r] : c0 + r;
        y = L.value[i * L.value_stride_i];
        m = (L.mask == nullptr || L.mask[i * L.mask_stride_i] != 0) ? 1.0f : 0.0f;
        const bool bad = FAMILY == MI_NORMAL ? (y != y) : !(y == 0.0f || y == 1.0f);
        fl |= (m != 0.0f && bad) ? MI_FLAG_SUPPORT : 0u;
      }
      ys[r] = m != 0.0f ? y : 0.0f;   // masked-out values (NaN in missing data) are never used
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

// ---- matrix-core formulation -------------------------------------------------------------------
// The site is two contractions around an elementwise step, per 32-row tile of X and 32 particles:
//   MU[i, k]     = sum_p X[i, p] theta[k, p]                 (v_mfma_f32_32x32x2_f32, A = X, B = theta^T)
//   R[i, k]      = mask_i * dlogp/dloc(y_i, MU[i, k])        (VALU, in the accumulator registers)
//   DTH[k, p]   += sum_i R[i, k] X[i, p]                     (v_mfma_f32_32x32x2_f32, A = R^T, B = X)
// The 32x32 accumulator of the first product holds particle k = lane & 31 and row
// (r & 3) + 8 (r >> 2) + 4 (lane >> 5) in register r, which is exactly the A operand of the second
// product's k-step r (A[m = lane & 31][kd = lane >> 5]), so R never leaves the registers; its B
// operand is the matching X row, read from LDS. f32-in MFMA is an exact fmaf chain, so the numerics
// are those of the VALU kernel's dot products, at the matrix-core rate (MI355X_MICROARCH.md: 157 TF).
//
// Block: 8 waves = WT particle tiles of 32 x RS row subsets (WT * RS = 8). X is staged through one
// LDS buffer in stages of CH rows (prefetched into registers during the previous stage's MFMAs) as
// [row][feature parity][feature / 2], so the first product's A fragment (lane: row lane & 31,
// features 2s + (lane >> 5)) is a contiguous 16-byte-read run. Partials: one tile per (block, row
// subset), reduced in fp64 by k_finalize as for the VALU kernel.
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Phase timestamps (MI_LINEAR_TIMING builds only, tools/linear_timing.py): wall clock at 8 points of
// every wave of k_linear_mfma, into a buffer behind the launch's workspace.
#ifndef MI_LINEAR_TIMING
#define MI_LINEAR_TIMING 0
#endif
#if MI_LINEAR_TIMING
__device__ unsigned long long* mi_lin_tbuf;
#define MI_LIN_STAMP(i) do { if ((threadIdx.x & 63) == 0) ts_[i] = wall_clock64(); } while (0)
#else
#define MI_LIN_STAMP(i) do { } while (0)
#endif

template <int PT, int NT>
struct MfShape {
  static constexpr int NW = NT / kWave;    // waves per block
  static constexpr int PM = 32 * PT;       // padded features
  static constexpr int HS = 16 * PT;       // floats per feature-parity half of an LDS row
  static constexpr int RSTR = PM + 4;      // LDS row stride (floats): 16-byte aligned, skewed banks
  static constexpr int CH = (NT >= 512 ? 256 : 128) / PT;   // rows per stage
  static constexpr int TILES = CH / 32;    // 32-row tiles per stage
  static constexpr int QPT = CH * PM / 4 / NT;   // float4 loads per thread per stage
};

// theta drawn by the launch (mi_linear.draw): the block's particles [kbase, kbase + nk) into LDS rows
// dst[(k - kbase) * dstr + j], one work item per (particle, feature quad) -- the normals of
// k_normal_rsample for the same (particle, element quad) and the same fmaf, so the values are
// bit-identical to the separate draw. The first row block also writes them to theta (every
// particle group its own particles) and, for an exp-transformed scale, group 0 writes the scale.
// Two phases: the items' parameters and the generator step are loaded before the stage's X rows
// (a wait for them then does not wait for the X loads, vector-memory counts being in order), the
// normals are computed while the X loads are in flight.
constexpr int kDrawItems = 4;   // items per thread: nk * P / 4 <= 4 * threads (host-checked)
struct DrawRegs {
  float loc[kDrawItems][4], sd[kDrawItems][4];
  uint64_t step;
};
template <int NT>
__device__ __forceinline__ void draw_theta_load(const mi_linear& L, int nk, DrawRegs& R) {
  const mi_draw& D = L.draw;
  R.step = D.step + (D.step_device != nullptr ? *D.step_device : 0ull);
  const int nq = (int)L.P / 4;
  const bool exp_scale = D.scale_exp != nullptr;
  const float* sp = exp_scale ? D.scale_exp : D.scale;
#pragma unroll
  for (int t = 0; t < kDrawItems; ++t) {
    const int item = (int)threadIdx.x + t * NT;
    const int ic = item < nk * nq ? item : 0;   // clamped: every load from a valid address
    const int q = ic % nq;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t i = 4 * q + j;
      R.loc[t][j] = D.loc[i * D.loc_stride];
      R.sd[t][j] = sp[i * D.scale_stride];
    }
  }
}
template <int NT>
__device__ __forceinline__ void draw_theta(const mi_linear& L, int64_t kbase, int nk, float* dst,
                                           int dstr, bool write_theta, bool write_scale,
                                           const DrawRegs& R) {
  const mi_draw& D = L.draw;
  const int nq = (int)L.P / 4;
  const bool exp_scale = D.scale_exp != nullptr;
#pragma unroll
  for (int t = 0; t < kDrawItems; ++t) {
    const int item = (int)threadIdx.x + t * NT;
    if (item >= nk * nq) break;
    const int kl = item / nq, q = item - kl * nq;
    const int64_t kk = kbase + kl;
    float e[4];
    guide_normals(D.seed, R.step, D.stream_id, (uint64_t)(D.element_offset / 4 + q),
                  (uint64_t)(D.particle_offset + kk), e);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t i = 4 * q + j;
      const float sd = exp_scale ? expf(R.sd[t][j]) : R.sd[t][j];
      const float z = fmaf(e[j], sd, R.loc[t][j]);
      dst[kl * dstr + i] = z;
      if (write_theta) const_cast<float*>(L.theta)[kk * L.theta_stride_k + i * L.theta_stride_j] = z;
      if (write_scale && exp_scale && kl == 0) const_cast<float*>(D.scale)[i * D.scale_stride] = sd;
    }
  }
}

// Grid: one dimension of gx * gy blocks, gx (row blocks) a multiple of 8. Blocks are dealt to the
// 8 XCDs round-robin, so block b's row block is chosen such that the gy particle groups of one row
// block run on one XCD (b, b + 8, ...) and share its L2 copy of the X rows.
// ONESTAGE: every block stages one row block (small N, e.g. a 65536-row minibatch): no stage
// loop, no prefetch and no software pipeline over tiles -- a third of the code, which matters
// when each wave runs through it once (the cold instruction fetch dominates such launches).
template <int FAMILY, int PT, int NT, bool FLUSH64, int MINW, bool GRADS, bool ONESTAGE>
__global__ __launch_bounds__(NT, MINW) void k_linear_mfma(const mi_linear L, int wt, int gy,
                                                          int64_t stages_per_block,
                                                          int64_t ntile,
                                                          float* __restrict__ part,
                                                          uint32_t* __restrict__ flags,
                                                          int rows_half) {
  using S = MfShape<PT, NT>;
  constexpr int kMfThreads = NT;
  constexpr int kMfWaves = S::NW;
#if MI_LINEAR_TIMING
  unsigned long long ts_[8] = {};
#endif
  MI_LIN_STAMP(0);
  // one-stage launches (C4's minibatch) run each wave through a short body once: the argument
  // chain at their start is on the critical path (C4 37.5 -> 36.5 us per step); the multi-stage
  // launches (C3) lose more to the prefetch's wait in wave 0 than they gain (300.5 -> 308 us)
  if (ONESTAGE) kernarg_prefetch<(int)sizeof(mi_linear)>();
  const unsigned long long span_t0 = span_begin(L.stamps);
  const int64_t bid = blockIdx.x;
  const int64_t row_block = (bid / (8 * gy)) * 8 + bid % 8;
  const int64_t group = (bid / 8) % gy;
  __shared__ __attribute__((aligned(16))) float xs[S::CH * S::RSTR];
  __shared__ float2 yms[S::CH];
  // rows drawn here (mi_linear.rows, ONESTAGE launches only): the stage's dataset rows
  __shared__ int32_t grows[ONESTAGE ? S::CH : 1];
  const bool gen_rows = ONESTAGE && L.rows.counter != nullptr;
  uint64_t batch_no = 0;

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1), wave = tid / kWave;
  const int h = lane >> 5, c = lane & 31;
  const int rs_count = kMfWaves / wt;
  const int pt = wave % wt, rs = wave / wt;
  const int64_t K = L.K, N = L.N;
  const int P = (int)L.P;
  const int64_t k0 = (group * wt + pt) * 32;
  constexpr bool grads = GRADS;
  const bool per_particle_sigma = FAMILY == MI_NORMAL && L.scale != nullptr;
  uint32_t fl = 0u;

  // B fragment of the first product: theta[k0 + c][2 s + h]. Branch-free: every load from a
  // clamped (valid) address, zeroed after -- guarded loads compile to one branch and one exec mask
  // per load, and a one-stage launch is a single pass through this code.
  float thf[S::HS];
  // theta drawn here (mi_linear.draw): into the X staging buffer after the first stage's loads are
  // issued, then into thf (draw_here below)
  const bool drawn = L.draw.operand != 0;
  if (!drawn) {
    const int64_t kk = k0 + c;
    const int64_t kc = kk < K ? kk : K - 1;
#pragma unroll
    for (int s = 0; s < S::HS; ++s) {
      const int p = 2 * s + h;
      const float v = L.theta[kc * L.theta_stride_k + (int64_t)(p < P ? p : P - 1) * L.theta_stride_j];
      thf[s] = keep_if(v, kk < K && p < P);
    }
  }

  // dtheta: fp32 MFMA accumulators per stage, carried in fp64 across stages (PT = 1); with two
  // feature tiles the fp64 copy would not fit the 256 registers of a 2-wave/SIMD launch, so the
  // accumulators run in fp32 over the block's rows, as in the VALU kernel.
  constexpr bool kFlush64 = FLUSH64;
  double dth[kFlush64 ? PT : 1][kFlush64 ? 16 : 1];
#pragma unroll
  for (int t = 0; t < (kFlush64 ? PT : 1); ++t)
#pragma unroll
    for (int r = 0; r < (kFlush64 ? 16 : 1); ++r) dth[t][r] = 0.0;
  f32x16 acc2[PT];
#pragma unroll
  for (int t = 0; t < PT; ++t) acc2[t] = f32x16{};
  double lpd = 0.0;      // Normal: sum of mask * (y - loc)^2; Bernoulli: sum of mask * log p
  float cnt = 0.0f;      // observed rows seen by this lane (Normal)

  const int64_t nstage = (N + S::CH - 1) / S::CH;
  const int64_t st0 = row_block * stages_per_block;
  const int64_t st1 = min(nstage, st0 + stages_per_block);

  // ---- staging: X quads and (y, mask) of one stage into registers, then into LDS ---------------
  float4 xq[S::QPT];
  float yraw = 0.0f;          // the stage's (y, mask) of row tid, as loaded
  uint32_t mraw = 1u;
  int64_t staged_row0 = 0;    // the stage whose loads xq / yraw / mraw hold
  // Source rows first (one uniform branch on how rows are given), then every X quad and the
  // (y, mask) of the stage issued together with no wait in between: a guarded load per quad
  // compiled to a branch and a wait per load, one memory round trip each.
  auto load_stage = [&](int64_t st) {
    const int64_t row0 = st * S::CH;
    int64_t src[S::QPT + 1];   // [QPT]: the (y, mask) row of lane tid < CH
    int64_t rows[S::QPT + 1];
#pragma unroll
    for (int q = 0; q < S::QPT; ++q) rows[q] = row0 + (tid + q * kMfThreads) / (S::PM / 4);
    rows[S::QPT] = row0 + (tid < S::CH ? tid : 0);
#pragma unroll
    for (int q = 0; q <= S::QPT; ++q) rows[q] = rows[q] < N ? rows[q] : N - 1;
    if (gen_rows) {
#pragma unroll
      for (int q = 0; q <= S::QPT; ++q) src[q] = (int64_t)grows[ONESTAGE ? (int)(rows[q] - row0) : 0];
    } else if (L.row_index != nullptr) {
#pragma unroll
      for (int q = 0; q <= S::QPT; ++q) src[q] = (int64_t)L.row_index[rows[q]];
    } else {
#pragma unroll
      for (int q = 0; q <= S::QPT; ++q) src[q] = rows[q];
    }
#pragma unroll
    for (int q = 0; q < S::QPT; ++q) {
      const int e = tid + q * kMfThreads;
      const int row = e / (S::PM / 4), c4 = e % (S::PM / 4);
      (void)row;
      xq[q] = *reinterpret_cast<const float4*>(L.x + src[q] * L.x_stride_i +
                                               4 * (4 * c4 < P ? c4 : 0));
    }
    yraw = L.value[src[S::QPT] * L.value_stride_i];
    mraw = L.mask == nullptr ? 1u : (uint32_t)L.mask[src[S::QPT] * L.mask_stride_i];
    staged_row0 = row0;
  };
  // The loads' values are first used here (rows past N and features past P zeroed, the (y, mask)
  // checks), so nothing waits for a stage's loads before store time: in one-stage launches the
  // theta draw runs while the row gathers are in flight (r06: zeroing them in load_stage made the
  // draw wait for them; C4 32.6 vs 33.9 us per step, profiles/r06_ab.json ab24/ab25).
  auto store_stage = [&]() {
    const int64_t row0 = staged_row0;
#pragma unroll
    for (int q = 0; q < S::QPT; ++q) {
      const int e = tid + q * kMfThreads;
      const int row = e / (S::PM / 4), c4 = e % (S::PM / 4);
      const bool in = row0 + row < N && 4 * c4 < P;
      const float4 v = xq[q];
      float* dst = xs + row * S::RSTR + 2 * c4;
      *reinterpret_cast<float2*>(dst) = make_float2(keep_if(v.x, in), keep_if(v.z, in));           // even features
      *reinterpret_cast<float2*>(dst + S::HS) = make_float2(keep_if(v.y, in), keep_if(v.w, in));   // odd features
    }
    if (tid < S::CH) {
      const int64_t row = row0 + tid;
      float y = 0.0f, m = 0.0f;
      if (row < N) {
        y = yraw;
        m = mraw != 0u ? 1.0f : 0.0f;
        const bool bad = FAMILY == MI_NORMAL ? (y != y) : !(y == 0.0f || y == 1.0f);
        fl |= (m != 0.0f && bad) ? MI_FLAG_SUPPORT : 0u;
      }
      yms[tid] = make_float2(m != 0.0f ? y : 0.0f, m);
    }
  };

  // The block's particles' draws through the (still unused) X staging buffer into thf: called by
  // every thread after the first stage's loads are issued and before they are stored.
  constexpr int kDrawStride = S::PM + 1;   // odd row stride: lanes c read distinct banks
  const int64_t draw_kbase = group * wt * 32;
  const int draw_nk = (int)min((int64_t)wt * 32, K - draw_kbase);
  DrawRegs dregs;
  auto draw_here = [&]() {
    const int64_t kbase = draw_kbase;
    const int nk = draw_nk;
    draw_theta<kMfThreads>(L, kbase, nk, xs, kDrawStride, row_block == 0, row_block == 0 && group == 0,
                           dregs);
    __syncthreads();
    const int kl = pt * 32 + c;
    const int klc = kl < nk ? kl : nk - 1;
#pragma unroll
    for (int s = 0; s < S::HS; ++s) {
      const int p = 2 * s + h;
      thf[s] = keep_if(xs[klc * kDrawStride + (p < P ? p : P - 1)], kl < nk && p < P);
    }
    __syncthreads();
  };

  // MU = X theta^T for the tile's 32 rows and this wave's 32 particles
  auto gemm1 = [&](int tile) -> f32x16 {
    f32x16 mu = f32x16{};
    const float* xa = xs + (tile * 32 + c) * S::RSTR + h * S::HS;
#pragma unroll
    for (int s = 0; s < S::HS; s += 4) {
      const float4 a = *reinterpret_cast<const float4*>(xa + s);
      mu = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, thf[s + 0], mu, 0, 0, 0);
      mu = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, thf[s + 1], mu, 0, 0, 0);
      mu = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, thf[s + 2], mu, 0, 0, 0);
      mu = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, thf[s + 3], mu, 0, 0, 0);
    }
    return mu;
  };
  // log density and mask * d/dloc in place (Normal: d = y - loc, the 1/sigma^2 factor is applied
  // per particle at the end)
  auto elementwise = [&](f32x16& mu, int tile) {
    float lpt = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = tile * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const float2 ym = yms[row];
      const float loc = mu[r];
      fl |= (loc != loc) ? MI_FLAG_PARAM : 0u;
      if (FAMILY == MI_NORMAL) {
        const float d = ym.y * (ym.x - loc);
        lpt = fmaf(d, d, lpt);
        cnt += ym.y;
        mu[r] = d;
      } else {
        Elem el;
        eval_bernoulli_logits(loc, ym.x, el);
        lpt = fmaf(ym.y, el.lp, lpt);
        mu[r] = ym.y * el.d[0];
      }
    }
    lpd += (double)lpt;
  };
  // DTH[k, p] += sum_rows R[row, k] X[row, p]: k-step r pairs register r with its row
  auto gemm2 = [&](const f32x16& R, int tile) {
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      const int p = 32 * t + c;
      const float* xb = xs + (p & 1) * S::HS + (p >> 1);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = tile * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        acc2[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(R[r], xb[row * S::RSTR], acc2[t], 0, 0, 0);
      }
    }
  };

  if constexpr (ONESTAGE) {
    if (gen_rows) {
      // this batch's rows of the block's stage, from the batch number every block reads before
      // the last one to finish advances it (below). (Issuing the draw's parameter loads before
      // or right after this read measured no faster: tools/linear_timing.py, round 4.)
      // (Rows computed one batch ahead by the previous launch and read here with the counter were
      // measured slower, round 6: C4 34.7-35.5 against 33.8-34.8 us per step -- the next batch's
      // permutation then delays the theta draw that overlaps the gathers; profiles/r06_ab.json.)
      batch_no = __hip_atomic_load(L.rows.counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tid < S::CH && st0 < st1) {
        const int64_t row = st0 * S::CH + tid;
        int32_t r = 0;
        if (row < N) {
          const BatchOrder order = batch_order(batch_no, L.rows.batches, L.rows.seed);
          r = batch_row(order, row, L.rows.n, L.rows.batch, L.rows.shuffle, rows_half);
          if (L.rows.out != nullptr && group == 0) L.rows.out[row] = r;
        }
        grows[tid] = r;
      }
      __syncthreads();
    }
    MI_LIN_STAMP(1);
    if (drawn) draw_theta_load<kMfThreads>(L, draw_nk, dregs);
    if (st0 < st1) load_stage(st0);
    if (drawn) draw_here();
    if (st0 < st1) store_stage();
    MI_LIN_STAMP(2);
    __syncthreads();
    MI_LIN_STAMP(3);
    if (st0 < st1) {
      const int ntl = (S::TILES - rs + rs_count - 1) / rs_count;
#pragma unroll 1
      for (int j = 0; j < ntl; ++j) {
        const int tile = rs + j * rs_count;
        f32x16 cur = gemm1(tile);
        elementwise(cur, tile);
        if (GRADS) gemm2(cur, tile);
      }
      if (kFlush64) {
#pragma unroll
        for (int t = 0; t < PT; ++t) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            dth[kFlush64 ? t : 0][kFlush64 ? r : 0] += (double)acc2[t][r];
          acc2[t] = f32x16{};
        }
      }
    }
    MI_LIN_STAMP(4);
    __syncthreads();
  }
  if (!ONESTAGE && drawn) draw_theta_load<kMfThreads>(L, draw_nk, dregs);
  if (!ONESTAGE && st0 < st1) load_stage(st0);
  if (!ONESTAGE && drawn) draw_here();
  if (!ONESTAGE && st0 < st1) store_stage();
  if (!ONESTAGE) __syncthreads();
  for (int64_t st = st0; !ONESTAGE && st < st1; ++st) {
    if (st + 1 < st1) load_stage(st + 1);   // in flight during this stage's MFMAs
    // Software pipeline over this wave's tiles: the first product of tile j + 1 is issued before
    // the elementwise step of tile j, so its MFMAs run while the VALU evaluates the densities.
    const int ntl = (S::TILES - rs + rs_count - 1) / rs_count;
    if (ntl > 0) {
      f32x16 cur = gemm1(rs);
      for (int j = 0; j + 1 < ntl; ++j) {
        const int tile = rs + j * rs_count;
        const f32x16 nxt = gemm1(tile + rs_count);
        elementwise(cur, tile);
        if (GRADS) gemm2(cur, tile);
        cur = nxt;
      }
      const int last = rs + (ntl - 1) * rs_count;
      elementwise(cur, last);
      if (GRADS) gemm2(cur, last);
    }
    if (kFlush64) {
#pragma unroll
      for (int t = 0; t < PT; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) dth[kFlush64 ? t : 0][kFlush64 ? r : 0] += (double)acc2[t][r];
        acc2[t] = f32x16{};
      }
    }
    // (two LDS buffers with one barrier per stage measured no faster, round 6: C3 313.6-316.1
    // against 311.9-314.0 us per step, profiles/r06_ab.json)
    __syncthreads();
    if (st + 1 < st1) {
      store_stage();
      __syncthreads();
    }
  }

  // ---- partials --------------------------------------------------------------------------------
  // val: [r * PT + t] dtheta (row r of the accumulator, feature tile t), then the log density and
  // dsigma of particle k0 + c (lanes h == 0). One tile per (block, row subset), or -- when the
  // block has several row subsets and their values fit the (now idle) X staging buffer -- the
  // subsets are combined through LDS in a fixed order and the block writes one tile (ntile = gx:
  // a smaller partial slab, short enough for mi_elbo_forward to reduce, mi_reduce).
  constexpr int kItems = 16 * PT + 2;
  float val[kItems];
  const float wscale = (float)L.site_scale;
  lpd += __shfl_xor(lpd, 32, kWave);
  cnt += __shfl_xor(cnt, 32, kWave);
  val[16 * PT] = val[16 * PT + 1] = 0.0f;
  if (h == 0 && k0 + c < K) {
    const int64_t kk = k0 + c;
    if (FAMILY == MI_NORMAL) {
      // -(y - loc)^2 / (2 sigma^2) - log(sigma) - log(sqrt(2 pi))   (normal.py:88-103)
      const float sigma = per_particle_sigma ? L.scale[kk * L.scale_stride_k] : L.scale_constant;
      fl |= !(sigma > 0.0f) ? MI_FLAG_PARAM : 0u;
      const double inv2 = 1.0 / ((double)sigma * (double)sigma);
      const double cst = -(double)logf(sigma) - (double)kHalfLog2Pi;
      val[16 * PT] = (float)(-0.5 * lpd * inv2 + (double)cnt * cst);
      if (per_particle_sigma)
        val[16 * PT + 1] = (float)((double)wscale * (lpd * inv2 - (double)cnt) / (double)sigma);
    } else {
      val[16 * PT] = (float)lpd;
    }
  }
  // a constant sigma: one division for all rows (sixteen fp64 divisions are a long serial tail of
  // a short launch)
  const double w_const = (FAMILY == MI_NORMAL && grads && !per_particle_sigma)
                             ? (double)wscale / ((double)L.scale_constant * (double)L.scale_constant)
                             : (double)wscale;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t kk = k0 + (r & 3) + 8 * (r >> 2) + 4 * h;
    double w = w_const;
    if (FAMILY == MI_NORMAL && grads && per_particle_sigma && kk < K) {
      const double sigma = (double)L.scale[kk * L.scale_stride_k];
      w = (double)wscale / (sigma * sigma);
    }
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      const double v = kFlush64 ? dth[kFlush64 ? t : 0][kFlush64 ? r : 0] : (double)acc2[t][r];
      val[r * PT + t] = grads ? (float)(v * w) : 0.0f;
    }
  }
  MI_LIN_STAMP(5);
  const bool combine = rs_count > 1 && (rs_count - 1) * wt * kWave * kItems <= S::CH * S::RSTR;
  int64_t tile_id = row_block * rs_count + rs;
  if (combine) {
    // (the stage loop ended with a barrier: xs is free)
    if (rs > 0) {
      float* dst = xs + (((rs - 1) * wt + pt) * kWave + lane) * kItems;
#pragma unroll
      for (int q = 0; q < kItems; ++q) dst[q] = val[q];
    }
    __syncthreads();
    if (rs == 0) {
#pragma unroll
      for (int q = 0; q < kItems; ++q) {
        double d = (double)val[q];
        for (int o = 1; o < rs_count; ++o) d += (double)xs[(((o - 1) * wt + pt) * kWave + lane) * kItems + q];
        val[q] = (float)d;
      }
    }
    tile_id = row_block;
  }
  MI_LIN_STAMP(6);
  if (!combine || rs == 0) {
    if (h == 0 && k0 + c < K) {
      part[tile_id * K + k0 + c] = val[16 * PT];
      if (per_particle_sigma && grads)
        part[((int64_t)(1 + P) * ntile + tile_id) * K + k0 + c] = val[16 * PT + 1];
    }
    if (grads) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t kk = k0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (kk >= K) continue;
#pragma unroll
        for (int t = 0; t < PT; ++t) {
          const int p = 32 * t + c;
          if (p < P) part[((int64_t)(1 + p) * ntile + tile_id) * K + kk] = val[r * PT + t];
        }
      }
    }
  }
  publish_flags(flags, fl);
  // The folded prior site over theta itself (mi_linear.prior): the first row block's first row
  // subset of every particle tile already holds theta[k0 + c][2 s + h] in thf -- no load -- and
  // writes the prior's value and d/dtheta as the slab's last tile.
  if (L.prior.present != 0 && row_block == 0 && rs == 0) {
    const int64_t kk = k0 + c;
    const int64_t ptile = ntile - 1;
    uint32_t pfl = 0u;
    float plp = 0.0f;
    if (!ONESTAGE) {
#pragma unroll
      for (int s = 0; s < S::HS; ++s) {
        const int p = 2 * s + h;
        if (kk < K && p < P) {
          Elem e;
          if (L.prior.family == MI_BETA) eval_beta(L.prior.constant[0], L.prior.constant[1], thf[s], e);
          else if (L.prior.family == MI_NORMAL) eval_normal(L.prior.constant[0], L.prior.constant[1], thf[s], e);
          else eval_gamma(L.prior.constant[0], L.prior.constant[1], thf[s], e);
          plp += e.lp;
          pfl |= (e.param_bad ? MI_FLAG_PARAM : 0u) | (e.support_bad ? MI_FLAG_SUPPORT : 0u);
          if (grads) part[((int64_t)(1 + p) * ntile + ptile) * K + kk] = (float)(L.prior.scale * (double)e.d[2]);
        }
      }
    } else {
      // One-stage launches choose the family once, outside the unrolled features: this code runs
      // in one wave of the launch, so its instructions are fetched cold, and the family test inside
      // the loop (above) lays the three families' code out per feature (r06, tools/linear_timing.py:
      // the 16 evaluations took 4.6 us in C4's launch, its last wave; 2.6 us hoisted). The
      // multi-stage kernel keeps the loop above (its code measured 2 us slower hoisted, C3
      // 313.8-314.2 vs 311.2-312.3 us per step, profiles/r06_ab.json ab17).
      auto features = [&](auto eval) {
#pragma unroll
        for (int s = 0; s < S::HS; ++s) {
          const int p = 2 * s + h;
          if (kk < K && p < P) {
            Elem e;
            eval(thf[s], e);
            plp += e.lp;
            pfl |= (e.param_bad ? MI_FLAG_PARAM : 0u) | (e.support_bad ? MI_FLAG_SUPPORT : 0u);
            if (grads) part[((int64_t)(1 + p) * ntile + ptile) * K + kk] = (float)(L.prior.scale * (double)e.d[2]);
          }
        }
      };
      const float pc0 = L.prior.constant[0], pc1 = L.prior.constant[1];
      if (L.prior.family == MI_NORMAL)
        features([&](float v, Elem& e) { eval_normal(pc0, pc1, v, e); });
      else if (L.prior.family == MI_BETA)
        features([&](float v, Elem& e) { eval_beta(pc0, pc1, v, e); });
      else
        features([&](float v, Elem& e) { eval_gamma(pc0, pc1, v, e); });
    }
    plp += __shfl_xor(plp, 32, kWave);   // the particle's two feature parities
    if (h == 0 && kk < K) {
      // the reduction scales the value row by the site's scale
      part[ptile * K + kk] = (float)((double)plp * L.prior.scale / L.site_scale);
      if (per_particle_sigma && grads) part[((int64_t)(1 + P) * ntile + ptile) * K + kk] = 0.0f;
    }
    publish_flags(L.prior.flags, pfl);
  }
  MI_LIN_STAMP(7);
#if MI_LINEAR_TIMING
  if ((threadIdx.x & 63) == 0) {
    unsigned long long* o = mi_lin_tbuf + ((int64_t)blockIdx.x * (NT / 64) + threadIdx.x / 64) * 8;
    for (int i = 0; i < 8; ++i) o[i] = ts_[i];
  }
#endif
  // the last block to finish advances the batch counter: every block has read it by then. (A
  // count taken right after the read instead made all blocks hit one address at once: measured
  // slower.)
  if (gen_rows && tid == 0) {
    const unsigned long long done = atomicAdd((unsigned long long*)&L.rows.counter[1], 1ull);
    if (done == (unsigned long long)gridDim.x - 1ull) {
      L.rows.counter[1] = 0;
      L.rows.counter[0] = batch_no + 1;
    }
  }
  span_end(L.stamps, span_t0);
}

}  // namespace mi

namespace {

int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

bool valid(const mi_linear* L) {
  if (L != nullptr && L->rows.counter != nullptr) {
    const mi_rows& R = L->rows;   // mi_minibatch_rows's conditions
    if (L->row_index != nullptr || R.n < 1 || R.n > INT32_MAX || R.batch < 1 || R.batches < 1 ||
        L->N > R.batch || (R.batches - 1) * R.batch >= R.n || R.batches * R.batch >= R.n + R.batch)
      return false;
  }
  if (L != nullptr && L->prior.present != 0 &&
      ((L->prior.family != MI_BETA && L->prior.family != MI_NORMAL && L->prior.family != MI_GAMMA) ||
       L->prior.flags == nullptr || !(L->site_scale != 0.0)))
    return false;
  return L != nullptr && L->K >= 1 && L->N >= 1 && L->P >= 1 && L->P <= MI_LINEAR_MAX_P &&
         (L->family == MI_NORMAL || L->family == MI_BERNOULLI_LOGITS) && L->x != nullptr &&
         L->theta != nullptr && L->value != nullptr;
}

struct Geometry {
  bool mfma;
  int kb;              // VALU kernel: particles per block
  int wt;              // MFMA kernel: 32-particle tiles per block
  int pt;              // MFMA kernel: 32-feature tiles (1 or 2)
  int variant;         // MFMA kernel: launch variant (kMfVariants)
  int64_t gx, gy, rows_per_tile, stages_per_block, ntile;
  int nv;
};

// The matrix-core kernel takes contiguous, 16-byte aligned rows of X (row stride a multiple of 4
// floats) with P % 4 == 0; anything else, or MI_LINEAR_VALU, runs the VALU kernel.
bool use_mfma(const mi_linear* L) {
  return !(L->options & MI_LINEAR_VALU) && L->P % 4 == 0 && L->x_stride_j == 1 &&
         L->x_stride_i >= L->P && L->x_stride_i % 4 == 0 &&
         (reinterpret_cast<uintptr_t>(L->x) & 15) == 0;
}

// Matrix-core launch variants: block size, fp64 carry of the dtheta accumulators across stages,
// minimum waves per SIMD (register budget). Measured on MI355X (tools/linear_bench.py, r02): one
// feature tile (P <= 32) runs 256 threads at 4 waves/SIMD with fp32 dtheta accumulators over the
// block's rows (C3 329 us vs 346 us for 512 threads with an fp64 carry), two tiles 256 threads at
// 2 waves/SIMD (350 us vs 370 us).
struct MfVariant {
  int threads;
  bool flush64;
  int minw;
};
constexpr MfVariant kMfVariants[] = {{256, false, 4}, {256, false, 2}};

int mf_variant(int pt) { return pt == 1 ? 0 : 1; }

Geometry geometry(const mi_linear* L) {
  Geometry g{};
  g.nv = 1 + (int)L->P + ((L->family == MI_NORMAL && L->scale != nullptr) ? 1 : 0);
  g.mfma = use_mfma(L);
  if (g.mfma) {
    g.pt = L->P <= 32 ? 1 : 2;
    g.variant = mf_variant(g.pt);
    const MfVariant v = kMfVariants[g.variant];
    const int waves = v.threads / 64;
    const int64_t ptiles = ceil_div(L->K, 32);
    int wt = 1;
    while (wt < waves && wt < ptiles) wt <<= 1;
    g.wt = wt;
    g.gy = ceil_div(ptiles, wt);
    const int64_t ch = (v.threads >= 512 ? 256 : 128) / g.pt;
    const int64_t nstage = ceil_div(L->N, ch);
    // about 512 (512-thread) or 1024 (256-thread) blocks over the grid, whole stages per block;
    // row blocks padded to a multiple of 8 (see k_linear_mfma)
    const int64_t target = std::max<int64_t>(1, (v.threads >= 512 ? 512 : 1024) / g.gy);
    g.stages_per_block = ceil_div(nstage, target);
    g.gx = ceil_div(ceil_div(nstage, g.stages_per_block), 8) * 8;
    // row subsets combined in the block when their values fit the X staging buffer
    // (k_linear_mfma's epilogue)
    const int rs_count = waves / wt;
    const int items = 16 * g.pt + 2;
    const int64_t lds_floats = ch * (32 * g.pt + 4);
    const bool combine = rs_count > 1 && (int64_t)(rs_count - 1) * wt * 64 * items <= lds_floats;
    g.ntile = (combine ? g.gx : g.gx * rs_count) + (L->prior.present != 0 ? 1 : 0);
    return g;
  }
  int kb = 1;
  while (kb < 256 && kb < L->K) kb <<= 1;
  g.kb = kb;
  g.gy = ceil_div(L->K, kb);
  // about 768 blocks in total (3 per CU), whole LDS chunks per tile
  const int64_t tiles = std::max<int64_t>(1, 768 / g.gy);
  g.rows_per_tile = std::max<int64_t>(mi::kLinChunk, ceil_div(ceil_div(L->N, tiles), mi::kLinChunk) * mi::kLinChunk);
  g.ntile = ceil_div(L->N, g.rows_per_tile);
  g.gx = g.ntile;
  return g;
}

int to_code(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

// The launch conditions of the site's options on this geometry (shared by the plain and the
// ELBO-finishing forward): 0, MI_EUNSUPPORTED or MI_EINVAL.
int launch_check(const mi_linear* site, const Geometry& g) {
  if (site->prior.present != 0 && !g.mfma) return MI_EUNSUPPORTED;   // (the VALU kernel has none)
  if (site->rows.counter != nullptr && (!g.mfma || g.stages_per_block != 1))
    return MI_EUNSUPPORTED;   // rows drawn only by one-stage matrix-core launches
  if (site->draw.operand != 0) {
    const mi_draw& D = site->draw;
    if (D.loc == nullptr || D.scale == nullptr || D.element_offset < 0 || (D.element_offset & 3) != 0 ||
        D.stream_id > 0xFFFFFFu)
      return MI_EINVAL;
    // theta drawn only by the matrix-core kernel, through its X staging buffer
    const int threads = g.mfma ? kMfVariants[g.variant].threads : 0;
    const int64_t lds_floats = (int64_t)((threads >= 512 ? 256 : 128) / std::max(1, g.pt)) * (32 * g.pt + 4);
    if (!g.mfma || site->P % 4 != 0 || (int64_t)g.wt * 32 * (32 * g.pt + 1) > lds_floats ||
        (int64_t)g.wt * 32 * (site->P / 4) > (int64_t)mi::kDrawItems * threads)
      return MI_EUNSUPPORTED;
  }
  return 0;
}

// Compute units of the current device (cached).
// per-(tile, particle) partials, 256-byte aligned so the finalize scratch behind them is too
size_t partial_bytes(const mi_linear* site, const Geometry& g) {
  return ((size_t)g.nv * (size_t)g.ntile * (size_t)site->K * sizeof(float) + 255) / 256 * 256;
}

template <int FAMILY, int PT, int NT, bool FLUSH64, int MINW>
void launch_mfma(const mi_linear& L, const Geometry& g, float* part, uint32_t* flags,
                 hipStream_t s) {
  const dim3 grid((unsigned)(g.gx * g.gy));
  const bool one = g.stages_per_block == 1;
#define MI_LAUNCH_MFMA(GRADS, ONE)                                                               \
  hipLaunchKernelGGL((mi::k_linear_mfma<FAMILY, PT, NT, FLUSH64, MINW, GRADS, ONE>), grid,       \
                     dim3(NT), 0, s, L, g.wt, (int)g.gy, g.stages_per_block, g.ntile, part, flags, \
                     L.rows.counter != nullptr ? mi_feistel_half(L.rows.n) : 0)
  if (L.compute_grads) {
    if (one) MI_LAUNCH_MFMA(true, true); else MI_LAUNCH_MFMA(true, false);
  } else {
    if (one) MI_LAUNCH_MFMA(false, true); else MI_LAUNCH_MFMA(false, false);
  }
#undef MI_LAUNCH_MFMA
}

template <int FAMILY, int PT>
void launch_mfma_variant(const mi_linear& L, const Geometry& g, float* part, uint32_t* flags,
                         hipStream_t s) {
  if (g.variant == 0)
    launch_mfma<FAMILY, PT, 256, false, 4>(L, g, part, flags, s);
  else
    launch_mfma<FAMILY, PT, 256, false, 2>(L, g, part, flags, s);
}

template <int FAMILY>
void launch(const mi_linear& L, const Geometry& g, float* part, uint32_t* flags, hipStream_t s) {
  const dim3 grid((unsigned)g.gx, (unsigned)g.gy);
  if (g.mfma) {
    if (g.pt == 1)
      launch_mfma_variant<FAMILY, 1>(L, g, part, flags, s);
    else
      launch_mfma_variant<FAMILY, 2>(L, g, part, flags, s);
    return;
  }
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

int mi_linear_prior_supported(const mi_linear* site, int* supported) {
  if (!valid(site) || supported == nullptr) return MI_EINVAL;
  *supported = geometry(site).mfma ? 1 : 0;
  return 0;
}

int mi_linear_workspace_bytes(const mi_linear* site, size_t* bytes) {
  if (!valid(site) || bytes == nullptr) return MI_EINVAL;
  const Geometry g = geometry(site);
  *bytes = partial_bytes(site, g) + mi_finalize_scratch_bytes(g.ntile, site->K, g.nv);
#if MI_LINEAR_TIMING
  *bytes = (*bytes + 255) / 256 * 256 + (size_t)g.gx * g.gy * 8 * 8 * sizeof(unsigned long long);
#endif
  return 0;
}

int mi_linear_forward_deferred(const mi_linear* site, void* workspace, size_t workspace_bytes,
                               float* total, float* dslots, uint32_t* flags, void* start_event,
                               void* stop_event, void* stream, mi_reduce* reduce) {
  if (reduce != nullptr) *reduce = mi_reduce{};
  if (!valid(site) || total == nullptr || flags == nullptr ||
      (site->compute_grads && dslots == nullptr))
    return MI_EINVAL;
  if (start_event != nullptr || stop_event != nullptr) {   // eager timing only (internal.hpp)
    bool capturing = false;
    const hipError_t ce = mi_stream_capturing(static_cast<hipStream_t>(stream), &capturing);
    if (ce != hipSuccess) return to_code(ce);
    if (capturing) return MI_EUNSUPPORTED;
  }
  size_t need = 0;
  mi_linear_workspace_bytes(site, &need);
  if (workspace == nullptr || workspace_bytes < need) return MI_EWORKSPACE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e;
  if (!(site->options & MI_GROUP_FLAGS_ZEROED)) {
    e = hipMemsetAsync(flags, 0, sizeof(uint32_t), s);
    if (e == hipSuccess && site->prior.present != 0)
      e = hipMemsetAsync(site->prior.flags, 0, sizeof(uint32_t), s);
    if (e != hipSuccess) return to_code(e);
  }
  const Geometry g = geometry(site);
  const int rc = launch_check(site, g);
  if (rc != 0) return rc;
  float* part = static_cast<float*>(workspace);
#if MI_LINEAR_TIMING
  {
    unsigned long long* tb = reinterpret_cast<unsigned long long*>(
        static_cast<char*>(workspace) +
        (partial_bytes(site, g) + mi_finalize_scratch_bytes(g.ntile, site->K, g.nv) + 255) / 256 * 256);
    if ((e = hipMemcpyToSymbolAsync(HIP_SYMBOL(mi::mi_lin_tbuf), &tb, sizeof(tb), 0,
                                    hipMemcpyHostToDevice, s)) != hipSuccess)
      return to_code(e);
  }
#endif
  if (start_event != nullptr && (e = mi_record_event(start_event, s)) != hipSuccess)
    return to_code(e);
  if (site->family == MI_NORMAL)
    launch<MI_NORMAL>(*site, g, part, flags, s);
  else
    launch<MI_BERNOULLI_LOGITS>(*site, g, part, flags, s);
  e = hipGetLastError();
  if (e != hipSuccess) return to_code(e);
  if (stop_event != nullptr && (e = mi_record_event(stop_event, s)) != hipSuccess)
    return to_code(e);
  const double scale = site->site_scale;
  if (reduce != nullptr && g.ntile <= MI_REDUCE_MAX_SEG) {   // the caller runs the finalize
    reduce->part = part;
    reduce->nseg = g.ntile;
    reduce->K = site->K;
    reduce->num_sites = 1;
    reduce->num_slots = site->compute_grads ? g.nv - 1 : 0;
    reduce->scale[0] = scale;
    reduce->slot_scale = (double)site->grad_scale;
    reduce->total = total;
    reduce->slot_grad = dslots;
    return 0;
  }
  double* scratch = reinterpret_cast<double*>(static_cast<char*>(workspace) + partial_bytes(site, g));
  return mi_launch_finalize(part, g.ntile, site->K, 1, site->compute_grads ? g.nv - 1 : 0, &scale,
                            (double)site->grad_scale, total, nullptr, dslots, scratch, s);
}

int mi_linear_forward(const mi_linear* site, void* workspace, size_t workspace_bytes, float* total,
                      float* dslots, uint32_t* flags, void* stream) {
  return mi_linear_forward_deferred(site, workspace, workspace_bytes, total, dslots, flags, nullptr,
                                    nullptr, stream, nullptr);
}

}  // extern "C"
