// Diagnostic copy of k_site_bcast_smem's main loop (Bernoulli logits, scalar-unit data loads) with
// per-workgroup start/end stamps (s_memrealtime, 100 MHz) and the in-kernel clock
// (s_memtime / s_memrealtime): where the C2 site kernel's time goes. Not used by the library.
//   hipcc -O3 --offload-arch=gfx950 -fno-slp-vectorize tools/bcast_probe.hip -o tools/bcast_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(4))) float smem_float;

template <int P, int CHUNK, bool LOADS, int PREP = 0, bool POST = false>
__global__ __launch_bounds__(256) void k_probe(const float* __restrict__ x, const float* __restrict__ logits,
                                               int64_t N, int64_t K, float* __restrict__ part,
                                               unsigned long long* __restrict__ stamps) {
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const int64_t c = blockIdx.x;
  const int64_t i0 = c * CHUNK;
  const int len = (int)min((int64_t)CHUNK, N - i0);
  const int64_t kbase = (int64_t)blockIdx.y * (256 * P) + threadIdx.x;
  f32x2 ld[P];
  double acc[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    float l = logits[min(kbase + p * 256, K - 1)];
    if (PREP == 1) {   // probs -> logits, precise libm (as bernoulli_probs_to_logits)
      const float pc = fminf(fmaxf(l * 0.5f, 1.1920929e-07f), 1.0f - 1.1920929e-07f);
      l = logf(pc) - log1pf(-pc) + (1.0f / pc + 1.0f / (1.0f - pc)) * 1e-30f;
    } else if (PREP == 2) {   // hardware v_log_f32 / v_rcp_f32
      const float pc = fminf(fmaxf(l * 0.5f, 1.1920929e-07f), 1.0f - 1.1920929e-07f);
      l = (__builtin_amdgcn_logf(pc) - __builtin_amdgcn_logf(1.0f - pc)) * 0.69314718f +
          (__builtin_amdgcn_rcpf(pc) + __builtin_amdgcn_rcpf(1.0f - pc)) * 1e-30f;
    }
    ld[p] = f32x2{l, l};
    acc[p] = 0.0;
  }
  smem_float* xs = (smem_float*)(x + i0);
  constexpr int kGroup = 32, kBlock = 256;
  const int nfull = len & ~(kBlock - 1);
  if (nfull > 0) {
    float xc[kGroup];
#pragma unroll
    for (int e = 0; e < kGroup; ++e) xc[e] = LOADS ? xs[e] : 1.0f;
    for (int j = 0; j < nfull; j += kBlock) {
      f32x2 in[2][P];
#pragma unroll
      for (int p = 0; p < P; ++p) in[0][p] = in[1][p] = f32x2{0.0f, 0.0f};
#pragma unroll
      for (int g = 0; g < kBlock; g += kGroup) {
        const int nxt = min(j + g + kGroup, nfull - kGroup);
        float xn[kGroup];
#pragma unroll
        for (int e = 0; e < kGroup; ++e) xn[e] = LOADS ? xs[nxt + e] : xc[(e + 1) % kGroup];
#pragma unroll
        for (int e = 0; e < kGroup; e += 2) {
          const f32x2 xv = f32x2{xc[e], xc[e + 1]};
#pragma unroll
          for (int p = 0; p < P; ++p)
            in[(e >> 1) & 1][p] = __builtin_elementwise_fma(xv, ld[p], in[(e >> 1) & 1][p]);
        }
#pragma unroll
        for (int e = 0; e < kGroup; ++e) xc[e] = xn[e];
      }
#pragma unroll
      for (int p = 0; p < P; ++p)
        acc[p] += (double)((in[0][p].x + in[0][p].y) + (in[1][p].x + in[1][p].y));
    }
  }
  float s_a = 0.0f;
  if (POST) {
    __shared__ float red[4];
    for (int i = threadIdx.x; i < len; i += 256) s_a += x[i0 + i];
    for (int o = 32; o > 0; o >>= 1) s_a += __shfl_xor(s_a, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s_a;
    __syncthreads();
    s_a = red[0] + red[1] + red[2] + red[3];
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int64_t k = kbase + p * 256;
    if (k < K) part[c * K + k] = (float)acc[p] + s_a;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t b = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(hw));
    unsigned hwid;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    stamps[4 * b + 0] = t0;
    stamps[4 * b + 1] = __builtin_amdgcn_s_memrealtime();
    stamps[4 * b + 2] = __builtin_amdgcn_s_memtime() - c0;
    stamps[4 * b + 3] = ((unsigned long long)hw << 32) | hwid;
  }
}

// The same sums with the chunk staged in LDS (coalesced float4 loads, one pass) and read back as
// broadcast ds_read_b128 (every lane the same address) into VGPR pairs: v_pk_fma_f32 with all
// operands in VGPRs and the data latency decoupled from the scalar unit.
template <int P, int CHUNK>
__global__ __launch_bounds__(256) void k_probe_lds(const float* __restrict__ x, const float* __restrict__ logits,
                                                   int64_t N, int64_t K, float* __restrict__ part,
                                                   unsigned long long* __restrict__ stamps) {
  __shared__ float4 xl[CHUNK / 4];
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const int64_t c = blockIdx.x;
  const int64_t i0 = c * CHUNK;
  const int len = (int)min((int64_t)CHUNK, N - i0);
  const int nq = len / 4;
  const float4* xg = reinterpret_cast<const float4*>(x + i0);
  for (int q = threadIdx.x; q < nq; q += 256) xl[q] = xg[q];
  const int64_t kbase = (int64_t)blockIdx.y * (256 * P) + threadIdx.x;
  f32x2 ld[P];
  double acc[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const float l = logits[min(kbase + p * 256, K - 1)];
    ld[p] = f32x2{l, l};
    acc[p] = 0.0;
  }
  __syncthreads();
  constexpr int kQ = 64;   // quads per fp32 partial (256 elements)
  int q = 0;
  for (; q + kQ <= nq; q += kQ) {
    f32x2 in[2][P];
#pragma unroll
    for (int p = 0; p < P; ++p) in[0][p] = in[1][p] = f32x2{0.0f, 0.0f};
#pragma unroll 16
    for (int e = 0; e < kQ; ++e) {
      const float4 v = xl[q + e];
      const f32x2 a = f32x2{v.x, v.y}, b = f32x2{v.z, v.w};
#pragma unroll
      for (int p = 0; p < P; ++p) {
        in[0][p] = __builtin_elementwise_fma(a, ld[p], in[0][p]);
        in[1][p] = __builtin_elementwise_fma(b, ld[p], in[1][p]);
      }
    }
#pragma unroll
    for (int p = 0; p < P; ++p)
      acc[p] += (double)((in[0][p].x + in[0][p].y) + (in[1][p].x + in[1][p].y));
  }
  for (; q < nq; ++q) {
    const float4 v = xl[q];
#pragma unroll
    for (int p = 0; p < P; ++p) acc[p] += (double)(v.x * ld[p].x + v.y * ld[p].x + v.z * ld[p].x + v.w * ld[p].x);
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int64_t k = kbase + p * 256;
    if (k < K) part[c * K + k] = (float)acc[p];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t b = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    stamps[4 * b + 0] = t0;
    stamps[4 * b + 1] = __builtin_amdgcn_s_memrealtime();
    stamps[4 * b + 2] = __builtin_amdgcn_s_memtime() - c0;
    stamps[4 * b + 3] = 0;
  }
}

// Half of each chunk through the scalar unit (SGPR pairs), the other half staged in LDS and read
// as broadcast ds_read_b128 (VGPR pairs), interleaved group by group: twice the FMAs per scalar
// group of lookahead, the LDS at half the rate of k_probe_lds. Full chunks only (CHUNK | N not
// required: the partial last chunk is skipped).
template <int P, int CHUNK>
__global__ __launch_bounds__(256) void k_probe_hyb(const float* __restrict__ x, const float* __restrict__ logits,
                                                   int64_t N, int64_t K, float* __restrict__ part,
                                                   unsigned long long* __restrict__ stamps) {
  constexpr int kHalf = CHUNK / 2, kGroup = 32, kGroups = kHalf / kGroup;
  static_assert(kHalf % kGroup == 0, "whole groups");
  __shared__ float4 xl[kHalf / 4];
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const int64_t c = blockIdx.x;
  const int64_t i0 = c * CHUNK;
  const int64_t kbase = (int64_t)blockIdx.y * (256 * P) + threadIdx.x;
  double acc[P];
#pragma unroll
  for (int p = 0; p < P; ++p) acc[p] = 0.0;
  if (i0 + CHUNK <= N) {
    const float4* xg = reinterpret_cast<const float4*>(x + i0 + kHalf);
    for (int q = threadIdx.x; q < kHalf / 4; q += 256) xl[q] = xg[q];
    f32x2 ld[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const float l = logits[min(kbase + p * 256, K - 1)];
      ld[p] = f32x2{l, l};
    }
    __syncthreads();
    smem_float* xs = (smem_float*)(x + i0);
    float xc[kGroup];
#pragma unroll
    for (int e = 0; e < kGroup; ++e) xc[e] = xs[e];
    for (int g = 0; g < kGroups; g += 8) {
      f32x2 in[2][P];
#pragma unroll
      for (int p = 0; p < P; ++p) in[0][p] = in[1][p] = f32x2{0.0f, 0.0f};
#pragma unroll
      for (int h = 0; h < 8; ++h) {
        const int nxt = min(g + h + 1, kGroups - 1) * kGroup;
        float xn[kGroup];
#pragma unroll
        for (int e = 0; e < kGroup; ++e) xn[e] = xs[nxt + e];
        float4 vb[kGroup / 4];
#pragma unroll
        for (int q = 0; q < kGroup / 4; ++q) vb[q] = xl[(g + h) * (kGroup / 4) + q];
#pragma unroll
        for (int e = 0; e < kGroup; e += 2) {
          const f32x2 xv = f32x2{xc[e], xc[e + 1]};
#pragma unroll
          for (int p = 0; p < P; ++p) in[0][p] = __builtin_elementwise_fma(xv, ld[p], in[0][p]);
        }
#pragma unroll
        for (int q = 0; q < kGroup / 4; ++q) {
          const f32x2 a = f32x2{vb[q].x, vb[q].y}, b = f32x2{vb[q].z, vb[q].w};
#pragma unroll
          for (int p = 0; p < P; ++p) {
            in[1][p] = __builtin_elementwise_fma(a, ld[p], in[1][p]);
            in[1][p] = __builtin_elementwise_fma(b, ld[p], in[1][p]);
          }
        }
#pragma unroll
        for (int e = 0; e < kGroup; ++e) xc[e] = xn[e];
      }
#pragma unroll
      for (int p = 0; p < P; ++p)
        acc[p] += (double)((in[0][p].x + in[0][p].y) + (in[1][p].x + in[1][p].y));
    }
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int64_t k = kbase + p * 256;
    if (k < K) part[c * K + k] = (float)acc[p];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t b = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    stamps[4 * b + 0] = t0;
    stamps[4 * b + 1] = __builtin_amdgcn_s_memrealtime();
    stamps[4 * b + 2] = __builtin_amdgcn_s_memtime() - c0;
    stamps[4 * b + 3] = 0;
  }
}

template <int P, int CHUNK, bool LOADS, int PREP = 0, bool POST = false, bool LDS = false, bool HYB = false>
void run(const char* name, const float* x, const float* lg, int64_t N, int64_t K, float* part,
         unsigned long long* stamps) {
  const dim3 grid((unsigned)((N + CHUNK - 1) / CHUNK), (unsigned)((K + 256 * P - 1) / (256 * P)));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto launch = [&]() {
    if (HYB) hipLaunchKernelGGL((k_probe_hyb<P, CHUNK>), grid, dim3(256), 0, 0, x, lg, N, K, part, stamps);
    else if (LDS) hipLaunchKernelGGL((k_probe_lds<P, CHUNK>), grid, dim3(256), 0, 0, x, lg, N, K, part, stamps);
    else hipLaunchKernelGGL((k_probe<P, CHUNK, LOADS, PREP, POST>), grid, dim3(256), 0, 0, x, lg, N, K, part, stamps);
  };
  for (int w = 0; w < 5; ++w) launch();
  (void)hipEventRecord(a);
  const int reps = 20;
  for (int r = 0; r < reps; ++r) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const int nb = grid.x * grid.y;
  std::vector<unsigned long long> h(4 * nb);
  (void)hipMemcpy(h.data(), stamps, 8 * 4 * nb, hipMemcpyDeviceToHost);
  unsigned long long tmin = ~0ull, tmax = 0, smin = ~0ull, smax = 0;
  double life = 0, clk = 0;
  for (int i = 0; i < nb; ++i) {
    tmin = std::min(tmin, h[4 * i]);
    smax = std::max(smax, h[4 * i]);
    tmax = std::max(tmax, h[4 * i + 1]);
    life += (double)(h[4 * i + 1] - h[4 * i]);
    clk += (double)h[4 * i + 2] / (double)(h[4 * i + 1] - h[4 * i] + 1) * 100.0;
  }
  const double us = 1e3 * ms / reps;
  if (FILE* f = fopen((std::string("gpurun_out/probe_") + name + ".csv").c_str(), "w")) {
    for (int i = 0; i < nb; ++i)
      fprintf(f, "%d,%llu,%llu,%llu,%llu\n", i, h[4 * i + 3] >> 32, h[4 * i + 3] & 0xffffffffull,
              h[4 * i] - tmin, h[4 * i + 1] - tmin);
    fclose(f);
  }
  printf("%-26s grid %4u x %u: %7.1f us  %6.1f TF | last launch: span %6.1f us  start spread %6.1f us  "
         "mean block life %6.1f us  clock %5.0f MHz\n",
         name, grid.x, grid.y, us, 2.0 * K * N / (us * 1e-6) / 1e12, (tmax - tmin) / 100.0,
         (smax - tmin) / 100.0, life / nb / 100.0, clk / nb);
}

int main() {
  const int64_t N = 1000000, K = 4096;
  float *x, *lg, *part;
  unsigned long long* stamps;
  (void)hipMalloc(&x, N * 4);
  (void)hipMalloc(&lg, K * 4);
  (void)hipMalloc(&part, 4 * 1024 * K);
  (void)hipMalloc(&stamps, 8 * 4 * 8192);
  std::vector<float> hx(N), hl(K);
  for (int64_t i = 0; i < N; ++i) hx[i] = (float)((i * 2654435761u >> 7) % 10 < 7);
  for (int64_t k = 0; k < K; ++k) hl[k] = 0.3f + 0.001f * (float)(k % 100);
  (void)hipMemcpy(x, hx.data(), N * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(lg, hl.data(), K * 4, hipMemcpyHostToDevice);
  run<4, 4096, true>("P4_C4096", x, lg, N, K, part, stamps);
  run<4, 4096, true, 0, false, false, true>("P4_C4096_hyb", x, lg, N, K, part, stamps);
  run<4, 3968, true>("P4_C3968", x, lg, N, K, part, stamps);
  run<4, 3968, true, 0, false, false, true>("P4_C3968_hyb", x, lg, N, K, part, stamps);
  run<8, 2048, true>("P8_C2048", x, lg, N, K, part, stamps);
  run<8, 2048, true, 0, false, false, true>("P8_C2048_hyb", x, lg, N, K, part, stamps);
  run<4, 4096, true>("P4_C4096", x, lg, N, K, part, stamps);
  run<4, 4096, true, 0, false, false, true>("P4_C4096_hyb", x, lg, N, K, part, stamps);
  return 0;
}
