// Streaming-bandwidth probe for the Adam update's access pattern (C5: two tensors of 1e6 floats;
// read param, grad, exp_avg, exp_avg_sq, write param, exp_avg, exp_avg_sq: 28 B per element).
// Each variant runs 200 launches captured in one hipGraph (back to back, as in a replayed step);
// prints the mean time per launch and the algorithmic bandwidth.
//
//   hipcc --offload-arch=gfx950 -O3 -Iinclude -Imininf_amd/csrc -o tools/_timing/stream_probe \
//       tools/stream_probe.hip
//   tools/_timing/stream_probe [elements per tensor]
#include <hip/hip_runtime.h>

#include "adam_math.hpp"   // (mininf_amd/csrc: torch's fused-Adam arithmetic, fp64 hyper-parameters)
#include "adam.hip"        // the library's k_adam_step / mi_adam_step itself, for the same harness

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

constexpr int kThreads = 256;

struct Tensors {
  float4* p[2];
  const float4* g[2];
  float4* m[2];
  float4* v[2];
  long quads;        // per tensor
  const float* step; // device step count
};

__device__ __forceinline__ void adam4(float4& p, const float4& g, float4& m, float4& v, float lr,
                                      float bc1, float bc2s) {
  const float b1 = 0.9f, b2 = 0.999f, eps = 1e-8f;
#define UPD(c)                                          \
  m.c = fmaf(b1, m.c - g.c, g.c);                       \
  v.c = fmaf(b2, v.c, (1.0f - b2) * g.c * g.c);         \
  p.c -= lr * bc1 * m.c / (sqrtf(v.c) * bc2s + eps);
  UPD(x) UPD(y) UPD(z) UPD(w)
#undef UPD
}

// MODE 0: Adam math, coefficients from the step count in fp64 (pow) per block
// MODE 1: Adam math, coefficients precomputed (a fixed float)
// MODE 2: pure copy (p += g; m, v rewritten), no math
// MODE 3: adam_math.hpp's adam_update (the library's arithmetic), coefficients precomputed
// MODE 4: MODE 3 plus the library kernel's prologue (step read, wait, barrier, one atomic per block)
// Q quads per lane per pass; blocks split the 2 * quads evenly (one tensor per half of the grid).
template <int MODE, int Q>
__global__ __launch_bounds__(kThreads) void k_stream(Tensors T, int blocks_per_tensor,
                                                      mi_adam H, unsigned* counter) {
  const int t = blockIdx.x >= blocks_per_tensor;
  const long b = blockIdx.x - t * blocks_per_tensor;
  const long chunk = (T.quads + blocks_per_tensor - 1) / blocks_per_tensor;
  const long q0 = b * chunk, q1 = min(T.quads, q0 + chunk);
  float4* __restrict__ P = T.p[t];
  const float4* __restrict__ G = T.g[t];
  float4* __restrict__ M = T.m[t];
  float4* __restrict__ V = T.v[t];
  float4 p[Q], g[Q], m[Q], v[Q];
  long q = q0 + threadIdx.x;
  auto load = [&](long base) {
#pragma unroll
    for (int u = 0; u < Q; ++u) {
      const long e = base + u * kThreads;
      if (e < q1) { p[u] = P[e]; g[u] = G[e]; m[u] = M[e]; v[u] = V[e]; }
    }
  };
  load(q);
  __builtin_amdgcn_sched_barrier(0);
  float bc1 = 1.0f, bc2s = 1.0f;
  if (MODE == 4) {
    const float s1 = *T.step + 1.0f;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    if (threadIdx.x == 0 && s1 > 0.0f) atomicAdd(counter + (blockIdx.x & 31) * 16, 1u);
  }
  const mi::AdamCoef coef{0.5f, 0.7f, 1e-9f};
  if (MODE == 0) {
    const double s = (double)*T.step + 1.0;
    bc1 = (float)(1.0 / (1.0 - pow(0.9, s)));
    bc2s = (float)(1.0 / sqrt(1.0 - pow(0.999, s)));
  } else if (MODE == 1) {
    bc1 = 1.5f;
    bc2s = 2.0f;
  }
  for (; q < q1; q += Q * kThreads) {
#pragma unroll
    for (int u = 0; u < Q; ++u) {
      const long e = q + u * kThreads;
      if (e < q1) {
        if (MODE == 2) {
          p[u].x += g[u].x; p[u].y += g[u].y; p[u].z += g[u].z; p[u].w += g[u].w;
        } else if (MODE >= 3) {
          mi::adam_update(H, coef, p[u].x, g[u].x, m[u].x, v[u].x);
          mi::adam_update(H, coef, p[u].y, g[u].y, m[u].y, v[u].y);
          mi::adam_update(H, coef, p[u].z, g[u].z, m[u].z, v[u].z);
          mi::adam_update(H, coef, p[u].w, g[u].w, m[u].w, v[u].w);
        } else {
          adam4(p[u], g[u], m[u], v[u], 1e-9f, bc1, bc2s);
        }
        P[e] = p[u];
        M[e] = m[u];
        V[e] = v[u];
      }
    }
    load(q + Q * kThreads);
  }
}

template <int MODE, int Q>
void run(const char* name, Tensors T, int blocks_per_tensor, hipStream_t s, long n,
         const mi_adam& H, unsigned* counter) {
  const int reps = 200;
  hipGraph_t graph;
  hipGraphExec_t exec;
  CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((k_stream<MODE, Q>), dim3(2 * blocks_per_tensor), dim3(kThreads), 0, s, T,
                       blocks_per_tensor, H, counter);
  CHECK(hipStreamEndCapture(s, &graph));
  CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  CHECK(hipGraphLaunch(exec, s));   // warm-up
  CHECK(hipEventRecord(a, s));
  for (int i = 0; i < 3; ++i) CHECK(hipGraphLaunch(exec, s));
  CHECK(hipEventRecord(b, s));
  CHECK(hipEventSynchronize(b));
  float ms = 0.0f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double us = 1e3 * ms / (3 * reps);
  const double bytes = 28.0 * 2 * n;
  std::printf("%-10s Q=%d blocks=%5d  %7.2f us  %5.2f TB/s\n", name, Q, 2 * blocks_per_tensor, us,
              bytes / (us * 1e-6) / 1e12);
  std::fflush(stdout);
  CHECK(hipGraphExecDestroy(exec));
  CHECK(hipGraphDestroy(graph));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : 1000000;
  const long quads = (n + 3) / 4;
  Tensors T{};
  T.quads = quads;
  for (int t = 0; t < 2; ++t) {
    float4 *p, *g, *m, *v;
    CHECK(hipMalloc(&p, quads * 16));
    CHECK(hipMalloc(&g, quads * 16));
    CHECK(hipMalloc(&m, quads * 16));
    CHECK(hipMalloc(&v, quads * 16));
    CHECK(hipMemset(p, 0, quads * 16));
    CHECK(hipMemset(g, 0, quads * 16));
    CHECK(hipMemset(m, 0, quads * 16));
    CHECK(hipMemset(v, 0, quads * 16));
    T.p[t] = p; T.g[t] = g; T.m[t] = m; T.v[t] = v;
  }
  float* step;
  CHECK(hipMalloc(&step, sizeof(float)));
  CHECK(hipMemset(step, 0, sizeof(float)));
  T.step = step;
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  mi_adam H{};
  H.lr = 1e-3;
  H.beta1 = 0.9;
  H.beta2 = 0.999;
  H.eps = 1e-8;
  unsigned* counter;
  CHECK(hipMalloc(&counter, 32 * 16 * sizeof(unsigned)));
  CHECK(hipMemset(counter, 0, 32 * 16 * sizeof(unsigned)));
  for (int bpt : {256, 512}) {
    run<1, 2>("adam-f32", T, bpt, s, n, H, counter);
    run<3, 2>("adam-lib", T, bpt, s, n, H, counter);
    run<4, 2>("adam-lib+p", T, bpt, s, n, H, counter);
    run<0, 2>("adam-pow", T, bpt, s, n, H, counter);
  }
  // the library's launch over the same two tensors (plus its step words)
  {
    float* steps;
    unsigned* words;
    CHECK(hipMalloc(&steps, 2 * sizeof(float)));
    CHECK(hipMemset(steps, 0, 2 * sizeof(float)));
    CHECK(hipMalloc(&words, MI_ADAM_COUNTER_WORDS * sizeof(unsigned)));
    CHECK(hipMemset(words, 0, MI_ADAM_COUNTER_WORDS * sizeof(unsigned)));
    mi_adam A = H;
    A.num = 2;
    for (int t = 0; t < 2; ++t) {
      A.tensors[t].param = reinterpret_cast<float*>(T.p[t]);
      A.tensors[t].grad = reinterpret_cast<const float*>(T.g[t]);
      A.tensors[t].exp_avg = reinterpret_cast<float*>(T.m[t]);
      A.tensors[t].exp_avg_sq = reinterpret_cast<float*>(T.v[t]);
      A.tensors[t].step = steps + t;
      A.tensors[t].numel = n;
    }
    const int reps = 200;
    hipGraph_t graph;
    hipGraphExec_t exec;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int r = 0; r < reps; ++r)
      if (mi_adam_step(&A, words, s) != 0) std::exit(2);
    CHECK(hipStreamEndCapture(s, &graph));
    CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipGraphLaunch(exec, s));
    CHECK(hipEventRecord(a, s));
    for (int i = 0; i < 3; ++i) CHECK(hipGraphLaunch(exec, s));
    CHECK(hipEventRecord(b, s));
    CHECK(hipEventSynchronize(b));
    float ms = 0.0f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double us = 1e3 * ms / (3 * reps);
    std::printf("%-10s             %7.2f us  %5.2f TB/s\n", "mi_adam_step", us,
                28.0 * 2 * n / (us * 1e-6) / 1e12);
  }
  CHECK(hipStreamSynchronize(s));
  return 0;
}
