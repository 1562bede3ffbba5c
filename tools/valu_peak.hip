// Microbenchmark: sustained FP32 VALU rate of v_pk_fma_f32 vs v_fma_f32 on this device (the
// ceiling the BCAST / linear site kernels are compared with). Build: hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int CH>
__global__ __launch_bounds__(256) void k_pk(float* out, float a, int iters) {
  f32x2 acc[CH];
  const f32x2 m = f32x2{a, a * 0.5f};
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = f32x2{(float)threadIdx.x + c, (float)c};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] = __builtin_elementwise_fma(acc[c], m, m);
  }
  float s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c].x + acc[c].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int CH>
__global__ __launch_bounds__(256) void k_fma(float* out, float a, int iters) {
  float acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = (float)threadIdx.x + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] = fmaf(acc[c], a, a);
  }
  float s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// 32x32->64 multiplies (v_mad_u64_u32) as Philox uses them: CH independent chains.
template <int CH>
__global__ __launch_bounds__(256) void k_mad64(float* out, unsigned a, int iters) {
  unsigned acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x * 7u + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const unsigned long long p = (unsigned long long)0xD2511F53u * acc[c];
        acc[c] = (unsigned)(p >> 32) + (unsigned)p;   // folds into the mad's add? no: one add
      }
  }
  unsigned s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = (float)(s + a);
}

// hardware exp2 (v_exp_f32): CH independent chains.
template <int CH>
__global__ __launch_bounds__(256) void k_exp(float* out, float a, int iters) {
  float acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = (float)threadIdx.x * 1e-3f + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_exp2f(acc[c]) * a;
  }
  float s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <typename F>
void run(const char* name, F launch, double flop) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) launch();
  hipEventRecord(a);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  printf("%-28s %8.1f us  %7.1f TFLOP/s\n", name, 1e3 * ms / reps, flop * reps / (ms * 1e-3) / 1e12);
}

int main() {
  float* out;
  const int blocks = 2048, iters = 2000;
  hipMalloc(&out, blocks * 256 * sizeof(float));
  const double lanes = (double)blocks * 256 * iters * 16;
  run("pk_fma 8 chains", [&] { hipLaunchKernelGGL(k_pk<8>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, iters); }, lanes * 8 * 4);
  run("pk_fma 4 chains", [&] { hipLaunchKernelGGL(k_pk<4>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, iters); }, lanes * 4 * 4);
  run("fma 8 chains", [&] { hipLaunchKernelGGL(k_fma<8>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, iters); }, lanes * 8 * 2);
  run("fma 16 chains", [&] { hipLaunchKernelGGL(k_fma<16>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, iters); }, lanes * 16 * 2);
  run("pk_fma 8 chains (1024 blk)", [&] { hipLaunchKernelGGL(k_pk<8>, dim3(1024), dim3(256), 0, 0, out, 0.999f, iters); }, lanes / 2 * 8 * 4);
  // per-lane operations: report the cost per wave-instruction pair in SIMD cycles at 2.4 GHz
  run("mad_u64+add 8 chains", [&] { hipLaunchKernelGGL(k_mad64<8>, dim3(blocks), dim3(256), 0, 0, out, 3u, iters); }, lanes * 8);
  run("exp2+mul 8 chains", [&] { hipLaunchKernelGGL(k_exp<8>, dim3(blocks), dim3(256), 0, 0, out, 0.5f, iters); }, lanes * 8);
  run("fma 8 chains (ops)", [&] { hipLaunchKernelGGL(k_fma<8>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, iters); }, lanes * 8);
  return 0;
}
