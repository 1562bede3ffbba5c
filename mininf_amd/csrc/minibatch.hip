// Device-resident minibatches: the host DataLoader of the reference's minibatch example
// (examples/minibatch.md:78-88: DataLoader(TensorDataset(X, y), batch_size, shuffle=True), one
// `condition(model, X=X, y=y)` per batch) as row indices computed on the device.
//
// Batch b of epoch e holds the rows perm_e(b * batch + j), j < batch (shuffle) or b * batch + j
// (sequential), where perm_e is a keyed Feistel permutation of [0, n): a random permutation per
// epoch without a sort, without storing it, and without any host involvement -- a captured
// training step draws the next batch on every replay. The batch counter lives in device memory;
// the launch that reads it advances it. Site kernels read the rows through the index
// (mi_linear.row_index); mi_gather_rows materialises a batch for any other use.
#include "common.hpp"
#include "internal.hpp"

namespace mi {

constexpr int kRowThreads = 256;
constexpr int kFeistelRounds = 4;

// murmur3's 32-bit finaliser of x ^ key: the Feistel round function.
MI_DEV uint32_t round_fn(uint32_t x, uint32_t key) {
  x ^= key;
  x *= 0xcc9e2d51u;
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

// One pass of the balanced Feistel network over 2 * half bits.
MI_DEV uint64_t feistel(uint64_t x, int half, const uint32_t (&keys)[kFeistelRounds]) {
  const uint64_t mask = (1ull << half) - 1ull;
  uint64_t l = x >> half, r = x & mask;
#pragma unroll
  for (int q = 0; q < kFeistelRounds; ++q) {
    const uint64_t t = l ^ ((uint64_t)round_fn((uint32_t)r, keys[q]) & mask);
    l = r;
    r = t;
  }
  return (l << half) | r;
}

// counter[0]: batches drawn so far; counter[1]: completion count of the launch's blocks (zero
// between launches). Every block reads counter[0]; the last block to finish advances it, so no
// block can read the advanced value.
__global__ __launch_bounds__(kRowThreads) void k_minibatch_rows(uint64_t* __restrict__ counter,
                                                                int64_t n, int64_t batch,
                                                                int64_t batches, int shuffle,
                                                                uint64_t seed, int half,
                                                                int32_t* __restrict__ rows,
                                                                int64_t count) {
  const uint64_t c = counter[0];
  const uint64_t epoch = c / (uint64_t)batches, b = c % (uint64_t)batches;
  uint32_t keys[kFeistelRounds];
#pragma unroll
  for (int q = 0; q < kFeistelRounds; ++q)
    keys[q] = round_fn((uint32_t)(seed ^ (seed >> 32)) ^ (uint32_t)q * 0x9e3779b9u,
                       round_fn((uint32_t)epoch, (uint32_t)(epoch >> 32) + 0x7f4a7c15u));
  const int64_t j = (int64_t)blockIdx.x * kRowThreads + threadIdx.x;
  if (j < count) {
    uint64_t x = b * (uint64_t)batch + (uint64_t)j;
    if (x >= (uint64_t)n) {
      x %= (uint64_t)n;   // (a batch position past the data: mi_minibatch_rows rejects it)
    } else if (shuffle) {
      // cycle walking: the orbit of x under the permutation of [0, 2^(2 half)) returns to
      // [0, n) because x itself lies there
      do {
        x = feistel(x, half, keys);
      } while (x >= (uint64_t)n);
    }
    rows[j] = (int32_t)x;
  }
  __syncthreads();   // every thread of the block has read the counter
  if (threadIdx.x == 0) {
    const unsigned long long done = atomicAdd((unsigned long long*)&counter[1], 1ull);
    if (done == gridDim.x - 1) {   // the last block: every block has read counter[0]
      counter[1] = 0;
      counter[0] = c + 1;
    }
  }
}

// count rows of `words` 32-bit words each: out[j] = base[rows[j]].
__global__ __launch_bounds__(256) void k_gather_rows(const uint32_t* __restrict__ base,
                                                     int64_t base_stride, int64_t words,
                                                     const int32_t* __restrict__ rows,
                                                     int64_t count, uint32_t* __restrict__ out,
                                                     int64_t out_stride) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t j = t / words, w = t % words;
  if (j >= count) return;
  out[j * out_stride + w] = base[(int64_t)rows[j] * base_stride + w];
}

}  // namespace mi

namespace {

int to_code(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

int feistel_half(int64_t n) {
  int bits = 2;
  while (bits < 62 && (1ll << bits) < n) ++bits;
  return (bits + 1) / 2;
}

}  // namespace

extern "C" {

int mi_minibatch_rows(uint64_t* counter, int64_t n, int64_t batch, int64_t batches_per_epoch,
                      int32_t shuffle, uint64_t seed, int32_t* rows, int64_t count,
                      void* stream) {
  if (counter == nullptr || rows == nullptr || n < 1 || n > INT32_MAX || batch < 1 ||
      batches_per_epoch < 1 || count < 1 || count > batch ||
      (batches_per_epoch - 1) * batch >= n || batches_per_epoch * batch >= n + batch)
    return MI_EINVAL;
  hipLaunchKernelGGL(mi::k_minibatch_rows,
                     dim3((unsigned)((count + mi::kRowThreads - 1) / mi::kRowThreads)),
                     dim3(mi::kRowThreads), 0,
                     static_cast<hipStream_t>(stream), counter, n, batch, batches_per_epoch,
                     shuffle ? 1 : 0, seed, feistel_half(n), rows, count);
  return to_code(hipGetLastError());
}

int mi_gather_rows(const void* base, int64_t base_stride_bytes, int64_t row_bytes,
                   const int32_t* rows, int64_t count, void* out, int64_t out_stride_bytes,
                   void* stream) {
  if (base == nullptr || rows == nullptr || out == nullptr || count < 1 || row_bytes < 4 ||
      row_bytes % 4 || base_stride_bytes % 4 || out_stride_bytes % 4 ||
      (reinterpret_cast<uintptr_t>(base) & 3) || (reinterpret_cast<uintptr_t>(out) & 3))
    return MI_EINVAL;
  const int64_t words = row_bytes / 4;
  const int64_t total = words * count;
  hipLaunchKernelGGL(mi::k_gather_rows, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint32_t*>(base),
                     base_stride_bytes / 4, words, rows, count, static_cast<uint32_t*>(out),
                     out_stride_bytes / 4);
  return to_code(hipGetLastError());
}

}  // extern "C"
