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
#include "rows.hpp"

namespace mi {

constexpr int kRowThreads = 256;
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
  const BatchOrder order = batch_order(c, batches, seed);
  const int64_t j = (int64_t)blockIdx.x * kRowThreads + threadIdx.x;
  if (j < count) rows[j] = batch_row(order, j, n, batch, shuffle, half);
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
                     shuffle ? 1 : 0, seed, mi_feistel_half(n), rows, count);
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
