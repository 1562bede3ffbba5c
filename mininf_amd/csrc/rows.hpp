// Minibatch row order (mi_minibatch_rows, and the site kernels that draw their batch's rows
// themselves, mi_linear.rows): batch b of epoch e holds the rows perm_e(b * batch + j), j < batch
// (shuffle) or b * batch + j (sequential), where perm_e is a keyed 4-round Feistel permutation of
// [0, n) (murmur3 finaliser rounds, cycle-walking into [0, n)) -- a fresh random order per epoch
// with no sort, nothing stored and no host involvement. oracle/minibatch.py restates it.
#pragma once

#include "common.hpp"

namespace mi {

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

// The row order of the batch numbered `c` (batches drawn so far): keys of its epoch.
struct BatchOrder {
  uint64_t b;                       // batch within the epoch
  uint32_t keys[kFeistelRounds];
};

MI_DEV BatchOrder batch_order(uint64_t c, int64_t batches, uint64_t seed) {
  BatchOrder o;
  const uint64_t epoch = c / (uint64_t)batches;
  o.b = c % (uint64_t)batches;
#pragma unroll
  for (int q = 0; q < kFeistelRounds; ++q)
    o.keys[q] = round_fn((uint32_t)(seed ^ (seed >> 32)) ^ (uint32_t)q * 0x9e3779b9u,
                         round_fn((uint32_t)epoch, (uint32_t)(epoch >> 32) + 0x7f4a7c15u));
  return o;
}

// Row j of the batch.
MI_DEV int32_t batch_row(const BatchOrder& o, int64_t j, int64_t n, int64_t batch, int shuffle,
                         int half) {
  uint64_t x = o.b * (uint64_t)batch + (uint64_t)j;
  if (x >= (uint64_t)n) {
    x %= (uint64_t)n;   // (a batch position past the data: mi_minibatch_rows rejects it)
  } else if (shuffle) {
    // cycle walking: the orbit of x under the permutation of [0, 2^(2 half)) returns to
    // [0, n) because x itself lies there
    do {
      x = feistel(x, half, o.keys);
    } while (x >= (uint64_t)n);
  }
  return (int32_t)x;
}

}  // namespace mi

// half-width of the Feistel network over at least n values
inline int mi_feistel_half(int64_t n) {
  int bits = 2;
  while (bits < 62 && (1ll << bits) < n) ++bits;
  return (bits + 1) / 2;
}
