/*
 * oracle/philox.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the guide generator of mininf_amd (csrc/device_math.hpp): Philox-4x32-7
 * (Salmon, Moraes, Dror, Shaw, SC'11) and the Box-Muller transform on 24-bit uniforms, with the
 * counter layout documented in include/mininf_amd.h (mi_normal_rsample). Built by oracle/build.py
 * with gcc into oracle/liboracle.so and used by the tests to pin the device generator bit-exactly
 * (integers) and to within float rounding (normals).
 */
#include <math.h>
#include <stdint.h>

static void round_fn(uint32_t c[4], uint32_t k0, uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
  c[0] = n0;
  c[1] = lo1;
  c[2] = n2;
  c[3] = lo0;
}

/* Philox-4x32 with `rounds` rounds (10: the published known-answer vectors; 7: the guide
 * generator, GUIDE_ROUNDS, device_math.hpp kGuideRounds). */
void oracle_philox4x32(const uint32_t ctr[4], uint32_t k0, uint32_t k1, int rounds,
                       uint32_t out[4]) {
  uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
  for (int r = 0; r < rounds; ++r) {
    round_fn(c, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c[0];
  out[1] = c[1];
  out[2] = c[2];
  out[3] = c[3];
}

void oracle_philox4x32_10(const uint32_t ctr[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
  oracle_philox4x32(ctr, k0, k1, 10, out);
}

enum { GUIDE_ROUNDS = 7 };

static float u01(uint32_t bits) { return ((float)(bits >> 8) + 0.5f) * 5.9604644775390625e-08f; }

/* eps[k * N + i] for k in [0, K), i in [0, N): the standard normals of mi_normal_rsample. */
void oracle_guide_normals(int64_t K, int64_t N, uint64_t seed, uint64_t step, uint32_t stream_id,
                          int64_t particle_offset, float* out) {
  for (int64_t k = 0; k < K; ++k) {
    for (int64_t q = 0; 4 * q < N; ++q) {
      const uint32_t ctr[4] = {(uint32_t)q, (uint32_t)(particle_offset + k),
                               (uint32_t)step ^ (uint32_t)(step >> 32), stream_id << 8};
      uint32_t b[4];
      oracle_philox4x32(ctr, (uint32_t)seed, (uint32_t)(seed >> 32), GUIDE_ROUNDS, b);
      float n[4];
      for (int j = 0; j < 2; ++j) {
        const double r = sqrt(-2.0 * log((double)u01(b[2 * j])));
        const double t = 2.0 * M_PI * (double)u01(b[2 * j + 1]);
        n[2 * j] = (float)(r * cos(t));
        n[2 * j + 1] = (float)(r * sin(t));
      }
      for (int j = 0; j < 4 && 4 * q + j < N; ++j) out[k * N + 4 * q + j] = n[j];
    }
  }
}
