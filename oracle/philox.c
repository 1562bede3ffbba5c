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

/*
 * Marsaglia-Tsang gamma draws of csrc/guide.hip (sample_gamma, Stream): the guide's Beta factors
 * (k_beta_rsample: two gamma variates on sub-streams 0 and 1) and Gamma factors (k_gamma_rsample:
 * sub-stream 2). The generator is a stream of Philox-4x32-7 blocks whose counter is
 *   {element, particle, step lo ^ hi, (stream_id << 8) | (sub << 6) | (block & 63)}
 * consumed four words per block; a uniform is u01(word), a normal the first Box-Muller output of
 * two consecutive words (the second is discarded). The device evaluates log/sqrt/cos and powf on
 * the hardware / OCML float routines; this restatement evaluates them in double precision and
 * rounds, and keeps every other operation in float in the device's order (1 + c x as one fused
 * multiply-add, as hipcc contracts it). Accept / reject decisions therefore agree unless a test
 * quantity lands within a few ulp of its threshold, and values agree to a few ulp.
 */
typedef struct {
  uint64_t seed, step;
  uint32_t stream_id, sub;
  uint64_t elem, particle;
  uint32_t block;
  uint32_t bits[4];
  int used;
} gamma_stream;

static uint32_t gs_next(gamma_stream* s) {
  if (s->used == 4) {
    const uint32_t ctr[4] = {(uint32_t)s->elem, (uint32_t)s->particle,
                             (uint32_t)s->step ^ (uint32_t)(s->step >> 32),
                             (s->stream_id << 8) | (s->sub << 6) | (s->block & 63u)};
    oracle_philox4x32(ctr, (uint32_t)s->seed, (uint32_t)(s->seed >> 32), GUIDE_ROUNDS, s->bits);
    ++s->block;
    s->used = 0;
  }
  return s->bits[s->used++];
}

static float gs_uniform(gamma_stream* s) { return u01(gs_next(s)); }

static float gs_normal(gamma_stream* s) {
  const uint32_t a = gs_next(s), b = gs_next(s);
  const double r = sqrt(-2.0 * log((double)u01(a)));
  return (float)(r * cos(2.0 * M_PI * (double)u01(b)));
}

/* One standard gamma draw; *blocks = Philox blocks consumed (1 + rejections show as more). */
static float gs_gamma(float alpha, gamma_stream* s, int32_t* blocks) {
  float boost = 1.0f;
  if (!(alpha > 0.0f)) {
    *blocks = (int32_t)s->block;
    return 0.0f;
  }
  if (alpha < 1.0f) {
    const float inv = 1.0f / alpha;
    boost = (float)pow((double)gs_uniform(s), (double)inv);
    alpha += 1.0f;
  }
  const float d = alpha - 1.0f / 3.0f;
  const float c = 1.0f / sqrtf(9.0f * d);
  for (int attempt = 0; attempt < 64; ++attempt) {
    float x, y;
    int tries = 0;
    do {
      x = gs_normal(s);
      y = fmaf(c, x, 1.0f);
    } while (y <= 0.0f && ++tries < 16);
    if (y <= 0.0f) continue;
    const float v = y * y * y;
    const float u = gs_uniform(s);
    const float xx = x * x;
    if ((double)u < 1.0 - 0.0331 * (double)xx * (double)xx) {
      *blocks = (int32_t)s->block;
      return boost * d * v;
    }
    if (log((double)u) < 0.5 * (double)xx + (double)d * (1.0 - (double)v + log((double)v))) {
      *blocks = (int32_t)s->block;
      return boost * d * v;
    }
  }
  *blocks = (int32_t)s->block;
  return boost * d;
}

/* Standard gamma draws g[k * N + i] of mi_gamma_rsample (sub-stream 2) for concentration[i];
 * blocks[k * N + i] = Philox blocks the draw consumed (may be NULL). */
void oracle_gamma_draws(int64_t K, int64_t N, const float* concentration, uint64_t seed,
                        uint64_t step, uint32_t stream_id, int64_t particle_offset, float* g,
                        int32_t* blocks) {
  for (int64_t k = 0; k < K; ++k)
    for (int64_t i = 0; i < N; ++i) {
      gamma_stream s = {seed, step, stream_id, 2u, (uint64_t)i, (uint64_t)(particle_offset + k),
                        0u, {0u, 0u, 0u, 0u}, 4};
      int32_t used = 0;
      g[k * N + i] = gs_gamma(concentration[i], &s, &used);
      if (blocks) blocks[k * N + i] = used;
    }
}

/* Beta draws x[k * N + i] of mi_beta_rsample for concentrations (c1[i], c0[i]): g1 / (g1 + g0)
 * with g1 on sub-stream 0 and g0 on sub-stream 1; g1, g0 and the blocks each consumed are
 * returned too (any of them may be NULL). */
void oracle_beta_draws(int64_t K, int64_t N, const float* c1, const float* c0, uint64_t seed,
                       uint64_t step, uint32_t stream_id, int64_t particle_offset, float* x,
                       float* g1_out, float* g0_out, int32_t* blocks1, int32_t* blocks0) {
  for (int64_t k = 0; k < K; ++k)
    for (int64_t i = 0; i < N; ++i) {
      const uint64_t p = (uint64_t)(particle_offset + k);
      gamma_stream sa = {seed, step, stream_id, 0u, (uint64_t)i, p, 0u, {0u, 0u, 0u, 0u}, 4};
      gamma_stream sb = {seed, step, stream_id, 1u, (uint64_t)i, p, 0u, {0u, 0u, 0u, 0u}, 4};
      int32_t b1 = 0, b0 = 0;
      const float g1 = gs_gamma(c1[i], &sa, &b1);
      const float g0 = gs_gamma(c0[i], &sb, &b0);
      const float s = g1 + g0;
      const int64_t t = k * N + i;
      x[t] = s > 0.0f ? g1 / s : (c1[i] >= c0[i] ? 1.0f : 0.0f);
      if (g1_out) g1_out[t] = g1;
      if (g0_out) g0_out[t] = g0;
      if (blocks1) blocks1[t] = b1;
      if (blocks0) blocks0[t] = b0;
    }
}
