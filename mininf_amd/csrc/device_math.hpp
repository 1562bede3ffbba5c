// Device math shared by the precompiled kernels (sites.hip) and the site programs specialised at
// trace time with hiprtc (jit.cpp embeds this file verbatim): family log-densities and their
// derivatives, special functions, wavefront reductions. No includes beyond mininf_amd.h so that it
// compiles both under hipcc (after hip_runtime.h) and under hiprtc.
#pragma once

#include "mininf_amd.h"

#define MI_DEV __device__ __forceinline__

namespace mi {

constexpr int kWave = 64;
constexpr float kHalfLog2Pi = 0.91893853320467274178f;   // log(sqrt(2*pi)), normal.py:103
constexpr float kFloatEps = 1.1920928955078125e-07f;    // torch.finfo(float32).eps, utils.py:101

// ---------------------------------------------------------------------------------------------
// Special functions (fp64).
// ---------------------------------------------------------------------------------------------
MI_DEV double digamma(double x) {
  // Recurrence up to x >= 6, then the asymptotic (Bernoulli-number) series.
  double shift = 0.0;
  if (x <= 0.0 && x == floor(x)) return __builtin_inf();
  if (x < 0.0) {
    // Reflection: psi(1 - x) - psi(x) = pi * cot(pi * x).
    shift = -3.14159265358979323846 / tan(3.14159265358979323846 * x);
    x = 1.0 - x;
  }
  while (x < 6.0) {
    shift -= 1.0 / x;
    x += 1.0;
  }
  const double r = 1.0 / (x * x);
  const double series =
      r * (1.0 / 12 - r * (1.0 / 120 - r * (1.0 / 252 - r * (1.0 / 240 - r * (1.0 / 132)))));
  return shift + log(x) - 0.5 / x - series;
}

// ---------------------------------------------------------------------------------------------
// Philox-4x32-R (Salmon, Moraes, Dror, Shaw: "Parallel random numbers: as easy as 1, 2, 3",
// SC'11). Counter-based: the output is a pure function of (counter, key), which is what makes the
// particle draws independent of the grid shape and of how particles are split across GPUs.
// ---------------------------------------------------------------------------------------------
struct U4 {
  uint32_t x, y, z, w;
};

template <int ROUNDS>
MI_DEV U4 philox4x32(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int round = 0; round < ROUNDS; ++round) {
    // one 32x32->64 multiply per word (v_mad_u64_u32) instead of separate low / high halves
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// The 10-round generator of the published known-answer vectors (mi_philox4x32).
MI_DEV U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) { return philox4x32<10>(c, k0, k1); }

// Rounds of the guide generator. Philox-4x32-7 passes TestU01's BigCrush (Salmon et al., table 2:
// 7 rounds is the smallest Crush-resistant count; 10 is their default safety margin). The
// fused-draw site programs spend ~1/4 of their VALU cycles here (v_mad_u64_u32 issues at ~3x an
// FMA), so the guide uses 7; oracle/philox.c restates the same count.
constexpr int kGuideRounds = 7;

// Uniform in the open interval (0, 1) from the top 24 bits: ((bits >> 8) + 0.5) * 2^-24 as one FMA
// (the same single rounding of the same exact value, scaled by a power of two).
MI_DEV float u01(uint32_t bits) {
  return fmaf((float)(bits >> 8), 5.9604644775390625e-08f, 2.98023223876953125e-08f);
}

// Two standard normals from two uniforms (Box-Muller) on the hardware transcendentals:
// v_log_f32 (log2), v_sqrt_f32 and v_sin_f32 / v_cos_f32, which take their argument in
// revolutions (sin(2 pi u) for u in (0, 1), no range reduction needed). Each is accurate to a few
// ulp; the oracle (oracle/philox.c) restates the same transform in double precision.
MI_DEV void box_muller(uint32_t a, uint32_t b, float& n0, float& n1) {
  const float r = __builtin_amdgcn_sqrtf(-1.38629436111989061883f * __builtin_amdgcn_logf(u01(a)));
  const float t = u01(b);
  n0 = r * __builtin_amdgcn_cosf(t);
  n1 = r * __builtin_amdgcn_sinf(t);
}

// Counter layout of the guide generator (see include/mininf_amd.h, mi_normal_rsample):
//   c.x = element quad (i / 4), c.y = global particle, c.z = step (low 32 bits),
//   c.w = (stream_id << 8) | sub-stream, key = seed.
MI_DEV U4 guide_bits(uint64_t seed, uint64_t step, uint32_t stream_id, uint32_t sub, uint64_t quad,
                     uint64_t particle) {
  U4 c{(uint32_t)quad, (uint32_t)particle, (uint32_t)step ^ (uint32_t)(step >> 32),
       (stream_id << 8) | (sub & 0xFFu)};
  return philox4x32<kGuideRounds>(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// eps for elements 4q .. 4q+3 of particle p.
MI_DEV void guide_normals(uint64_t seed, uint64_t step, uint32_t stream_id, uint64_t quad,
                          uint64_t particle, float out[4]) {
  const U4 b = guide_bits(seed, step, stream_id, 0, quad, particle);
  box_muller(b.x, b.y, out[0], out[1]);
  box_muller(b.z, b.w, out[2], out[3]);
}

// x if keep, else +0, through a bit mask the compiler cannot see through: "keep ? load : 0" is
// otherwise turned back into a branch around the load, with a wait for it at the join -- a chain
// of such loads then costs one memory round trip each instead of one for all.
MI_DEV float keep_if(float x, bool keep) {
  uint32_t m = keep ? 0xffffffffu : 0u;
  asm volatile("" : "+v"(m));
  return __uint_as_float(__float_as_uint(x) & m);
}

MI_DEV double keep_if_d(double x, bool keep) {
  uint32_t m = keep ? 0xffffffffu : 0u;
  asm volatile("" : "+v"(m));
  const uint64_t u = (uint64_t)__double_as_longlong(x) & (((uint64_t)m << 32) | m);
  return __longlong_as_double((long long)u);
}

// ---------------------------------------------------------------------------------------------
// Wavefront reductions.
// ---------------------------------------------------------------------------------------------
MI_DEV float wave_sum(float v) {
#pragma unroll
  for (int offset = 32; offset > 0; offset >>= 1) v += __shfl_xor(v, offset, kWave);
  return v;
}

MI_DEV double wave_sum(double v) {
#pragma unroll
  for (int offset = 32; offset > 0; offset >>= 1) v += __shfl_xor(v, offset, kWave);
  return v;
}

// Progress-balanced wave priority for loops whose waves share SIMDs for their whole length: one
// s_setprio level less per quarter of the loop (step `i` of `n`), so the arbiter (priority, then
// age) lets the waves behind catch up and a SIMD's waves finish together rather than the oldest
// first -- a wave left issuing alone runs at half the VALU rate.
MI_DEV void balance_priority(long i, long n) {
  const long q = (4 * i) / n;
  if (i != 0 && q == (4 * (i - 1)) / n) return;
  if (q == 0) __builtin_amdgcn_s_setprio(3);
  else if (q == 1) __builtin_amdgcn_s_setprio(2);
  else if (q == 2) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}

// Orders a wave's LDS accesses (lanes exchanging values through LDS): a wave's LDS operations
// execute in issue order, so only the compiler has to be kept from moving them across this point.
MI_DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Row sums of a wave's [T][65] LDS tile (row p: the 64 lanes' values for particle p; the odd
// stride keeps the column reads on distinct banks). Lane T * q + p adds columns [q T, q T + T) of
// row p, then the 64 / T partial sums of a row meet in a shuffle tree; lane p < T returns row p.
template <int T>
MI_DEV float tile_row_sums(const float* tile, int lane) {
  const int p = lane & (T - 1), q = lane / T;
  const float* row = tile + p * 65 + q * T;
  float s = 0.0f;
#pragma unroll
  for (int j = 0; j < T; ++j) s += row[j];
#pragma unroll
  for (int offset = T; offset < kWave; offset <<= 1) s += __shfl_xor(s, offset, kWave);
  return s;
}

// Sum over lanes that differ only in bits >= log2(width) (lanes sharing lane % width).
MI_DEV float wave_sum_strided(float v, int width) {
  for (int offset = 32; offset >= width; offset >>= 1) v += __shfl_xor(v, offset, kWave);
  return v;
}

// A uniform value pinned to a scalar register at this point of the program (an empty asm): its load
// cannot be sunk to a later use, nor a select over several such values turned back into an indexed
// load of the argument segment.
template <typename V>
MI_DEV V pin(V v) {
  asm("" : "+s"(v));
  return v;
}
// Kernel-argument prefetch: one vector load touches every 64-byte line of the first BYTES of the
// argument segment (lane l reads a dword of line l), so the segment is in the L2 after one memory
// round trip. The descriptor-driven kernels read their arguments through the scalar cache in
// dependent chains (a job index from one field selects the next fields); each miss there cost a
// memory round trip at the start of every workgroup (k_elbo_forward's reducing blocks: 2.4-3 us
// from entry to their first data load, tools/elbo_timing.py), an L2 hit a fraction of one. (Scalar
// loads of every line would need one wait per 15: the counter's limit.)
template <int BYTES>
MI_DEV void kernarg_prefetch() {
  static_assert(BYTES > 0 && BYTES <= 64 * 64, "argument segment");
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t base = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr());
  const int lane = (int)(threadIdx.x & 63);
  if (threadIdx.x < 64 && lane * 64 < BYTES) {
    typedef const __attribute__((address_space(1))) uint32_t gword;
    const uint32_t x = *(gword*)(base + (uint64_t)lane * 64);
    asm volatile("" : : "v"(x));
  }
#endif
}

// Kernel span stamps (bench.py's timing of a replayed kernel): every workgroup of a launch folds
// its start and end times on the device's constant-rate clock (s_memrealtime, 100 MHz) into
// stamps[0] (minimum) and stamps[1] (maximum), so the launch's span is stamps[1] - stamps[0] --
// first workgroup start to last workgroup end, inside the replayed step. stamps == NULL: nothing
// (one uniform branch per workgroup). span_end is reached by every thread of the workgroup.
MI_DEV unsigned long long span_begin(const unsigned long long* stamps) {
  return stamps != nullptr ? __builtin_amdgcn_s_memrealtime() : 0ull;
}

MI_DEV void span_end(unsigned long long* stamps, unsigned long long t0) {
  if (stamps == nullptr) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    __hip_atomic_fetch_min(stamps, t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_max(stamps + 1, t1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// OR-combine per-lane flag words across the wave and publish them with one atomic; must be called
// with every lane of the wave active.
MI_DEV void publish_flags(uint32_t* flags, uint32_t mine) {
#pragma unroll
  for (int offset = 32; offset > 0; offset >>= 1) mine |= __shfl_xor(mine, offset, kWave);
  if (mine != 0u && (threadIdx.x & (kWave - 1)) == 0) atomicOr(flags, mine);
}

// ---------------------------------------------------------------------------------------------
// Hardware transcendentals (fp32).
// ---------------------------------------------------------------------------------------------
MI_DEV float rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// exp(x) = 2^(x log2 e) on v_exp_f32; results below FLT_MIN flush to zero, which only drops terms
// smaller than every sum they enter.
MI_DEV float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896341f); }

// log1p(t), t in [0, 1], from u = fl(1 + t) and ru = 1 / u (which the Bernoulli caller needs for
// the sigmoid anyway): log(u) plus the first-order correction (t - (u - 1)) / u for the rounding
// of u (u - 1 is exact for u in [1, 2]); v_log_f32 is log2. For t below half an ulp of 1, u = 1
// and the result is t.
MI_DEV float log1p_unit(float t, float u, float ru) {
  return fmaf(t - (u - 1.0f), ru, __builtin_amdgcn_logf(u) * 0.69314718055994531f);
}

// -------------------------------------------------------------------------------------------------
// Per-element family math.  d[r] = d log p / d role_r.
// -------------------------------------------------------------------------------------------------
struct Elem {
  float lp;
  float d[3];
  uint32_t param_bad;
  uint32_t support_bad;
};

// Normal(loc, scale): -(v-loc)^2 / (2 scale^2) - log(scale) - log(sqrt(2 pi))
// torch/distributions/normal.py:88-103; support real (constraints.py: `value == value`).
MI_DEV void eval_normal(float loc, float scale, float v, Elem& e) {
  // in terms of diff = v - loc: -diff^2 / (2 sigma^2) - log sigma - log sqrt(2 pi), and
  // d/dloc = diff / sigma^2 -- with a constant scale, (-0.5 / sigma^2) and 1 / sigma^2 are loop
  // invariants and an element costs four instructions
  const float inv = rcp(scale);
  const float inv2 = inv * inv;
  const float diff = v - loc;
  e.lp = fmaf((-0.5f * inv2) * diff, diff, -(logf(scale) + kHalfLog2Pi));
  const float g = diff * inv2;
  e.d[0] = g;
  e.d[1] = fmaf(diff, g, -1.0f) * inv;   // (z^2 - 1) / sigma, z = diff / sigma
  e.d[2] = -g;
  e.param_bad = !(scale > 0.0f) || (loc != loc);
  e.support_bad = (v != v);
}

// Bernoulli(logits): -BCE_with_logits(l, v) = -(max(l, 0) - l v + log1p(exp(-|l|)))
// torch/distributions/bernoulli.py:121-125; support boolean {0, 1} (constraints.py:317-325).
// The streaming site programs evaluate this per (particle, element), so it is written with the
// hardware transcendentals (v_exp_f32 / v_log_f32 / v_rcp_f32, ~1 ulp each) instead of libm's
// correctly-rounded-ish expf/log1pf/division sequences (~100 VALU ops per element on gfx950):
// log1p(t) for t in [0, 1] is log(u) corrected for the rounding of u = 1 + t (log1p_unit).
MI_DEV void eval_bernoulli_logits(float l, float v, Elem& e) {
  const float t = fast_exp(-fabsf(l));
  const float u = 1.0f + t;
  const float r = rcp(u);
  e.lp = -(fmaxf(l, 0.0f) - l * v + log1p_unit(t, u, r));
  const float sig = l >= 0.0f ? r : t * r;
  e.d[0] = v - sig;
  e.d[1] = 0.0f;
  e.d[2] = l;
  e.param_bad = (l != l);
  e.support_bad = !(v == 0.0f || v == 1.0f);
}

// ---- packed pairs ---------------------------------------------------------------------------
// The same Normal / Bernoulli-logits arithmetic on two elements at once, written on two-wide float
// vectors so that the adds, multiplies and FMAs issue as v_pk_add_f32 / v_pk_mul_f32 /
// v_pk_fma_f32 (two fp32 lanes per instruction on CDNA4, the same IEEE rounding per element as the
// scalar forms above); compares, selects and transcendentals stay per element. The fused-draw site
// programs use them for their element pairs (jit.cpp, "packed").
typedef float f2 __attribute__((ext_vector_type(2)));

MI_DEV f2 splat2(float a) { return f2{a, a}; }
MI_DEV f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

struct Elem2 {
  f2 lp;
  f2 d[3];
  bool param_bad;        // either element
  bool support_bad[2];
};

// guide_normals for one quad as two pairs (elements 0-1 and 2-3): the uniforms' scale-and-offset,
// the radius' multiply and the final products on packed instructions; per element the same
// operations as box_muller, so the values are bit-identical.
MI_DEV void guide_normals2(uint64_t seed, uint64_t step, uint32_t stream_id, uint64_t quad,
                           uint64_t particle, f2& n01, f2& n23) {
  const U4 b = guide_bits(seed, step, stream_id, 0, quad, particle);
  const f2 ua = fma2(f2{(float)(b.x >> 8), (float)(b.z >> 8)}, splat2(5.9604644775390625e-08f),
                     splat2(2.98023223876953125e-08f));
  const f2 ut = fma2(f2{(float)(b.y >> 8), (float)(b.w >> 8)}, splat2(5.9604644775390625e-08f),
                     splat2(2.98023223876953125e-08f));
  const f2 l = -1.38629436111989061883f * f2{__builtin_amdgcn_logf(ua.x), __builtin_amdgcn_logf(ua.y)};
  const f2 r = f2{__builtin_amdgcn_sqrtf(l.x), __builtin_amdgcn_sqrtf(l.y)};
  n01 = splat2(r.x) * f2{__builtin_amdgcn_cosf(ut.x), __builtin_amdgcn_sinf(ut.x)};
  n23 = splat2(r.y) * f2{__builtin_amdgcn_cosf(ut.y), __builtin_amdgcn_sinf(ut.y)};
}

MI_DEV void eval_normal2(f2 loc, f2 scale, f2 v, Elem2& e) {
  const f2 inv = f2{rcp(scale.x), rcp(scale.y)};
  const f2 inv2 = inv * inv;
  const f2 diff = v - loc;
  const f2 c = -(f2{logf(scale.x), logf(scale.y)} + kHalfLog2Pi);
  e.lp = fma2((-0.5f * inv2) * diff, diff, c);
  const f2 g = diff * inv2;
  e.d[0] = g;
  e.d[1] = fma2(diff, g, splat2(-1.0f)) * inv;
  e.d[2] = -g;
  // bitwise, not short-circuit, combinations: lane masks the compiler keeps in SGPR pairs
  e.param_bad = !(scale.x > 0.0f) | (loc.x != loc.x) | !(scale.y > 0.0f) | (loc.y != loc.y);
  e.support_bad[0] = (v.x != v.x);
  e.support_bad[1] = (v.y != v.y);
}

MI_DEV void eval_bernoulli_logits2(f2 l, f2 v, Elem2& e) {
  const f2 t = f2{fast_exp(-fabsf(l.x)), fast_exp(-fabsf(l.y))};
  const f2 u = 1.0f + t;
  const f2 r = f2{rcp(u.x), rcp(u.y)};
  // log1p_unit per element: fma(t - (u - 1), r, log(u) * ln 2)
  const f2 lu = f2{__builtin_amdgcn_logf(u.x), __builtin_amdgcn_logf(u.y)} * 0.69314718055994531f;
  const f2 l1p = fma2(t - (u - 1.0f), r, lu);
  const f2 mx = f2{fmaxf(l.x, 0.0f), fmaxf(l.y, 0.0f)};
  e.lp = -(mx - l * v + l1p);
  const f2 tr = t * r;
  const f2 sig = f2{l.x >= 0.0f ? r.x : tr.x, l.y >= 0.0f ? r.y : tr.y};
  e.d[0] = v - sig;
  e.d[1] = splat2(0.0f);
  e.d[2] = l;
  e.param_bad = (l.x != l.x) | (l.y != l.y);
  e.support_bad[0] = !((v.x == 0.0f) | (v.x == 1.0f));
  e.support_bad[1] = !((v.y == 0.0f) | (v.y == 1.0f));
}

// Bernoulli(probs): logits = log(p_c) - log1p(-p_c), p_c = clamp(p, eps, 1 - eps)
// (bernoulli.py:104-106 -> utils.py probs_to_logits / clamp_probs); clamp passes the gradient
// only inside [eps, 1 - eps].
MI_DEV void bernoulli_probs_to_logits(float p, float& l, float& dl_dp) {
  const float hi = 1.0f - kFloatEps;
  const float pc = fminf(fmaxf(p, kFloatEps), hi);
  l = logf(pc) - log1pf(-pc);
  dl_dp = (p >= kFloatEps && p <= hi) ? (1.0f / pc + 1.0f / (1.0f - pc)) : 0.0f;
}

MI_DEV void eval_bernoulli_probs(float p, float v, Elem& e) {
  float l, dl_dp;
  bernoulli_probs_to_logits(p, l, dl_dp);
  eval_bernoulli_logits(l, v, e);
  e.d[0] *= dl_dp;
  e.param_bad = !(p >= 0.0f && p <= 1.0f);
}

MI_DEV float xlogy(float x, float y) { return (y != y) ? y : (x == 0.0f ? 0.0f : x * logf(y)); }

// Beta(c1, c0) = Dirichlet([c1, c0]) at [v, 1 - v]:
//   xlogy(c1 - 1, v) + xlogy(c0 - 1, 1 - v) + lgamma(c1 + c0) - lgamma(c1) - lgamma(c0)
// torch/distributions/beta.py:88-92 -> dirichlet.py:90-97; support [0, 1] (unit_interval).
MI_DEV void eval_beta(float a, float b, float v, Elem& e) {
  const float w = 1.0f - v;
  e.lp = xlogy(a - 1.0f, v) + xlogy(b - 1.0f, w) + lgammaf(a + b) - lgammaf(a) - lgammaf(b);
  const double psi_ab = digamma((double)a + (double)b);
  e.d[0] = logf(v) + (float)(psi_ab - digamma((double)a));
  e.d[1] = logf(w) + (float)(psi_ab - digamma((double)b));
  e.d[2] = (a - 1.0f) / v - (b - 1.0f) / w;
  e.param_bad = !(a > 0.0f) || !(b > 0.0f);
  e.support_bad = !(v >= 0.0f && v <= 1.0f);
}

// Gamma(a, r): xlogy(a, r) + xlogy(a - 1, v) - r v - lgamma(a)
// torch/distributions/gamma.py:90-99; support positive (v > 0), a > 0 and r > 0 (arg_constraints).
MI_DEV void eval_gamma(float a, float r, float v, Elem& e) {
  e.lp = xlogy(a, r) + xlogy(a - 1.0f, v) - r * v - lgammaf(a);
  e.d[0] = logf(r) + logf(v) - (float)digamma((double)a);
  e.d[1] = a / r - v;
  e.d[2] = (a - 1.0f) / v - r;
  e.param_bad = !(a > 0.0f) || !(r > 0.0f);
  e.support_bad = !(v > 0.0f);
}

// Poisson(rate): xlogy(v, rate) - rate - lgamma(v + 1)
// torch/distributions/poisson.py:60-65; support nonnegative integers, rate >= 0. d/dv is torch's
// continuous derivative (log rate - digamma(v + 1)).
MI_DEV void eval_poisson(float rate, float v, Elem& e) {
  e.lp = xlogy(v, rate) - rate - lgammaf(v + 1.0f);
  e.d[0] = v / rate - 1.0f;
  e.d[1] = 0.0f;
  e.d[2] = logf(rate) - (float)digamma((double)v + 1.0);
  e.param_bad = !(rate >= 0.0f);
  e.support_bad = !(v >= 0.0f && v == floorf(v));
}

// InverseGamma(a, r) = Gamma(a, r) pushed through y = x^-1 (mininf/distributions.py:5-11):
// TransformedDistribution.log_prob (transformed_distribution.py) with x = y^-1 and
// PowerTransform.log_abs_det_jacobian = log|-y / x| (transforms.py):
//   Gamma.log_prob(x) - log|-y / x|;  support positive.
MI_DEV void eval_inverse_gamma(float a, float r, float y, Elem& e) {
  const float x = 1.0f / y;
  Elem g;
  eval_gamma(a, r, x, g);
  e.lp = g.lp - logf(fabsf(-y / x));
  e.d[0] = g.d[0];
  e.d[1] = g.d[1];
  e.d[2] = g.d[2] * (-x * x) - 2.0f / y;   // dx/dy = -x^2; d log(y / x) / dy = 2 / y
  e.param_bad = g.param_bad;
  e.support_bad = !(y > 0.0f);
}

MI_DEV void eval_family(int family, float r0, float r1, float r2, Elem& e) {
  switch (family) {
    case MI_NORMAL: eval_normal(r0, r1, r2, e); break;
    case MI_BERNOULLI_LOGITS: eval_bernoulli_logits(r0, r2, e); break;
    case MI_BERNOULLI_PROBS: eval_bernoulli_probs(r0, r2, e); break;
    case MI_GAMMA: eval_gamma(r0, r1, r2, e); break;
    case MI_POISSON: eval_poisson(r0, r2, e); break;
    case MI_INVERSE_GAMMA: eval_inverse_gamma(r0, r1, r2, e); break;
    default: eval_beta(r0, r1, r2, e); break;
  }
}

}  // namespace mi
