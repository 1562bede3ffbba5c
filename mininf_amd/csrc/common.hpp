// Device helpers shared by the site and guide kernels (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mininf_amd.h"
#include "device_math.hpp"


namespace mi {


// ---------------------------------------------------------------------------------------------
// Philox-4x32-10 (Salmon, Moraes, Dror, Shaw: "Parallel random numbers: as easy as 1, 2, 3",
// SC'11). Counter-based: the output is a pure function of (counter, key), which is what makes the
// particle draws independent of the grid shape and of how particles are split across GPUs.
// ---------------------------------------------------------------------------------------------
struct U4 {
  uint32_t x, y, z, w;
};

MI_DEV U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int round = 0; round < 10; ++round) {
    const uint32_t lo0 = 0xD2511F53u * c.x;
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Uniform in the open interval (0, 1) from the top 24 bits (exactly representable in fp32).
MI_DEV float u01(uint32_t bits) { return ((float)(bits >> 8) + 0.5f) * 5.9604644775390625e-08f; }

// Two standard normals from two uniforms (Box-Muller).
MI_DEV void box_muller(uint32_t a, uint32_t b, float& n0, float& n1) {
  const float r = sqrtf(-2.0f * logf(u01(a)));
  float s, c;
  sincospif(2.0f * u01(b), &s, &c);
  n0 = r * c;
  n1 = r * s;
}

// Counter layout of the guide generator (see include/mininf_amd.h, mi_normal_rsample):
//   c.x = element quad (i / 4), c.y = global particle, c.z = step (low 32 bits),
//   c.w = (stream_id << 8) | sub-stream, key = seed.
MI_DEV U4 guide_bits(uint64_t seed, uint64_t step, uint32_t stream_id, uint32_t sub, uint64_t quad,
                     uint64_t particle) {
  U4 c{(uint32_t)quad, (uint32_t)particle, (uint32_t)step ^ (uint32_t)(step >> 32),
       (stream_id << 8) | (sub & 0xFFu)};
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// eps for elements 4q .. 4q+3 of particle p.
MI_DEV void guide_normals(uint64_t seed, uint64_t step, uint32_t stream_id, uint64_t quad,
                          uint64_t particle, float out[4]) {
  const U4 b = guide_bits(seed, step, stream_id, 0, quad, particle);
  box_muller(b.x, b.y, out[0], out[1]);
  box_muller(b.z, b.w, out[2], out[3]);
}

}  // namespace mi
