// fp32 digamma / trigamma and the Beta entropy terms of the ELBO tail, shared by the ELBO kernels
// (elbo.hip) and the site launches that finish the ELBO themselves (sites.hip).
#pragma once

#include "common.hpp"

namespace mi {

// fp32 digamma / trigamma for the Beta entropy, evaluated in the guide's dtype as torch does
// (torch.digamma / torch.polygamma(1, .) on float tensors). Recurrence up to x >= 6, then the
// asymptotic series.
MI_DEV float digammaf(float x) {
  float shift = 0.0f;
  while (x < 6.0f) {
    shift -= 1.0f / x;
    x += 1.0f;
  }
  const float r = 1.0f / (x * x);
  const float series = r * (1.0f / 12 - r * (1.0f / 120 - r * (1.0f / 252 - r * (1.0f / 240))));
  return shift + logf(x) - 0.5f / x - series;
}

MI_DEV float trigammaf(float x) {
  float acc = 0.0f;
  while (x < 6.0f) {
    acc += 1.0f / (x * x);
    x += 1.0f;
  }
  const float r = 1.0f / (x * x);
  return acc + 1.0f / x + 0.5f * r +
         r / x * (1.0f / 6 - r * (1.0f / 30 - r * (1.0f / 42 - r * (1.0f / 30))));
}

// Beta(a, b) entropy = Dirichlet([a, b]) (dirichlet.py:122-130 with k = 2, a0 = a + b):
//   lgamma(a) + lgamma(b) - lgamma(a0) - (2 - a0) psi(a0) - (a - 1) psi(a) - (b - 1) psi(b)
// in fp32 terms as torch evaluates them, carried in fp64.
MI_DEV double beta_entropy(float a, float b) {
  const float t = a + b;  // concentration.sum(-1)
  return (double)(lgammaf(a) + lgammaf(b) - lgammaf(t)) -
         (double)((2.0f - t) * digammaf(t)) - (double)((a - 1.0f) * digammaf(a)) -
         (double)((b - 1.0f) * digammaf(b));
}

// dH/da, dH/db: (a0 - 2) psi'(a0) - (a - 1) psi'(a) and the same with b.
MI_DEV void beta_entropy_grad(float a, float b, double& d0, double& d1) {
  const float t = a + b;
  const float tt = (t - 2.0f) * trigammaf(t);
  d0 = (double)(tt - (a - 1.0f) * trigammaf(a));
  d1 = (double)(tt - (b - 1.0f) * trigammaf(b));
}

}  // namespace mi
