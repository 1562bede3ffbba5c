// Adam arithmetic shared by the one-launch optimizer step (adam.hip) and the launches that finish
// a whole training step themselves (linear.hip lin_finish, sites.hip bcast_finish): restated from
// torch's fused Adam (ATen/native/cuda/fused_adam_utils.cuh adam_math, ADAM_MODE::ORIGINAL, no
// AMSGrad) -- hyper-parameters in double, moments and parameter in float, bias corrections
// 1 - beta^step in double: bit-identical to torch.optim.Adam(fused=True).
#pragma once

#include "common.hpp"

namespace mi {

struct AdamCoef {
  float bc1, bc2_sqrt, step_size;
};

// H: a descriptor with Adam's hyper-parameters (mi_adam, mi_elbo_adam)
template <typename H>
MI_DEV AdamCoef adam_coef(const H& A, float s1) {
  AdamCoef c;
  c.bc1 = (float)(1.0 - pow(A.beta1, (double)s1));
  c.bc2_sqrt = (float)sqrt(1.0 - pow(A.beta2, (double)s1));
  c.step_size = (float)(A.lr / (double)c.bc1);
  return c;
}

template <typename H>
MI_DEV void adam_update(const H& A, const AdamCoef& c, float& param, float grad, float& m,
                        float& v) {
  if (A.maximize) grad = -grad;
  // the contractions spelled out: fma(beta, moment, (1 - beta) * grad [* grad]), the form
  // torch's kernel compiles to (the compiler may pick another when left to itself)
  if (A.weight_decay != 0.0) grad = (float)fma((double)param, A.weight_decay, (double)grad);
  m = (float)fma(A.beta1, (double)m, (1.0 - A.beta1) * (double)grad);
  v = (float)fma(A.beta2, (double)v, ((1.0 - A.beta2) * (double)grad) * (double)grad);
  const float denom = (float)((double)(sqrtf(v) / c.bc2_sqrt) + A.eps);
  param -= c.step_size * m / denom;
}

MI_DEV mi_adam_tensor adam_tensor_at(const mi_adam& A, int t) {
  switch (t) {
#define MI_ADAM_CASE(Q) case Q: return A.tensors[Q];
    MI_ADAM_CASE(1) MI_ADAM_CASE(2) MI_ADAM_CASE(3) MI_ADAM_CASE(4) MI_ADAM_CASE(5)
    MI_ADAM_CASE(6) MI_ADAM_CASE(7)
#undef MI_ADAM_CASE
    default: return A.tensors[0];
  }
}

// The whole step of small tensors in one workgroup (the last block of a step-finishing launch,
// after the gradients are written and a barrier): every element's update, then each tensor's step
// count (every thread has read it by then).
template <int NT>
MI_DEV void adam_block(const mi_adam& A) {
  for (int t = 0; t < A.num; ++t) {
    const mi_adam_tensor T = adam_tensor_at(A, t);
    const float s1 = *T.step + 1.0f;
    const AdamCoef c = adam_coef(A, s1);
    for (int64_t j = threadIdx.x; j < T.numel; j += NT) {
      float p = T.param[j], m = T.exp_avg[j], v = T.exp_avg_sq[j];
      adam_update(A, c, p, T.grad[j], m, v);
      T.param[j] = p;
      T.exp_avg[j] = m;
      T.exp_avg_sq[j] = v;
    }
    __syncthreads();   // every thread has read the step
    if (threadIdx.x == 0) *T.step = s1;
  }
}

// The optimizer step a step-finishing launch may run in its last block: at most this many
// elements in all (a few hundred threads' worth; a larger step keeps its own launch).
constexpr int64_t kFusedAdamMaxNumel = 16384;

// 0: `A` (NULL: none) can run in a finishing launch's last block; MI_EINVAL: malformed;
// MI_EUNSUPPORTED: too large.
inline int fused_adam_check(const mi_adam* A) {
  if (A == nullptr) return 0;
  if (A->num < 1 || A->num > MI_ADAM_MAX_TENSORS) return MI_EINVAL;
  int64_t total = 0;
  for (int t = 0; t < A->num; ++t) {
    const mi_adam_tensor& T = A->tensors[t];
    if (T.param == nullptr || T.grad == nullptr || T.exp_avg == nullptr ||
        T.exp_avg_sq == nullptr || T.step == nullptr || T.numel < 0)
      return MI_EINVAL;
    total += T.numel;
  }
  return total <= kFusedAdamMaxNumel ? 0 : MI_EUNSUPPORTED;
}

}  // namespace mi
