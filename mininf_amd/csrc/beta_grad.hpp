// Beta implicit reparameterisation gradient, shared by the guide backward (guide.hip) and the
// ELBO backward with absorbed draws (elbo.hip).
#pragma once

#include "common.hpp"

namespace mi {

// ---- Beta implicit reparameterisation gradient -----------------------------------------------
// Restatement (fp64 throughout) of the piecewise approximation used by torch._dirichlet_grad
// (torch/include/ATen/native/Distributions.h, dirichlet_grad_one and helpers): the derivative of the
// Beta(alpha, total - alpha) draw x with respect to alpha, -(d/dalpha CDF) / pdf, divided by
// (1 - x). Four regimes: x near 0 (Taylor series), x near 1 (series for the mirrored variable),
// both shapes large (Rice saddle-point expansion), otherwise a fitted rational correction of the
// analytic approximation x (psi(total) - psi(alpha)) / beta.
// psi_a = digamma(a), psi_ab = digamma(a + b): parameter-only, hoisted out of the particle loop.
MI_DEV double beta_grad_small_alpha(double x, double a, double b, double psi_a, double psi_ab) {
  const double factor = psi_a - psi_ab - log(x);
  double coeff = 1.0;
  const double ra = 1.0 / a;
  double series = ra * (factor + ra);
  // one division per term: 1/n folds to a constant once unrolled
#pragma unroll
  for (int n = 1; n <= 10; ++n) {
    coeff *= (n - b) * x * (1.0 / n);
    const double rd = 1.0 / (a + n);
    series += coeff * rd * (factor + rd);
  }
  const double r = x * exp(-b * log1p(-x)) * series;   // (1 - x)^-b
  return r != r ? 0.0 : r;
}

// psi_ab = digamma(a + b), psi_b = digamma(b).
MI_DEV double beta_grad_small_beta(double x, double a, double b, double psi_ab, double psi_b) {
  const double factor = psi_ab - psi_b;
  double coeff = 1.0, prod = 1.0, dprod = 0.0, series = factor / a;
#pragma unroll
  for (int n = 1; n <= 8; ++n) {
    coeff *= -x * (1.0 / n);
    dprod = dprod * (b - n) + prod;
    prod *= (b - n);
    series += coeff / (a + n) * (dprod + factor * prod);
  }
  const double r = -exp((1.0 - b) * log1p(-x)) * series;   // (1 - x)^(1 - b)
  return r != r ? 0.0 : r;
}

MI_DEV double beta_grad_mid(double x, double a, double b) {
  const double t = a + b;
  const double mean = a / t;
  const double sd = sqrt(a * b / (t + 1.0)) / t;
  if (mean - 0.1 * sd <= x && x <= mean + 0.1 * sd) {
    const double b2 = b * b;
    const double poly = 47 * x * b2 * b2 +
        a * ((43 + 20 * (16 + 27 * b) * x) * b2 * b +
             a * (3 * (59 + 180 * b - 90 * x) * b2 +
                  a * ((453 + 1620 * b * (1 - x) - 455 * x) * b + a * (8 * (1 - x) * (135 * b - 11)))));
    const double pre_num = (1 + 12 * a) * (1 + 12 * b) / (t * t);
    const double pre_den = 12960 * a * a * a * b * b * (1 + 12 * t);
    return pre_num / (1 - x) * poly / pre_den;
  }
  const double prefactor = -x / sqrt(2 * a * b / t);
  const double stirling = (1 + 1 / (12 * a) + 1 / (288 * a * a)) *
                          (1 + 1 / (12 * b) + 1 / (288 * b * b)) /
                          (1 + 1 / (12 * t) + 1 / (288 * t * t));
  const double axbx = a * (x - 1) + b * x;
  const double term1 = (2 * a * a * (x - 1) + a * b * (x - 1) - x * b * b) /
                       (sqrt(2 * a / b) * pow(t, 1.5) * axbx * axbx);
  const double term2 = 0.5 * log(a / (t * x));
  const double term3 = sqrt(8 * a * b / t) / (b * x + a * (x - 1));
  const double term4 = pow(b * log(b / (t * (1 - x))) + a * log(a / (t * x)), -1.5);
  return stirling * prefactor * (term1 + term2 * (term3 + (x < mean ? term4 : -term4)));
}

// Fitted coefficients of the rational correction (numerator [0] and denominator [1] as
// polynomials in u = log x, a = log(alpha) - u, b = log(total) - a); values as published in
// torch's Distributions.h.
static __constant__ double kBetaGradCoef[2][3][3][4] = {
    {{{1.003668233, -0.01061107488, -0.0657888334, 0.01201642863},
      {0.6336835991, -0.3557432599, 0.05486251648, -0.001465281033},
      {-0.03276231906, 0.004474107445, 0.002429354597, -0.0001557569013}},
     {{0.221950385, -0.3187676331, 0.01799915743, 0.01074823814},
      {-0.2951249643, 0.06219954479, 0.01535556598, 0.001550077057},
      {0.02155310298, 0.004170831599, 0.001292462449, 6.976601077e-05}},
     {{-0.05980841433, 0.008441916499, 0.01085618172, 0.002319392565},
      {0.02911413504, 0.01400243777, -0.002721828457, 0.000751041181},
      {0.005900514878, -0.001936558688, -9.495446725e-06, 5.385558597e-05}}},
    {{{1, -0.02924021934, -0.04438342661, 0.007285809825},
      {0.6357567472, -0.3473456711, 0.05454656494, -0.002407477521},
      {-0.03301322327, 0.004845219414, 0.00231480583, -0.0002307248149}},
     {{0.5925320577, -0.1757678135, 0.01505928619, 0.000564515273},
      {0.1014815858, -0.06589186703, 0.01272886114, -0.0007316646956},
      {-0.007258481865, 0.001096195486, 0.0003934994223, -4.12701925e-05}},
     {{0.06469649321, -0.0236701437, 0.002902096474, -5.896963079e-05},
      {0.001925008108, -0.002869809258, 0.0008000589141, -6.063713228e-05},
      {-0.0003477407336, 6.959756487e-05, 1.097287507e-05, -1.650964693e-06}}}};

// Every regime needs only digamma(alpha) and digamma(total) of the parameters, which the caller
// evaluates once per element rather than once per particle.
MI_DEV double dirichlet_grad(double x, double alpha, double total, double psi_alpha,
                             double psi_total) {
  const double beta = total - alpha;
  const double boundary = total * x * (1.0 - x);
  if (x <= 0.5 && boundary < 2.5) return beta_grad_small_alpha(x, alpha, beta, psi_alpha, psi_total);
  if (x >= 0.5 && boundary < 0.75)
    return -beta_grad_small_beta(1.0 - x, beta, alpha, psi_total, psi_alpha);
  if (alpha > 6.0 && beta > 6.0) return beta_grad_mid(x, alpha, beta);
  const double u = log(x);
  const double a = log(alpha) - u;
  const double b = log(total) - a;
  const double pu[3] = {1.0, u, u * u};
  const double pa[3] = {1.0, a, a * a};
  double num = 0.0, den = 0.0;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double w = pu[r] * pa[c];
      const double* n = kBetaGradCoef[0][r][c];
      const double* d = kBetaGradCoef[1][r][c];
      num += w * (n[0] + b * (n[1] + b * (n[2] + b * n[3])));
      den += w * (d[0] + b * (d[1] + b * (d[2] + b * d[3])));
    }
  }
  const double analytic = x * (psi_total - psi_alpha) / beta;
  return num / den * analytic;
}

// ---- Gamma implicit reparameterisation gradient ----------------------------------------------
// d x / d alpha of a standard Gamma(alpha) draw x, restating torch._standard_gamma_grad
// (torch/include/ATen/native/Distributions.h:310, standard_gamma_grad_one) with the CPU
// accumulation type (double), which is what the reference evaluates: a Taylor series of the CDF
// for x < 0.8, the Rice saddle-point expansion for alpha > 8, a bivariate rational fit otherwise.
MI_DEV double standard_gamma_grad(double alpha, double x) {
  if (x < (double)0.8f) {   // the source compares against float literals
    double numer = 1.0, denom = alpha;
    double series1 = numer / denom, series2 = numer / (denom * denom);
#pragma unroll
    for (int i = 1; i <= 5; ++i) {
      numer *= -x / (double)i;
      denom += 1.0;
      series1 += numer / denom;
      series2 += numer / (denom * denom);
    }
    const double pow_x_alpha = pow(x, alpha);
    const double gamma_pdf = pow(x, alpha - 1.0) * exp(-x);
    const double gamma_cdf = pow_x_alpha * series1;
    const double gamma_cdf_alpha = (log(x) - digamma(alpha)) * gamma_cdf - pow_x_alpha * series2;
    const double result = -gamma_cdf_alpha / gamma_pdf;
    return result != result ? 0.0 : result;
  }
  if (alpha > 8.0) {
    if ((double)0.9f * alpha <= x && x <= (double)1.1f * alpha) {
      const double numer_1 = 1.0 + 24.0 * alpha * (1.0 + 12.0 * alpha);
      const double numer_2 = 1440.0 * (alpha * alpha) + 6.0 * x * (53.0 - 120.0 * x) -
                             65.0 * x * x / alpha + alpha * (107.0 + 3600.0 * x);
      const double denom = 1244160.0 * (alpha * alpha) * (alpha * alpha);
      return numer_1 * numer_2 / denom;
    }
    const double denom = sqrt(8.0 * alpha);
    const double term2 = denom / (alpha - x);
    const double term3 = pow(x - alpha - alpha * log(x / alpha), -1.5);
    const double term23 = (x < alpha) ? term2 - term3 : term2 + term3;
    const double term1 = log(x / alpha) * term23 -
                         sqrt(2.0 / alpha) * (alpha + x) / ((alpha - x) * (alpha - x));
    const double stirling = 1.0 + 1.0 / (12.0 * alpha) * (1.0 + 1.0 / (24.0 * alpha));
    const double numer = x * term1;
    return -stirling * numer / denom;
  }
  const double u = log(x / alpha);
  const double v = log(alpha);
  // the fitted coefficients of the cited source (double literals there)
  constexpr double kCoef[3][8] = {
      {0.16009398, -0.094634809, 0.025146376, -0.0030648343, 1, 0.32668115, 0.10406089,
       0.0014179084},
      {0.53487893, 0.1298071, 0.065735949, -0.0015649758, 0.16639465, 0.020070113,
       -0.0035938915, -0.00058392623},
      {0.040121004, -0.0065914022, -0.0026286047, -0.0013441777, 0.017050642, -0.0021309326,
       0.00085092367, -1.5247877e-07},
  };
  double c[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = kCoef[0][i] + u * (kCoef[1][i] + u * kCoef[2][i]);
  const double p = c[0] + v * (c[1] + v * (c[2] + v * c[3]));
  const double q = c[4] + v * (c[5] + v * (c[6] + v * c[7]));
  return exp(p / q);
}

}  // namespace mi
