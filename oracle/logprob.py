"""
Per-family log densities and their derivatives in numpy float64 (test infrastructure only).

Each function restates the torch.distributions formula the reference calls at
mininf/core.py:241 (cited per function, TORCH = torch/ of torch 2.10 as installed here).
"""
from __future__ import annotations

import math

import numpy as np
from scipy import special

FLOAT32_EPS = float(np.finfo(np.float32).eps)   # clamp_probs, TORCH/distributions/utils.py
HALF_LOG_2PI = 0.5 * math.log(2 * math.pi)      # TORCH/distributions/normal.py:103


def normal(loc, scale, v):
    """
    TORCH/distributions/normal.py:88-103. Returns (lp, dloc, dscale, dv).
    """
    loc, scale, v = (np.asarray(a, dtype=np.float64) for a in (loc, scale, v))
    z = (v - loc) / scale
    lp = -0.5 * z * z - np.log(scale) - HALF_LOG_2PI
    return lp, z / scale, (z * z - 1.0) / scale, -z / scale


def bernoulli_logits(l, v):
    """
    TORCH/distributions/bernoulli.py:121-125 (-BCE with logits). Returns (lp, dl).
    """
    l, v = np.asarray(l, np.float64), np.asarray(v, np.float64)
    lp = -(np.maximum(l, 0.0) - l * v + np.log1p(np.exp(-np.abs(l))))
    return lp, v - special.expit(l)


def probs_to_logits(p):
    """
    TORCH/distributions/utils.py probs_to_logits(is_binary=True) after clamp_probs (float32 eps).
    Returns (logits, dlogits/dp) with clamp's pass-through mask.
    """
    p = np.asarray(p, np.float64)
    lo, hi = np.float32(FLOAT32_EPS), np.float32(1.0) - np.float32(FLOAT32_EPS)
    pc = np.clip(p, float(lo), float(hi))
    logits = np.log(pc) - np.log1p(-pc)
    inside = (p >= float(lo)) & (p <= float(hi))
    return logits, np.where(inside, 1.0 / pc + 1.0 / (1.0 - pc), 0.0)


def bernoulli_probs(p, v):
    """
    TORCH/distributions/bernoulli.py:104-106 + 121-125. Returns (lp, dp).
    """
    l, dl_dp = probs_to_logits(p)
    lp, dl = bernoulli_logits(l, v)
    return lp, dl * dl_dp


def _xlogy(x, y):
    return np.where(x == 0, 0.0, x * np.log(np.where(x == 0, 1.0, y)))


def beta(a, b, v):
    """
    TORCH/distributions/beta.py:88-92 -> dirichlet.py:90-97. Returns (lp, da, db, dv).
    """
    a, b, v = (np.asarray(t, np.float64) for t in (a, b, v))
    lp = _xlogy(a - 1, v) + _xlogy(b - 1, 1 - v) + special.gammaln(a + b) - special.gammaln(a) \
        - special.gammaln(b)
    psi = special.digamma(a + b)
    return (lp, np.log(v) + psi - special.digamma(a), np.log1p(-v) + psi - special.digamma(b),
            (a - 1) / v - (b - 1) / (1 - v))


def beta_entropy(a, b):
    """
    TORCH/distributions/dirichlet.py:122-130 for two components; returns (H, dH/da, dH/db).
    """
    a, b = float(a), float(b)
    t = a + b
    h = special.betaln(a, b) - (a - 1) * special.digamma(a) - (b - 1) * special.digamma(b) \
        + (t - 2) * special.digamma(t)
    da = -(a - 1) * special.polygamma(1, a) + (t - 2) * special.polygamma(1, t)
    db = -(b - 1) * special.polygamma(1, b) + (t - 2) * special.polygamma(1, t)
    return h, da, db


def categorical(logits, v):
    """
    TORCH/distributions/categorical.py:74-78 (normalisation) and 150-156 (gather).
    Returns (lp, dlogits) for raw logits [..., C].
    """
    logits = np.asarray(logits, np.float64)
    norm = logits - special.logsumexp(logits, axis=-1, keepdims=True)
    v = np.asarray(v)
    lp = np.take_along_axis(norm, v[..., None], -1)[..., 0]
    soft = np.exp(norm)
    onehot = np.zeros_like(norm)
    np.put_along_axis(onehot, v[..., None], 1.0, -1)
    return lp, onehot - soft


# ---- implicit reparameterisation gradient of Beta draws ---------------------------------------
# Restatement of torch._dirichlet_grad (TORCH/include/ATen/native/Distributions.h,
# dirichlet_grad_one and helpers), evaluated in float64.

def _grad_small_alpha(x, a, b):
    factor = special.digamma(a) - special.digamma(a + b) - math.log(x)
    coeff = 1.0
    series = coeff / a * (factor + 1 / a)
    for n in range(1, 11):
        coeff *= (n - b) * x / n
        series += coeff / (a + n) * (factor + 1 / (a + n))
    r = x * (1 - x) ** (-b) * series
    return 0.0 if math.isnan(r) else r


def _grad_small_beta(x, a, b):
    factor = special.digamma(a + b) - special.digamma(b)
    coeff, prod, dprod, series = 1.0, 1.0, 0.0, factor / a
    for n in range(1, 9):
        coeff *= -x / n
        dprod = dprod * (b - n) + prod
        prod *= (b - n)
        series += coeff / (a + n) * (dprod + factor * prod)
    r = -(1 - x) ** (1 - b) * series
    return 0.0 if math.isnan(r) else r


def _grad_mid(x, a, b):
    t = a + b
    mean = a / t
    sd = math.sqrt(a * b / (t + 1)) / t
    if mean - 0.1 * sd <= x <= mean + 0.1 * sd:
        poly = (47 * x * b ** 4 + a * ((43 + 20 * (16 + 27 * b) * x) * b ** 3 + a * (
            3 * (59 + 180 * b - 90 * x) * b * b + a * ((453 + 1620 * b * (1 - x) - 455 * x) * b
                                                       + a * (8 * (1 - x) * (135 * b - 11))))))
        pre_num = (1 + 12 * a) * (1 + 12 * b) / (t * t)
        pre_den = 12960 * a ** 3 * b * b * (1 + 12 * t)
        return pre_num / (1 - x) * poly / pre_den
    prefactor = -x / math.sqrt(2 * a * b / t)
    stirling = ((1 + 1 / (12 * a) + 1 / (288 * a * a)) * (1 + 1 / (12 * b) + 1 / (288 * b * b))
                / (1 + 1 / (12 * t) + 1 / (288 * t * t)))
    axbx = a * (x - 1) + b * x
    term1 = (2 * a * a * (x - 1) + a * b * (x - 1) - x * b * b) / (
        math.sqrt(2 * a / b) * t ** 1.5 * axbx * axbx)
    term2 = 0.5 * math.log(a / (t * x))
    term3 = math.sqrt(8 * a * b / t) / (b * x + a * (x - 1))
    term4 = (b * math.log(b / (t * (1 - x))) + a * math.log(a / (t * x))) ** -1.5
    return stirling * prefactor * (term1 + term2 * (term3 + (term4 if x < mean else -term4)))


# Coefficient table of the rational correction, as published in torch's Distributions.h.
_COEF = np.array([
    [[[1.003668233, -0.01061107488, -0.0657888334, 0.01201642863],
      [0.6336835991, -0.3557432599, 0.05486251648, -0.001465281033],
      [-0.03276231906, 0.004474107445, 0.002429354597, -0.0001557569013]],
     [[0.221950385, -0.3187676331, 0.01799915743, 0.01074823814],
      [-0.2951249643, 0.06219954479, 0.01535556598, 0.001550077057],
      [0.02155310298, 0.004170831599, 0.001292462449, 6.976601077e-05]],
     [[-0.05980841433, 0.008441916499, 0.01085618172, 0.002319392565],
      [0.02911413504, 0.01400243777, -0.002721828457, 0.000751041181],
      [0.005900514878, -0.001936558688, -9.495446725e-06, 5.385558597e-05]]],
    [[[1, -0.02924021934, -0.04438342661, 0.007285809825],
      [0.6357567472, -0.3473456711, 0.05454656494, -0.002407477521],
      [-0.03301322327, 0.004845219414, 0.00231480583, -0.0002307248149]],
     [[0.5925320577, -0.1757678135, 0.01505928619, 0.000564515273],
      [0.1014815858, -0.06589186703, 0.01272886114, -0.0007316646956],
      [-0.007258481865, 0.001096195486, 0.0003934994223, -4.12701925e-05]],
     [[0.06469649321, -0.0236701437, 0.002902096474, -5.896963079e-05],
      [0.001925008108, -0.002869809258, 0.0008000589141, -6.063713228e-05],
      [-0.0003477407336, 6.959756487e-05, 1.097287507e-05, -1.650964693e-06]]]])


def dirichlet_grad_one(x, alpha, total):
    """
    d x / d alpha of a Beta(alpha, total - alpha) draw, divided by (1 - x) (torch convention).
    """
    x, alpha, total = float(x), float(alpha), float(total)
    beta_ = total - alpha
    boundary = total * x * (1 - x)
    if x <= 0.5 and boundary < 2.5:
        return _grad_small_alpha(x, alpha, beta_)
    if x >= 0.5 and boundary < 0.75:
        return -_grad_small_beta(1 - x, beta_, alpha)
    if alpha > 6 and beta_ > 6:
        return _grad_mid(x, alpha, beta_)
    u = math.log(x)
    a = math.log(alpha) - u
    b = math.log(total) - a
    pu = (1.0, u, u * u)
    pa = (1.0, a, a * a)
    num = den = 0.0
    for r in range(3):
        for c in range(3):
            w = pu[r] * pa[c]
            n, d = _COEF[0, r, c], _COEF[1, r, c]
            num += w * (n[0] + b * (n[1] + b * (n[2] + b * n[3])))
            den += w * (d[0] + b * (d[1] + b * (d[2] + b * d[3])))
    approx = x * (special.digamma(total) - special.digamma(alpha)) / beta_
    return num / den * approx


def dirichlet_grad(x, alpha, total):
    return np.vectorize(dirichlet_grad_one, otypes=[np.float64])(x, alpha, total)


def beta_draw_grads(x, c1, c0):
    """
    d x / d c1 and d x / d c0 of Beta(c1, c0) draws x (torch _Dirichlet_backward with
    grad_output = (1, 0), TORCH/distributions/dirichlet.py:17-20).
    """
    x = np.asarray(x, np.float64)
    x32 = np.asarray(x, np.float32)
    tot = float(np.float32(c1) + np.float32(c0))
    w = (np.float32(1.0) - x32).astype(np.float64)
    d1 = dirichlet_grad(x, c1, tot) * (1.0 - x)
    d0 = -dirichlet_grad(w, c0, tot) * x
    return d1, d0


# ---- families of the reference's examples (round 2) -------------------------------------------

def gamma(a, r, v):
    """
    TORCH/distributions/gamma.py:90-99: xlogy(a, r) + xlogy(a - 1, v) - r v - lgamma(a).
    Returns (lp, da, dr, dv).
    """
    a, r, v = (np.asarray(t, np.float64) for t in (a, r, v))
    lp = _xlogy(a, r) + _xlogy(a - 1.0, v) - r * v - special.gammaln(a)
    return lp, np.log(r) + np.log(v) - special.digamma(a), a / r - v, (a - 1.0) / v - r


def poisson(rate, v):
    """
    TORCH/distributions/poisson.py:60-65: xlogy(v, rate) - rate - lgamma(v + 1).
    Returns (lp, drate, dv) (dv: torch's continuous derivative).
    """
    rate, v = np.asarray(rate, np.float64), np.asarray(v, np.float64)
    lp = _xlogy(v, rate) - rate - special.gammaln(v + 1.0)
    return lp, v / rate - 1.0, np.log(rate) - special.digamma(v + 1.0)


def inverse_gamma(a, r, y):
    """
    mininf/distributions.py:5-11 (Gamma through PowerTransform(-1)), i.e. TORCH
    transformed_distribution.py log_prob: Gamma.log_prob(1 / y) - log|-y / x|, x = 1 / y.
    Returns (lp, da, dr, dy).
    """
    a, r, y = (np.asarray(t, np.float64) for t in (a, r, y))
    x = 1.0 / y
    lp, da, dr, dx = gamma(a, r, x)
    return lp - np.log(y / x), da, dr, -dx * x * x - 2.0 / y


def gamma_entropy(a, r):
    """
    TORCH/distributions/gamma.py:101-107: a - log r + lgamma(a) + (1 - a) psi(a).
    Returns (H, dH/da, dH/dr).
    """
    a, r = np.asarray(a, np.float64), np.asarray(r, np.float64)
    h = a - np.log(r) + special.gammaln(a) + (1.0 - a) * special.digamma(a)
    return h, 1.0 + (1.0 - a) * special.polygamma(1, a), -1.0 / r


def standard_gamma_grad(alpha, x):
    """
    d x / d alpha of standard Gamma draws: TORCH/include/ATen/native/Distributions.h:310
    (standard_gamma_grad_one, accumulation in double as on the CPU). Vectorised over inputs.
    """
    alpha = np.asarray(alpha, np.float64)
    x = np.asarray(x, np.float64)
    alpha, x = np.broadcast_arrays(alpha, x)
    out = np.empty(alpha.shape)
    f = np.float32
    for idx in np.ndindex(alpha.shape):
        a, xv = float(alpha[idx]), float(x[idx])
        if xv < float(f(0.8)):
            numer, denom = 1.0, a
            s1, s2 = numer / denom, numer / (denom * denom)
            for i in range(1, 6):
                numer *= -xv / i
                denom += 1.0
                s1 += numer / denom
                s2 += numer / (denom * denom)
            pxa = xv ** a
            pdf = xv ** (a - 1.0) * math.exp(-xv)
            cdf = pxa * s1
            cdf_a = (math.log(xv) - float(special.digamma(a))) * cdf - pxa * s2
            res = -cdf_a / pdf
            out[idx] = 0.0 if math.isnan(res) else res
        elif a > 8.0:
            if float(f(0.9)) * a <= xv <= float(f(1.1)) * a:
                n1 = 1 + 24 * a * (1 + 12 * a)
                n2 = 1440 * a * a + 6 * xv * (53 - 120 * xv) - 65 * xv * xv / a + \
                    a * (107 + 3600 * xv)
                out[idx] = n1 * n2 / (1244160 * a * a * a * a)
            else:
                den = math.sqrt(8 * a)
                t2 = den / (a - xv)
                t3 = (xv - a - a * math.log(xv / a)) ** -1.5
                t23 = t2 - t3 if xv < a else t2 + t3
                t1 = math.log(xv / a) * t23 - math.sqrt(2 / a) * (a + xv) / ((a - xv) ** 2)
                stirling = 1 + 1 / (12 * a) * (1 + 1 / (24 * a))
                out[idx] = -stirling * xv * t1 / den
        else:
            u, v = math.log(xv / a), math.log(a)
            coef = ((0.16009398, -0.094634809, 0.025146376, -0.0030648343, 1, 0.32668115,
                     0.10406089, 0.0014179084),
                    (0.53487893, 0.1298071, 0.065735949, -0.0015649758, 0.16639465, 0.020070113,
                     -0.0035938915, -0.00058392623),
                    (0.040121004, -0.0065914022, -0.0026286047, -0.0013441777, 0.017050642,
                     -0.0021309326, 0.00085092367, -1.5247877e-07))
            c = [coef[0][i] + u * (coef[1][i] + u * coef[2][i]) for i in range(8)]
            p = c[0] + v * (c[1] + v * (c[2] + v * c[3]))
            q = c[4] + v * (c[5] + v * (c[6] + v * c[7]))
            out[idx] = math.exp(p / q)
    return out
