"""
K-particle ELBO oracles (numpy float64, test infrastructure only) for the build's configs.

Semantics restated from the reference: loss = -(sum of site contributions + guide entropy) for one
guide draw (mininf/nn.py:212-228, contributions per mininf/core.py:247-273, minibatch scale
core.py:267-271, masked sums core.py:262-265); the K-particle estimator is the mean of K such
single-draw losses. Guide draws are injected (eps for Normal factors, x for Beta
factors), parameters are the reference's unconstrained ones (nn.py:75-80: log for positive
parameters, identity for real ones), and gradients are with respect to those.
"""
from __future__ import annotations

import numpy as np
from scipy import special

from . import logprob as lpf


def _f64(a):
    return np.asarray(a, dtype=np.float64)


def beta_bernoulli_elbo(x, a0, b0, c1, c0, theta):
    """
    Biased coin (README.md:40-44): theta ~ Beta(a0, b0), x ~ Bernoulli(theta)[n]; guide
    Beta(c1, c0) with draws ``theta`` [K].
    """
    x = _f64(x)
    theta = _f64(np.asarray(theta, np.float32))
    K = theta.shape[0]
    lp_prior, _, _, dprior = lpf.beta(a0, b0, theta)
    logits, dl_dp = lpf.probs_to_logits(theta)
    S, n = x.sum(), float(x.size)
    softplus = np.logaddexp(0.0, logits)
    lp_lik = S * logits - n * softplus
    dlik = (S - n * special.expit(logits)) * dl_dp
    T = lp_prior + lp_lik
    H, dHa, dHb = lpf.beta_entropy(c1, c0)
    loss = -(T.mean() + H)
    d1, d0 = lpf.beta_draw_grads(theta, c1, c0)
    g_theta = -(dprior + dlik) / K
    grad_c1 = float((g_theta * d1).sum() - dHa)
    grad_c0 = float((g_theta * d0).sum() - dHb)
    return {"loss": float(loss), "T": T, "H": H,
            "grad_u_concentration1": grad_c1 * float(c1),
            "grad_u_concentration0": grad_c0 * float(c0)}


def regression_elbo(X, y, loc, scale, eps, batch_scale=1.0):
    """
    Linear regression (tests/test_mininf.py:13-18, examples/minibatch.md:24-33):
    theta ~ N(0, 1)[p], y ~ N(X theta, 1) (scaled by ``batch_scale`` under ``batch``); guide
    MF Normal(loc, scale) with eps [K, p].
    """
    X, y, loc, scale, eps = (_f64(a) for a in (X, y, loc, scale, eps))
    K = eps.shape[0]
    theta = _f64(np.float32(loc) + np.float32(eps) * np.float32(scale))
    mu = theta @ X.T                                   # [K, n]
    lp_prior = (-0.5 * theta ** 2 - lpf.HALF_LOG_2PI).sum(1)
    resid = y[None, :] - mu
    lp_y = batch_scale * (-0.5 * resid ** 2 - lpf.HALF_LOG_2PI).sum(1)
    T = lp_prior + lp_y
    H = (0.5 + lpf.HALF_LOG_2PI + np.log(scale)).sum()
    loss = -(T.mean() + H)
    dT = -theta + batch_scale * resid @ X                # [K, p]
    grad_loc = -dT.mean(0)
    grad_scale = -(dT * eps).mean(0) - 1.0 / scale
    return {"loss": float(loss), "T": T, "grad_loc": grad_loc, "grad_u_scale": grad_scale * scale}


def hierarchical_masked_elbo(y, b, mask, mu_loc, mu_scale, z_loc, z_scale, eps_mu, eps_z,
                             y_scale=0.5):
    """
    Masked hierarchical model (examples/missing-observations.md:33-45 restated):
    mu ~ N(0, 1); z ~ N(mu, 1)[n]; y ~ N(z, 0.5)[n] masked; b ~ Bernoulli(logits=z)[n] masked.
    Guide: MF Normal over mu (scalars) and z ([n]).
    """
    y, b, m = _f64(y), _f64(b), _f64(mask)
    mu_loc, mu_scale = float(mu_loc), float(mu_scale)
    z_loc, z_scale, eps_mu, eps_z = (_f64(a) for a in (z_loc, z_scale, eps_mu, eps_z))
    K = eps_z.shape[0]
    mu = _f64(np.float32(mu_loc) + np.float32(eps_mu) * np.float32(mu_scale))        # [K]
    z = _f64(np.float32(z_loc) + np.float32(eps_z) * np.float32(z_scale))           # [K, n]
    lp_mu = -0.5 * mu ** 2 - lpf.HALF_LOG_2PI
    d = z - mu[:, None]
    lp_z = (-0.5 * d ** 2 - lpf.HALF_LOG_2PI).sum(1)
    ry = (y[None, :] - z) / y_scale
    lp_y = (m * (-0.5 * ry ** 2 - np.log(y_scale) - lpf.HALF_LOG_2PI)).sum(1)
    lb, dlb = lpf.bernoulli_logits(z, b[None, :])
    lp_b = (m * lb).sum(1)
    T = lp_mu + lp_z + lp_y + lp_b
    H = (0.5 + lpf.HALF_LOG_2PI + np.log(mu_scale)) + (0.5 + lpf.HALF_LOG_2PI + np.log(z_scale)).sum()
    loss = -(T.mean() + H)
    dT_mu = -mu + d.sum(1)
    dT_z = -d + m * ry / y_scale + m * dlb
    out = {"loss": float(loss), "T": T}
    out["grad_mu_loc"] = float(-dT_mu.mean())
    out["grad_mu_scale"] = float((-(dT_mu * eps_mu).mean() - 1.0 / mu_scale) * mu_scale)
    out["grad_z_loc"] = -dT_z.mean(0)
    out["grad_z_scale"] = (-(dT_z * eps_z).mean(0) - 1.0 / z_scale) * z_scale
    return out


def categorical_masked_elbo(y, mask, loc, scale, eps):
    """
    Categorical model (no reference test or example): theta ~ N(0, 1)[C];
    y ~ Categorical(logits=theta)[n] masked (torch categorical.py:74-78 normalisation,
    150-156 gather; masked sum core.py:262-265). Guide MF Normal(loc, scale)[C], eps [K, C].
    """
    y, m = np.asarray(y, np.int64), _f64(mask)
    loc, scale, eps = (_f64(a) for a in (loc, scale, eps))
    K, C = eps.shape
    theta = _f64(np.float32(loc) + np.float32(eps) * np.float32(scale))       # [K, C]
    lse = special.logsumexp(theta, axis=1, keepdims=True)
    norm = theta - lse
    counts = np.bincount(y, weights=m, minlength=C)[:C]                         # [C]
    T = (-0.5 * theta ** 2 - lpf.HALF_LOG_2PI).sum(1) + norm @ counts
    H = (0.5 + lpf.HALF_LOG_2PI + np.log(scale)).sum()
    loss = -(T.mean() + H)
    dT = -theta + counts[None, :] - m.sum() * np.exp(norm)
    grad_loc = -dT.mean(0)
    grad_scale = -(dT * eps).mean(0) - 1.0 / scale
    return {"loss": float(loss), "T": T, "grad_loc": grad_loc, "grad_u_scale": grad_scale * scale}


def regression_elbo_gram(G, Xty, yty, n, loc, scale, eps, batch_scale=1.0):
    """
    ``regression_elbo`` through the data's sufficient statistics G = X^T X, X^T y, y^T y (fp64),
    for full-size checks: sum_i (y_i - x_i theta)^2 = y^T y - 2 theta^T X^T y + theta^T G theta.
    """
    G, Xty, loc, scale, eps = (_f64(a) for a in (G, Xty, loc, scale, eps))
    K = eps.shape[0]
    theta = _f64(np.float32(loc) + np.float32(eps) * np.float32(scale))
    rss = float(yty) - 2.0 * theta @ Xty + np.einsum("kp,pq,kq->k", theta, G, theta)
    lp_prior = (-0.5 * theta ** 2 - lpf.HALF_LOG_2PI).sum(1)
    lp_y = batch_scale * (-0.5 * rss - n * lpf.HALF_LOG_2PI)
    T = lp_prior + lp_y
    H = (0.5 + lpf.HALF_LOG_2PI + np.log(scale)).sum()
    loss = -(T.mean() + H)
    dT = -theta + batch_scale * (Xty[None, :] - theta @ G)
    grad_loc = -dT.mean(0)
    grad_scale = -(dT * eps).mean(0) - 1.0 / scale
    return {"loss": float(loss), "T": T, "grad_loc": grad_loc, "grad_u_scale": grad_scale * scale}


def hierarchical_masked_elbo_chunked(y, b, mask, mu_loc, mu_scale, z_loc, z_scale, eps_mu,
                                     eps_z_rows, K, chunk=16, y_scale=0.5):
    """
    ``hierarchical_masked_elbo`` over K particles taken ``chunk`` at a time (full-size checks):
    ``eps_z_rows(k0, k1)`` returns the z noise of particles [k0, k1). Loss and gradients are
    particle means, so the chunks combine with weights k1 - k0.
    """
    eps_mu = _f64(eps_mu)
    T = []
    acc = {"grad_mu_loc": 0.0, "grad_mu_scale": 0.0, "grad_z_loc": 0.0, "grad_z_scale": 0.0}
    z_scale64 = _f64(z_scale)
    for k0 in range(0, K, chunk):
        k1 = min(K, k0 + chunk)
        part = hierarchical_masked_elbo(y, b, mask, mu_loc, mu_scale, z_loc, z_scale,
                                        eps_mu[k0:k1], eps_z_rows(k0, k1), y_scale)
        w = (k1 - k0) / K
        T.append(part["T"])
        # undo the entropy terms (added once below) before weighting the particle means
        acc["grad_mu_loc"] += w * part["grad_mu_loc"]
        acc["grad_mu_scale"] += w * (part["grad_mu_scale"] + 1.0)
        acc["grad_z_loc"] = acc["grad_z_loc"] + w * part["grad_z_loc"]
        acc["grad_z_scale"] = acc["grad_z_scale"] + w * (part["grad_z_scale"] + 1.0)
    T = np.concatenate(T)
    H = (0.5 + lpf.HALF_LOG_2PI + np.log(float(mu_scale))) + \
        (0.5 + lpf.HALF_LOG_2PI + np.log(z_scale64)).sum()
    acc["grad_mu_scale"] -= 1.0
    acc["grad_z_scale"] = acc["grad_z_scale"] - 1.0
    return {"loss": float(-(T.mean() + H)), "T": T, **acc}
