"""
K-particle ELBO of the reference's missing-observations example (test infrastructure only).

The model of examples/missing-observations.md:33-45 (Gamma and InverseGamma priors, a
MultivariateNormal GP prior with a 1e-3 jitter, a masked Normal likelihood) with the guide of
:77-83 (mean-field Normal over z, Gamma over sigma and length_scale), evaluated with torch-CPU
autograd in a chosen precision and with injected draws (Normal eps; Gamma: the
standard draw g with x = g / rate, backward through torch._standard_gamma_grad).

Why it exists: the GP prior's Cholesky factorisation of an ill-conditioned covariance rounds
differently in float32 on every device, so the reference's own float32 fixture is itself only
accurate to ~1e-4. In float32 this restatement reproduces that fixture (tests/test_oracle.py pins
it); in float64 it is the truth the device result is measured against.
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch
from torch.distributions import (Gamma, MultivariateNormal, Normal, PowerTransform,
                                 TransformedDistribution)


class _InjectedStandardGamma(torch.autograd.Function):
    """torch._standard_gamma with a supplied result g (backward: torch._standard_gamma_grad)."""
    @staticmethod
    def forward(ctx, concentration, g):
        ctx.save_for_backward(concentration, g)
        return g.clone()

    @staticmethod
    def backward(ctx, grad):
        concentration, g = ctx.saved_tensors
        return grad * torch._standard_gamma_grad(concentration, g), None


def missing_observations_elbo(fixture: Dict[str, np.ndarray], dtype=torch.float64,
                              n: int = 50) -> Dict[str, np.ndarray]:
    """
    Loss and gradients with respect to the guide's unconstrained parameters
    (``grad_<factor>_<parameter>``, the fixture's keys) for the fixture's data and draws.
    """
    def t(a):
        return torch.as_tensor(np.asarray(a), dtype=dtype)

    x = torch.linspace(0, 1, n, dtype=torch.float32).to(dtype)
    y, mask, kappa = t(fixture["y"]), torch.as_tensor(fixture["mask"]), t(fixture["kappa"])
    eps_z, g_sigma, g_len = t(fixture["eps_z"]), t(fixture["g_sigma"]), t(fixture["g_length_scale"])
    K = eps_z.shape[0]
    # unconstrained parameters as ParameterizedDistribution stores them (nn.py:75-80)
    u = {
        ("z", "loc"): t(fixture["z_loc"]).clone(),
        ("z", "scale"): torch.log(torch.ones(n, dtype=torch.float32) *
                                  torch.tensor(float(fixture["kappa"]))).to(dtype),
        ("sigma", "concentration"): torch.log(torch.tensor(2.0)).to(dtype),
        ("sigma", "rate"): torch.log(torch.tensor(2.0)).to(dtype),
        ("length_scale", "concentration"): torch.log(torch.tensor(2.0)).to(dtype),
        ("length_scale", "rate"): torch.log(torch.tensor(2.0)).to(dtype),
    }
    for v in u.values():
        v.requires_grad_()
    loc, scale = u[("z", "loc")], u[("z", "scale")].exp()
    cs, rs = u[("sigma", "concentration")].exp(), u[("sigma", "rate")].exp()
    cl, rl = u[("length_scale", "concentration")].exp(), u[("length_scale", "rate")].exp()
    two, one, ten = (torch.tensor(v, dtype=dtype) for v in (2.0, 1.0, 10.0))
    total = 0
    for k in range(K):
        z = loc + eps_z[k] * scale
        sigma = _InjectedStandardGamma.apply(cs, g_sigma[k]) / rs
        length = _InjectedStandardGamma.apply(cl, g_len[k]) / rl
        lp = Gamma(two, two).log_prob(sigma)
        lp = lp + TransformedDistribution(Gamma(ten, one), [PowerTransform(-one)]).log_prob(length)
        lp = lp + Gamma(two, ten).log_prob(kappa)
        residuals = (x[:, None] - x) / length
        cov = sigma * sigma * (- residuals ** 2 / 2).exp() + 1e-3 * torch.eye(n, dtype=dtype)
        lp = lp + MultivariateNormal(torch.zeros(n, dtype=dtype), cov).log_prob(z)
        lp = lp + Normal(z, kappa).log_prob(y)[mask].sum()
        entropy = Normal(loc, scale).entropy().sum() + Gamma(cs, rs).entropy() + \
            Gamma(cl, rl).entropy()
        total = total - (lp + entropy)
    loss = total / K
    loss.backward()
    out = {"loss": float(loss)}
    for (factor, pname), v in u.items():
        out[f"grad_{factor}_{pname}"] = v.grad.detach().double().numpy()
    return out
