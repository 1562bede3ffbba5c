"""
The reference's example models, written against ``mininf_amd`` exactly as the examples write them
against ``mininf`` (only the import differs), for the "existing model functions run unchanged" tests:

* ``feature_model``: examples/regression-with-feature-uncertainty.md:26-38 (Gamma, Normal and
  Poisson sites);
* ``missing_model``: examples/missing-observations.md:28-45 (Gamma, InverseGamma,
  MultivariateNormal and Normal sites; host globals ``x`` and ``torch.eye`` inside the model);
* ``predictive_model``: examples/predictive.md:22-38 (values, Gamma, Normal).

The fixtures they are checked against (tests/golden/*.npz) were produced by running the same code
through the reference (tests/golden/make_golden.py).
"""
import torch
from torch.distributions import Gamma, MultivariateNormal, Normal, Poisson
from torch.distributions.constraints import nonnegative_integer

import mininf_amd as mininf
import mininf_amd.distributions

FEATURE_N = 30
MISSING_N = 50
MISSING_X = torch.linspace(0, 1, MISSING_N)


def feature_model():
    n = FEATURE_N
    # Latent features (z) and noisy observations (x).
    population_scale = mininf.sample("population_scale", Gamma(2, 2))
    z = mininf.sample("z", Normal(0, population_scale), n)
    noise_scale = mininf.sample("noise_scale", Gamma(2, 2))
    x = mininf.sample("x", Normal(z, noise_scale))  # noqa: F841

    # Count-valued outcomes (y).
    intercept = mininf.sample("intercept", Normal(0, 1))
    slope = mininf.sample("slope", Normal(0, 1))
    y = mininf.sample("y", Poisson((intercept + z * slope).exp()))  # noqa: F841


def missing_model() -> None:
    n, x = MISSING_N, MISSING_X
    # Marginal GP variance, length scale, and observation noise scale.
    sigma = mininf.sample("sigma", Gamma(2, 2))
    length_scale = mininf.sample("length_scale", mininf_amd.distributions.InverseGamma(10, 1))
    kappa = mininf.sample("kappa", Gamma(2, 10))

    # GP sample with squared exponential covariance and jitter.
    residuals = (x[:, None] - x) / length_scale
    cov = sigma * sigma * (- residuals ** 2 / 2).exp() + 1e-3 * torch.eye(n)
    z = mininf.sample("z", MultivariateNormal(torch.zeros(n), cov))

    # Observation model.
    mininf.sample("y", Normal(z, kappa))


def predictive_model():
    # Sample size and number of polynomial features.
    n = mininf.value("n", 30, support=nonnegative_integer)
    p = mininf.value("p", 3, support=nonnegative_integer)

    # Covariates and predictions.
    x = mininf.sample("x", torch.distributions.Normal(0, 1), n)
    X = mininf.value("X", x[:, None] ** torch.arange(p))
    theta = mininf.sample("theta", torch.distributions.Normal(0, 1), p)
    prediction = mininf.value("prediction", X @ theta)

    # Observations.
    sigma = mininf.sample("sigma", torch.distributions.Gamma(2, 2))
    y = mininf.sample("y", torch.distributions.Normal(prediction, sigma))  # noqa: F841
