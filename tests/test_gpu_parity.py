"""
Parity of the HIP ELBO path against the reference (golden fixtures made by running the reference,
tests/golden/make_golden.py) and against the numpy float64 oracle (oracle/elbo.py) on the same
injected guide draws.

Tolerance (BASELINE.json north_star): ELBO values and gradients within 1e-5 relative of the reference
path. Gradients of individual vector entries are compared against the vector's max-norm
(|g - g_ref| <= 1e-5 * max|g_ref| + atol) because single entries can cancel to ~0.
"""
import numpy as np
import pytest
import torch
from torch.distributions import Bernoulli, Beta, Normal

import mininf_amd
from mininf_amd.nn import EvidenceLowerBoundLoss, ParameterizedDistribution, \
    ParameterizedFactorizedDistribution
from oracle import elbo as oracle
from tests.conftest import golden

pytestmark = pytest.mark.gpu
RTOL = 1e-5


def close(got, want, rtol=RTOL, atol=1e-6):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    scale = np.abs(want).max() if want.size else 0.0
    err = np.abs(got - want).max() if want.size else 0.0
    assert err <= rtol * scale + atol, (err, scale, got, want)


def beta_bernoulli(n):
    def model():
        theta = mininf_amd.sample("theta", Beta(2, 2))
        mininf_amd.sample("x", Bernoulli(theta), sample_shape=[n])
    return model


def test_c1_readme_three_adam_steps(device):
    g = golden("c1_readme.npz")
    x = torch.as_tensor(g["x"], device=device)
    approximation = ParameterizedDistribution(Beta, concentration0=2, concentration1=2).to(device)
    optimizer = torch.optim.Adam(approximation.parameters(), lr=0.02)
    loss = EvidenceLowerBoundLoss()
    conditioned = mininf_amd.condition(beta_bernoulli(10), x=x)
    for step in range(3):
        optimizer.zero_grad()
        value = loss(conditioned, {"theta": approximation()},
                     _noise={"theta": torch.as_tensor(g["draws"][step:step + 1], device=device)})
        value.backward()
        optimizer.step()
        close(float(value), g["losses"][step])
        close([float(p) for p in approximation.distribution_parameters.values()],
              g["params"][step], rtol=1e-5)


def test_c2_beta_bernoulli_small(device):
    g = golden("c2_beta_bernoulli.npz")
    n = g["x"].shape[0]
    approximation = ParameterizedDistribution(Beta, concentration1=float(g["c1"]),
                                              concentration0=float(g["c0"])).to(device)
    K = g["draws"].shape[0]
    loss = EvidenceLowerBoundLoss(num_particles=K)
    value = loss(mininf_amd.condition(beta_bernoulli(n), x=torch.as_tensor(g["x"], device=device)),
                 {"theta": approximation()},
                 _noise={"theta": torch.as_tensor(g["draws"], device=device)})
    value.backward()
    params = approximation.distribution_parameters
    close(float(value), g["loss"])
    close(params["concentration1"].grad.cpu(), g["grad_concentration1"])
    close(params["concentration0"].grad.cpu(), g["grad_concentration0"])
    ref = oracle.beta_bernoulli_elbo(g["x"], 2, 2, float(g["c1"]), float(g["c0"]), g["draws"])
    close(float(value), ref["loss"])
    close(params["concentration1"].grad.cpu(), ref["grad_u_concentration1"])


def regression_model(n_total, p, batched):
    def model():
        theta = mininf_amd.sample("theta", Normal(0, 1), sample_shape=p)
        if batched:
            with mininf_amd.batch(n_total):
                with mininf_amd.no_log_prob():
                    X = mininf_amd.sample("X", Normal(0, 1), sample_shape=(n_total, p))
                mininf_amd.sample("y", Normal(X @ theta, 1))
        else:
            with mininf_amd.no_log_prob():
                X = mininf_amd.sample("X", Normal(0, 1), sample_shape=(n_total, p))
            mininf_amd.sample("y", Normal(X @ theta, 1))
    return model


@pytest.mark.parametrize("name, batched", [("c3_regression.npz", False),
                                           ("c4_minibatch.npz", True)])
def test_c3_c4_regression_small(device, name, batched):
    g = golden(name)
    n_obs, p = g["X"].shape
    n_total = int(g["n_total"])
    approximation = ParameterizedDistribution(Normal, loc=torch.as_tensor(g["loc0"]),
                                              scale=torch.as_tensor(g["scale0"])).to(device)
    K = g["eps"].shape[0]
    loss = EvidenceLowerBoundLoss(num_particles=K)
    conditioned = mininf_amd.condition(regression_model(n_total, p, batched),
                                       X=torch.as_tensor(g["X"], device=device),
                                       y=torch.as_tensor(g["y"], device=device))
    value = loss(conditioned, {"theta": approximation()},
                 _noise={"theta": torch.as_tensor(g["eps"], device=device)})
    value.backward()
    params = approximation.distribution_parameters
    close(float(value), g["loss"])
    close(params["loc"].grad.cpu(), g["grad_loc"])
    close(params["scale"].grad.cpu(), g["grad_scale"])


def test_c5_masked_hierarchical_small(device):
    g = golden("c5_masked_hierarchical.npz")
    n = g["y"].shape[0]

    def model():
        mu = mininf_amd.sample("mu", Normal(0, 1))
        z = mininf_amd.sample("z", Normal(mu, 1), sample_shape=[n])
        mininf_amd.sample("y", Normal(z, 0.5))
        mininf_amd.sample("b", Bernoulli(logits=z))

    mask = torch.as_tensor(g["mask"], device=device)
    y = torch.masked.as_masked_tensor(torch.as_tensor(g["y"], device=device), mask)
    b = torch.masked.as_masked_tensor(torch.as_tensor(g["b"], device=device), mask)
    approximation = ParameterizedFactorizedDistribution(
        mu=ParameterizedDistribution(Normal, loc=0.1, scale=0.9),
        z=ParameterizedDistribution(Normal, loc=torch.as_tensor(g["z_loc0"]),
                                    scale=torch.ones(n) * 0.8),
    ).to(device)
    K = g["eps_z"].shape[0]
    loss = EvidenceLowerBoundLoss(num_particles=K)
    value = loss(mininf_amd.condition(model, y=y, b=b), approximation(),
                 _noise={"mu": torch.as_tensor(g["eps_mu"], device=device),
                         "z": torch.as_tensor(g["eps_z"], device=device)})
    value.backward()
    close(float(value), g["loss"])
    for factor in ("mu", "z"):
        for pname, param in approximation[factor].distribution_parameters.items():
            close(param.grad.cpu(), g[f"grad_{factor}_{pname}"])
