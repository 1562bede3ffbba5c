"""
Deferred X @ theta predictors (mininf_amd.linear) on the host: a Normal / Bernoulli-logits site
whose location is the model's own X @ theta becomes a linear site without the product ever being
computed, and every other use of the product sees its real value.
"""
import pytest
import torch
from torch.distributions import Bernoulli, Normal

import mininf_amd as mi
from mininf_amd import particles
from mininf_amd.linear import DeferredMatmul


@pytest.fixture(autouse=True)
def host_deferral(monkeypatch):
    monkeypatch.setattr(DeferredMatmul, "require_device", False)


def trace(model, K=4, p=3, seed=0):
    theta = torch.randn(K, p, generator=torch.Generator().manual_seed(seed))
    return particles.trace_particles(model, {"theta": theta}, K), theta


def test_linear_site_recorded_without_product():
    X, y = torch.randn(50, 3), torch.randn(50)

    def model():
        theta = mi.sample("theta", Normal(0.0, 1.0), sample_shape=3)
        mi.sample("y", Normal(X @ theta, 1.5))

    t, theta = trace(mi.condition(model, y=y))
    site = next(s for s in t.sites if s.name == "y")
    assert site.linear_X is X
    torch.testing.assert_close(site.linear_theta, theta)
    assert site.tensors[0].shape == (4, 50) and site.tensors[0].stride() == (0, 0)


def test_bernoulli_logits_linear_site():
    X, y = torch.randn(20, 3), (torch.rand(20) < 0.5).float()

    def model():
        theta = mi.sample("theta", Normal(0.0, 1.0), sample_shape=3)
        mi.sample("y", Bernoulli(logits=X @ theta))

    t, _ = trace(mi.condition(model, y=y))
    site = next(s for s in t.sites if s.name == "y")
    assert site.family == "bernoulli_logits" and site.linear_X is X


@pytest.mark.parametrize("use", ["shifted", "probs", "reduced"])
def test_other_uses_materialise(use):
    X, y = torch.randn(30, 3), torch.randn(30)

    def model():
        theta = mi.sample("theta", Normal(0.0, 1.0), sample_shape=3)
        loc = X @ theta
        if use == "shifted":
            mi.sample("y", Normal(loc + 1.0, 1.0))
        elif use == "probs":
            mi.sample("y", Normal(torch.sigmoid(loc), 1.0))
        else:
            mi.sample("y", Normal(loc.sum() * torch.ones(30), 1.0))

    t, theta = trace(mi.condition(model, y=y))
    site = next(s for s in t.sites if s.name == "y")
    assert site.linear_X is None
    real = theta @ X.T
    want = {"shifted": real + 1.0, "probs": torch.sigmoid(real),
            "reduced": real.sum(1, keepdim=True).expand(4, 30)}[use]
    torch.testing.assert_close(site.tensors[0], want)


def test_placeholder_as_non_linear_parameter_materialises():
    X, y = torch.randn(30, 3), torch.randn(30)

    def model():
        theta = mi.sample("theta", Normal(0.0, 1.0), sample_shape=3)
        mi.sample("y", Normal(0.0, (X @ theta).exp()))

    t, theta = trace(mi.condition(model, y=y))
    site = next(s for s in t.sites if s.name == "y")
    assert site.linear_X is None
    torch.testing.assert_close(site.tensors[1], (theta @ X.T).exp())
