"""
Which fast paths an ELBO evaluation takes (EvidenceLowerBoundLoss.last_fusions, reported in the
bench line as config.fusions; VERDICT r03 "What's weak" 8): the planner's fusions fire on
structural patterns, so a model slightly off a pattern silently takes the general path -- these
tests pin what each bench model takes, and that an off-pattern model (a Beta(3, 2) prior over two
observed Bernoulli sites, README.md:40-47 with its data split in two) still evaluates correctly:
loss and gradients against the oracle ELBO on the restated device draws (oracle/philox.c).
"""
import numpy as np
import pytest
import torch
from torch.distributions import Bernoulli, Beta, Normal

import mininf_amd as mi
from mininf_amd.data import DeviceDataLoader
from oracle import build as oracle_build, elbo as oracle

pytestmark = pytest.mark.gpu


def test_readme_model_fusions(device):
    n, K = 20000, 1024
    x = (torch.rand(n, generator=torch.Generator().manual_seed(0)) < 0.7).float().to(device)

    def model():
        theta = mi.sample("theta", Beta(2, 2))
        mi.sample("x", Bernoulli(theta), sample_shape=[n])

    approx = mi.nn.ParameterizedDistribution(Beta, concentration1=2.0,
                                             concentration0=2.0).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K)
    loss_fn(mi.condition(model, x=x), {"theta": approx()}).backward()
    f = loss_fn.last_fusions
    assert f["folded_priors"] == 1 and f["final_grads"] == 1 and f["deferred_reductions"] == 1
    assert f["fused_draws"] == 0


def test_minibatch_regression_fusions(device):
    n, p, B, K = 65536, 32, 4096, 32
    gen = torch.Generator().manual_seed(0)
    X = torch.randn(n, p, generator=gen).to(device)
    y = (X @ torch.randn(p, generator=gen).to(device)) + 0.1

    def model():
        theta = mi.sample("theta", Normal(0, 1), sample_shape=p)
        with mi.batch(n):
            with mi.no_log_prob():
                Xs = mi.sample("X", Normal(0, 1), sample_shape=(n, p))
            mi.sample("y", Normal(Xs @ theta, 1))

    loader = DeviceDataLoader(X, y, batch_size=B, shuffle=True, drop_last=True, seed=0)
    approx = mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(p),
                                             scale=torch.ones(p)).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K)
    Xb, yb = loader.next()
    loss_fn(mi.condition(model, X=Xb, y=yb), {"theta": approx()}).backward()
    f = loss_fn.last_fusions
    assert f["linear_theta_draws"] == 1 and f["linear_rows"] == 1
    assert f["folded_priors"] == 1 and f["final_grads"] == 1


def test_masked_hierarchical_fusions(device):
    n, K = 4096, 64
    rng = np.random.default_rng(0)
    mask = torch.as_tensor(rng.random(n) > 0.2, device=device)
    y = torch.as_tensor(rng.normal(size=n).astype(np.float32), device=device)
    b = torch.as_tensor((rng.random(n) < 0.5).astype(np.float32), device=device)

    def model():
        mu = mi.sample("mu", Normal(0, 1))
        z = mi.sample("z", Normal(mu, 1), sample_shape=[n])
        mi.sample("y", Normal(z, 0.5))
        mi.sample("b", Bernoulli(logits=z))

    approx = mi.nn.ParameterizedFactorizedDistribution(
        mu=mi.nn.ParameterizedDistribution(Normal, loc=0.0, scale=1.0),
        z=mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(n), scale=torch.ones(n)),
    ).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K)
    cond = mi.condition(model, y=torch.masked.as_masked_tensor(y, mask),
                        b=torch.masked.as_masked_tensor(b, mask))
    loss_fn(cond, approx()).backward()
    f = loss_fn.last_fusions
    assert f["fused_draws"] == 1
    # mu ~ Normal(0, 1) is evaluated by the fused-draw program's block-row flush (mi_prior): no
    # launch of its own
    assert f["folded_priors"] == 1


def test_off_pattern_prior_over_two_sites_matches_oracle(device):
    """theta ~ Beta(3, 2) read by two Bernoulli sites (the coin's data split in two): the prior
    can fold into at most one of the two launches; whatever the planner takes, the loss and the
    guide gradients equal the oracle ELBO over the restated device draws at 1e-5."""
    n1, n2, K, seed = 30000, 12345, 2048, 77
    gen = torch.Generator().manual_seed(4)
    x1 = (torch.rand(n1, generator=gen) < 0.6).float()
    x2 = (torch.rand(n2, generator=gen) < 0.6).float()

    def model():
        theta = mi.sample("theta", Beta(3, 2))
        mi.sample("x1", Bernoulli(theta), sample_shape=[n1])
        mi.sample("x2", Bernoulli(theta), sample_shape=[n2])

    approx = mi.nn.ParameterizedDistribution(Beta, concentration1=2.2,
                                             concentration0=1.7).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=seed)
    q = approx()
    loss = loss_fn(mi.condition(model, x1=x1.to(device), x2=x2.to(device)), {"theta": q})
    loss.backward()
    f = loss_fn.last_fusions
    assert f["folded_priors"] <= 1
    c1 = float(q.concentration1.detach().cpu())
    c0 = float(q.concentration0.detach().cpu())
    draws = oracle_build.beta_draws([c1], [c0], K, seed, 0, 0, 0)[0][:, 0]
    ref = oracle.beta_bernoulli_elbo(np.concatenate([x1.numpy(), x2.numpy()]), 3, 2, c1, c0, draws)
    assert abs(float(loss) - ref["loss"]) <= 1e-5 * abs(ref["loss"])
    g = approx.distribution_parameters
    for name in ("concentration1", "concentration0"):
        want = ref[f"grad_u_{name}"]
        assert abs(float(g[name].grad) - want) <= 1e-5 * abs(want), name
