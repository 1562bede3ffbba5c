"""
Prior sites folded into the likelihood's launch (``mi_prior``, ``engine.fold_priors``): the README
model's ``theta ~ Beta(2, 2)`` under ``x ~ Bernoulli(theta)`` (README.md:43-47) evaluated by the
Bernoulli BCAST kernel's particle-constant workgroups instead of a launch of its own.

* the folded step equals the unfolded one (MININF_AMD_FOLD_PRIOR=0) -- loss and gradients, for
  Beta, Normal and Gamma priors on the probability / logit;
* validation words keep the model order: invalid data of the likelihood is reported for its own
  site, a prior value outside its support for the prior's;
* the folded step launches one site kernel fewer.
"""
import pytest
import torch
from torch.distributions import Bernoulli, Beta, Gamma, Normal

import mininf_amd
from mininf_amd import engine
from mininf_amd.nn import EvidenceLowerBoundLoss, ParameterizedDistribution

pytestmark = pytest.mark.gpu

N, K = 20_000, 512


def _step(device, monkeypatch, fold, prior, logits=False, x=None):
    monkeypatch.setenv("MININF_AMD_FOLD_PRIOR", "1" if fold else "0")
    gen = torch.Generator().manual_seed(3)
    if x is None:
        x = (torch.rand(N, generator=gen) < 0.3).float()
    x = x.to(device)

    def model():
        if logits:
            t = mininf_amd.sample("theta", prior)
            mininf_amd.sample("x", Bernoulli(logits=t), sample_shape=[N])
        else:
            t = mininf_amd.sample("theta", prior)
            mininf_amd.sample("x", Bernoulli(t), sample_shape=[N])

    if logits:
        guide = ParameterizedDistribution(Normal, loc=-0.5, scale=0.3).to(device)
    else:
        guide = ParameterizedDistribution(Beta, concentration1=3.0, concentration0=5.0).to(device)
    loss_fn = EvidenceLowerBoundLoss(num_particles=K, seed=11)
    loss = loss_fn(mininf_amd.condition(model, x=x), {"theta": guide()})
    loss.backward()
    torch.cuda.synchronize()
    return float(loss), [p.grad.clone() for p in guide.parameters()]


@pytest.mark.parametrize("prior, logits", [
    (Beta(2.0, 2.0), False),
    (Gamma(2.0, 3.0), False),
    (Normal(0.0, 1.5), True),
])
def test_folded_prior_matches_separate_launch(device, monkeypatch, prior, logits):
    lf, gf = _step(device, monkeypatch, True, prior, logits)
    lu, gu = _step(device, monkeypatch, False, prior, logits)
    assert lf == pytest.approx(lu, rel=1e-6)
    for a, b in zip(gf, gu):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-7)


def test_prior_is_folded(device, monkeypatch):
    calls = []
    real = engine.fold_priors

    def spy(launchers):
        out = real(launchers)
        calls.append((len(launchers), len(out), [l.prior is not None for l in out]))
        return out

    monkeypatch.setattr(engine, "fold_priors", spy)
    _step(device, monkeypatch, True, Beta(2.0, 2.0))
    assert calls == [(2, 1, [True])]


def test_folded_prior_reports_the_likelihood_site(device, monkeypatch):
    x = torch.zeros(N)
    x[7] = 2.0   # outside Bernoulli's support
    with pytest.raises(ValueError, match="'x'"):
        _step(device, monkeypatch, True, Beta(2.0, 2.0), x=x)


def test_folded_prior_reports_its_own_support(device, monkeypatch):
    # a Normal guide on a probability: draws below 0 leave Beta's support [0, 1]; the error names
    # the prior site, as the separate launch does
    monkeypatch.setenv("MININF_AMD_FOLD_PRIOR", "1")
    x = (torch.rand(N, generator=torch.Generator().manual_seed(1)) < 0.3).float().to(device)

    def model():
        t = mininf_amd.sample("theta", Beta(2.0, 2.0))
        mininf_amd.sample("x", Bernoulli(logits=t), sample_shape=[N])

    guide = ParameterizedDistribution(Normal, loc=-3.0, scale=0.1).to(device)
    loss_fn = EvidenceLowerBoundLoss(num_particles=K, seed=1)
    with pytest.raises(ValueError, match="'theta'"):
        loss_fn(mininf_amd.condition(model, x=x), {"theta": guide()})


def _regression(device, monkeypatch, fold, minibatch):
    """C3 / C4-shaped regression (examples/minibatch.md): theta ~ Normal(0, 1) under the fused
    linear site, over a device minibatch when `minibatch`."""
    monkeypatch.setenv("MININF_AMD_FOLD_PRIOR", "1" if fold else "0")
    gen = torch.Generator().manual_seed(5)
    n, p, K = 8192, 32, 64
    X = torch.randn(n, p, generator=gen)
    y = X @ torch.randn(p, generator=gen) + torch.randn(n, generator=gen)
    X, y = X.to(device), y.to(device)

    def model():
        theta = mininf_amd.sample("theta", Normal(0, 1), sample_shape=p)
        with mininf_amd.batch(n):
            with mininf_amd.no_log_prob():
                Xs = mininf_amd.sample("X", Normal(0, 1), sample_shape=(n, p))
            mininf_amd.sample("y", Normal(Xs @ theta, 1))

    guide = ParameterizedDistribution(Normal, loc=torch.zeros(p), scale=torch.ones(p)).to(device)
    loss_fn = EvidenceLowerBoundLoss(num_particles=K, seed=2)
    if minibatch:
        loader = mininf_amd.DeviceDataLoader(X, y, batch_size=1024, shuffle=True, drop_last=True,
                                             seed=7)
        Xb, yb = loader.next()
    else:
        Xb, yb = X, y
    loss = loss_fn(mininf_amd.condition(model, X=Xb, y=yb), {"theta": guide()})
    loss.backward()
    torch.cuda.synchronize()
    return float(loss), [q.grad.clone() for q in guide.parameters()]


@pytest.mark.parametrize("minibatch", [False, True])
def test_folded_linear_prior_matches_separate_launch(device, monkeypatch, minibatch):
    folds = []
    real = engine.fold_linear_priors

    def spy(launchers, linears):
        out = real(launchers, linears)
        folds.append([l.prior is not None for l in linears])
        return out

    monkeypatch.setattr(engine, "fold_linear_priors", spy)
    lf, gf = _regression(device, monkeypatch, True, minibatch)
    assert folds == [[True]]
    lu, gu = _regression(device, monkeypatch, False, minibatch)
    assert lf == pytest.approx(lu, rel=1e-6)
    for a, b in zip(gf, gu):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
