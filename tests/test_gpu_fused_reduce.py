"""
Deferred finalize reductions (mi_group_forward_deferred / mi_linear_forward_deferred, run inside
mi_elbo_forward) against the same reductions launched on their own (MININF_AMD_FUSE_REDUCE=0):
the loss and every guide gradient agree, and the generator advances once per evaluation either way.
"""
import pytest
import torch
from torch.distributions import Bernoulli, Beta, Normal

import mininf_amd as mi

pytestmark = pytest.mark.gpu


def coin(device, n=20000):
    gen = torch.Generator().manual_seed(3)
    x = (torch.rand(n, generator=gen) < 0.3).float().to(device)

    def model():
        theta = mi.sample("theta", Beta(2, 2))
        mi.sample("x", Bernoulli(theta), sample_shape=[n])

    module = mi.nn.ParameterizedDistribution(Beta, concentration0=2.5,
                                             concentration1=1.5).to(device)
    return mi.condition(model, x=x), lambda: {"theta": module()}, module


def regression(device, n=4096, p=8):
    gen = torch.Generator().manual_seed(4)
    X = torch.randn(n, p, generator=gen)
    y = X @ torch.randn(p, generator=gen) + torch.randn(n, generator=gen)

    def model():
        theta = mi.sample("theta", Normal(0, 1), sample_shape=p)
        with mi.no_log_prob():
            Xs = mi.sample("X", Normal(0, 1), sample_shape=(n, p))
        mi.sample("y", Normal(Xs @ theta, 1))

    module = mi.nn.ParameterizedDistribution(Normal, loc=0.1 * torch.randn(p, generator=gen),
                                             scale=torch.ones(p)).to(device)
    return (mi.condition(model, X=X.to(device), y=y.to(device)), lambda: {"theta": module()},
            module)


def evaluate(setup, device, K, fuse, monkeypatch, steps=2):
    monkeypatch.setenv("MININF_AMD_FUSE_REDUCE", "1" if fuse else "0")
    conditioned, guide, module = setup(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=11)
    out = []
    for _ in range(steps):
        module.zero_grad()
        loss = loss_fn(conditioned, guide())
        loss.backward()
        out.append((float(loss), [p.grad.clone() for p in module.parameters()]))
    return out


@pytest.mark.parametrize("setup,K", [(coin, 512), (regression, 64)])
def test_fused_reduce_matches_separate_launches(device, monkeypatch, setup, K):
    fused = evaluate(setup, device, K, True, monkeypatch)
    separate = evaluate(setup, device, K, False, monkeypatch)
    for (lf, gf), (ls, gs) in zip(fused, separate):
        assert lf == pytest.approx(ls, rel=1e-6)
        for a, b in zip(gf, gs):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    # two evaluations, two generator steps: the draws (and so the losses) differ
    assert fused[0][0] != fused[1][0]
