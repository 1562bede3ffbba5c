"""
The regression's guide draw made by the linear site launch (``mi_linear.draw``,
``engine.claim_linear_draws``): ``theta ~ q(theta)`` (a small mean-field Normal factor,
examples/minibatch.md) is drawn by the ``X @ theta`` site kernel instead of a ``mi_normal_rsample``
launch before it.

* the step equals the separate draw (MININF_AMD_DRAW_IN_LINEAR=0) bit for bit -- loss and
  gradients -- with and without a device minibatch, for one and several particle groups, ragged K
  and a deferred exp transform of the scale;
* the separate draw is not launched when the linear launch takes it, and is launched when anything
  else reads the draw first: the prior over theta evaluated by its own launch (not folded), or the
  model's own torch operations on theta during the trace;
* a captured step replays the fused draw like eager steps.
"""
import pytest
import torch
from torch.distributions import Normal

import mininf_amd
from mininf_amd import guide as guide_mod
from mininf_amd.graph import StepGraph
from mininf_amd.nn import EvidenceLowerBoundLoss, ParameterizedDistribution

pytestmark = pytest.mark.gpu


def _data(device, n=8192, p=32):
    gen = torch.Generator().manual_seed(5)
    X = torch.randn(n, p, generator=gen)
    y = X @ torch.randn(p, generator=gen) + torch.randn(n, generator=gen)
    return X.to(device), y.to(device)


def _model(n, p, reads_theta=False):
    def model():
        theta = mininf_amd.sample("theta", Normal(0, 1), sample_shape=p)
        with mininf_amd.batch(n):
            with mininf_amd.no_log_prob():
                Xs = mininf_amd.sample("X", Normal(0, 1), sample_shape=(n, p))
            scale = 1.0 + 0.0 * theta.abs().sum() if reads_theta else 1.0
            mininf_amd.sample("y", Normal(Xs @ theta, scale))
    return model


def _launches(monkeypatch):
    calls = []
    real = guide_mod.PendingDraw.launch

    def spy(self):
        if not self.done:
            calls.append(tuple(self.z.shape))
        return real(self)

    monkeypatch.setattr(guide_mod.PendingDraw, "launch", spy)
    return calls


def _step(device, monkeypatch, fused, K=64, minibatch=False, fold=True, reads_theta=False,
          steps=2):
    monkeypatch.setenv("MININF_AMD_DRAW_IN_LINEAR", "1" if fused else "0")
    monkeypatch.setenv("MININF_AMD_FOLD_PRIOR", "1" if fold else "0")
    X, y = _data(device)
    n, p = X.shape
    gen = torch.Generator().manual_seed(9)
    module = ParameterizedDistribution(Normal, loc=0.1 * torch.randn(p, generator=gen),
                                       scale=torch.rand(p, generator=gen) + 0.5).to(device)
    loss_fn = EvidenceLowerBoundLoss(num_particles=K, seed=2)
    loader = mininf_amd.DeviceDataLoader(X, y, batch_size=1024, shuffle=True, drop_last=True,
                                         seed=7) if minibatch else None
    out = []
    for _ in range(steps):   # the second step draws from the advanced counter
        Xb, yb = loader.next() if loader is not None else (X, y)
        loss = loss_fn(mininf_amd.condition(_model(n, p, reads_theta), X=Xb, y=yb),
                       {"theta": module()})
        loss.backward()
        out.append((float(loss), [q.grad.clone() for q in module.parameters()]))
        for q in module.parameters():
            q.grad = None
    torch.cuda.synchronize()
    return out


def _same(a, b):
    for (la, ga), (lb, gb) in zip(a, b):
        assert la == lb
        for x, z in zip(ga, gb):
            torch.testing.assert_close(x, z, rtol=0, atol=0)


@pytest.mark.parametrize("K", [64, 40, 256])
@pytest.mark.parametrize("minibatch", [False, True])
def test_linear_draw_matches_separate_draw(device, monkeypatch, K, minibatch):
    calls = _launches(monkeypatch)
    fused = _step(device, monkeypatch, True, K=K, minibatch=minibatch)
    assert calls == []   # every step's theta drawn by the linear launch
    plain = _step(device, monkeypatch, False, K=K, minibatch=minibatch)
    _same(fused, plain)


def test_unfolded_prior_launches_the_draw_first(device, monkeypatch):
    calls = _launches(monkeypatch)
    fused = _step(device, monkeypatch, True, fold=False)
    assert calls == [(64, 32)] * 2   # the prior's own launch reads theta before the linear site
    plain = _step(device, monkeypatch, False, fold=False)
    _same(fused, plain)


def test_model_reading_theta_flushes_the_draw(device, monkeypatch):
    calls = _launches(monkeypatch)
    fused = _step(device, monkeypatch, True, reads_theta=True)
    assert len(calls) == 2   # launched by the trace's first read, one per step
    plain = _step(device, monkeypatch, False, reads_theta=True)
    _same(fused, plain)


def test_captured_linear_draw_matches_eager(device, monkeypatch):
    monkeypatch.setenv("MININF_AMD_DRAW_IN_LINEAR", "1")
    X, y = _data(device)
    n, p = X.shape

    def run(captured):
        gen = torch.Generator().manual_seed(9)
        module = ParameterizedDistribution(Normal, loc=0.1 * torch.randn(p, generator=gen),
                                           scale=torch.rand(p, generator=gen) + 0.5).to(device)
        optimizer = mininf_amd.optim.Adam(module.parameters(), lr=0.01)
        loss_fn = EvidenceLowerBoundLoss(num_particles=64, seed=4)
        loader = mininf_amd.DeviceDataLoader(X, y, batch_size=1024, shuffle=True,
                                             drop_last=True, seed=3)

        def step():
            optimizer.zero_grad(set_to_none=False)
            Xb, yb = loader.next()
            loss = loss_fn(mininf_amd.condition(_model(n, p), X=Xb, y=yb), {"theta": module()})
            loss.backward()
            optimizer.step()
            return loss

        losses = []
        if captured:   # two eager warm-up steps, then three replays of two steps each
            graph = StepGraph(step, warmup=2, repeat=2)
            for _ in range(3):
                losses.append(float(graph()))
            graph.check()
        else:
            for i in range(8):
                loss = step()
                if i >= 2 and i % 2 == 1:
                    losses.append(float(loss))
        torch.cuda.synchronize()
        return losses, [q.detach().clone() for q in module.parameters()]

    le, pe = run(False)
    lc, pc = run(True)
    assert le == pytest.approx(lc, rel=1e-6)
    for a, b in zip(pe, pc):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
