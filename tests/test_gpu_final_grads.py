"""
Final guide gradients written by the ELBO forward (``MI_ELBO_FINAL_GRADS``): for the README model
(``theta ~ Beta`` guide over a Bernoulli likelihood, README.md:43-69) the forward's last block
finishes the Beta factor's particle sums, so for ``loss.backward()`` -- an upstream of exactly 1,
nn._Loss's unit seed -- it also writes the gradients and ``mi_elbo_backward`` is not launched.

* the gradients equal those of the backward launch (MININF_AMD_FINAL_GRADS=0), eager and over
  several steps;
* the backward kernel is skipped for loss.backward() and launched for any other upstream
  (``torch.autograd.grad`` with a non-unit gradient), whose gradients scale accordingly;
* a captured step (StepGraph) replays without the backward kernel and matches eager steps.
"""
import pytest
import torch
from torch.distributions import Bernoulli, Beta, Normal

import mininf_amd
from mininf_amd import _native as nat
from mininf_amd.graph import StepGraph
from mininf_amd.nn import EvidenceLowerBoundLoss, ParameterizedDistribution

pytestmark = pytest.mark.gpu

N, K = 50_000, 1024


def _setup(device, seed=3):
    gen = torch.Generator().manual_seed(seed)
    x = (torch.rand(N, generator=gen) < 0.3).float().to(device)

    def model():
        theta = mininf_amd.sample("theta", Beta(2.0, 2.0))
        mininf_amd.sample("x", Bernoulli(theta), sample_shape=[N])

    guide = ParameterizedDistribution(Beta, concentration1=3.0, concentration0=5.0).to(device)
    return mininf_amd.condition(model, x=x), guide, EvidenceLowerBoundLoss(num_particles=K, seed=7)


def _spy_backward(monkeypatch):
    lib = nat.lib()
    real = lib.mi_elbo_backward
    calls = []

    def spy(*args):
        calls.append(1)
        return real(*args)
    monkeypatch.setattr(lib, "mi_elbo_backward", spy)
    return calls


def _steps(device, monkeypatch, final, steps=3):
    monkeypatch.setenv("MININF_AMD_FINAL_GRADS", "1" if final else "0")
    # the ELBO forward's own tail (the site launch finishing the whole ELBO is
    # test_gpu_group_elbo.py's subject)
    monkeypatch.setenv("MININF_AMD_GROUP_ELBO", "0")
    model, guide, loss_fn = _setup(device)
    out = []
    for _ in range(steps):
        loss = loss_fn(model, {"theta": guide()})
        loss.backward()
        out.append((float(loss), [p.grad.clone() for p in guide.parameters()]))
        for p in guide.parameters():
            p.grad = None
    torch.cuda.synchronize()
    return out


def test_final_grads_match_the_backward_launch(device, monkeypatch):
    calls = _spy_backward(monkeypatch)
    fused = _steps(device, monkeypatch, True)
    assert calls == []            # no mi_elbo_backward for loss.backward()
    plain = _steps(device, monkeypatch, False)
    assert len(calls) == 3
    for (lf, gf), (lp, gp) in zip(fused, plain):
        assert lf == lp
        for a, b in zip(gf, gp):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=0)


def test_other_upstream_launches_the_backward(device, monkeypatch):
    monkeypatch.setenv("MININF_AMD_FINAL_GRADS", "1")
    calls = _spy_backward(monkeypatch)
    model, guide, loss_fn = _setup(device)
    params = list(guide.parameters())
    torch.manual_seed(0)
    loss = loss_fn(model, {"theta": guide()})
    g2 = torch.autograd.grad(loss, params, torch.tensor(2.0, device=device))
    assert calls == [1]
    model, guide, loss_fn = _setup(device)
    loss = loss_fn(model, {"theta": guide()})
    loss.backward()
    assert calls == [1]
    for a, b in zip(g2, guide.parameters()):
        torch.testing.assert_close(a, 2 * b.grad, rtol=1e-6, atol=0)


def test_captured_final_grads_match_eager(device, monkeypatch):
    monkeypatch.setenv("MININF_AMD_FINAL_GRADS", "1")

    def run(captured):
        model, guide, loss_fn = _setup(device)
        optimizer = mininf_amd.optim.Adam(guide.parameters(), lr=0.02)

        def step():
            optimizer.zero_grad(set_to_none=False)
            loss = loss_fn(model, {"theta": guide()})
            loss.backward()
            optimizer.step()
            return loss

        losses = []
        if captured:
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
        return losses, [p.detach().clone() for p in guide.parameters()]

    le, pe = run(False)
    lc, pc = run(True)
    assert le == pytest.approx(lc, rel=1e-6)
    for a, b in zip(pe, pc):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)


def _regression_steps(device, monkeypatch, final, K, minibatch, steps=3):
    """C3 / C4-shaped regression (examples/minibatch.md): the theta factor's gradients finished by
    the ELBO forward from the linear site's slot rows (the Normal tail)."""
    monkeypatch.setenv("MININF_AMD_FINAL_GRADS", "1" if final else "0")
    # the ELBO forward's own Normal tail (the linear launch finishing the whole ELBO is
    # test_gpu_linear_elbo.py's subject)
    monkeypatch.setenv("MININF_AMD_LINEAR_ELBO", "0")
    gen = torch.Generator().manual_seed(5)
    n, p = 8192, 32
    X = torch.randn(n, p, generator=gen)
    y = X @ torch.randn(p, generator=gen) + torch.randn(n, generator=gen)
    X, y = X.to(device), y.to(device)

    def model():
        theta = mininf_amd.sample("theta", Normal(0, 1), sample_shape=p)
        with mininf_amd.batch(n):
            with mininf_amd.no_log_prob():
                Xs = mininf_amd.sample("X", Normal(0, 1), sample_shape=(n, p))
            mininf_amd.sample("y", Normal(Xs @ theta, 1))

    guide = ParameterizedDistribution(Normal, loc=0.1 * torch.randn(p, generator=gen),
                                      scale=torch.rand(p, generator=gen) + 0.5).to(device)
    loss_fn = EvidenceLowerBoundLoss(num_particles=K, seed=2)
    loader = mininf_amd.DeviceDataLoader(X, y, batch_size=1024, shuffle=True, drop_last=True,
                                         seed=7) if minibatch else None
    out = []
    for _ in range(steps):
        Xb, yb = loader.next() if loader is not None else (X, y)
        loss = loss_fn(mininf_amd.condition(model, X=Xb, y=yb), {"theta": guide()})
        loss.backward()
        out.append((float(loss), [q.grad.clone() for q in guide.parameters()]))
        for q in guide.parameters():
            q.grad = None
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("K, minibatch", [(64, False), (256, False), (40, True)])
def test_regression_final_grads_match_the_backward_launch(device, monkeypatch, K, minibatch):
    calls = _spy_backward(monkeypatch)
    fused = _regression_steps(device, monkeypatch, True, K, minibatch)
    assert calls == []
    plain = _regression_steps(device, monkeypatch, False, K, minibatch)
    assert len(calls) == 3
    for (lf, gf), (lp, gp) in zip(fused, plain):
        assert lf == lp
        for a, b in zip(gf, gp):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)


def _masked_steps(device, monkeypatch, final, n=20000, K=64, steps=3, shard=None):
    """The masked hierarchical model (examples/missing-observations.md restated, C5): z drawn in
    registers by the site program (MI_DRAW_PARTIALS), mu a one-element Normal factor whose sources
    are the program's slot and the prior site's slot."""
    monkeypatch.setenv("MININF_AMD_FINAL_GRADS", "1" if final else "0")
    import numpy as np
    rng = np.random.default_rng(0)
    mask = torch.as_tensor(rng.random(n) > 0.2, device=device)
    y = torch.as_tensor(rng.normal(size=n).astype(np.float32), device=device)
    b = torch.as_tensor((rng.random(n) < 0.5).astype(np.float32), device=device)

    def model():
        mu = mininf_amd.sample("mu", Normal(0.0, 1.0))
        z = mininf_amd.sample("z", Normal(mu, 1.0), sample_shape=[n])
        mininf_amd.sample("y", Normal(z, 0.5))
        mininf_amd.sample("b", Bernoulli(logits=z))

    guide = mininf_amd.nn.ParameterizedFactorizedDistribution(
        mu=ParameterizedDistribution(Normal, loc=0.3, scale=0.8),
        z=ParameterizedDistribution(Normal, loc=torch.linspace(-1, 1, n),
                                    scale=torch.linspace(0.5, 1.5, n))).to(device)
    loss_fn = EvidenceLowerBoundLoss(num_particles=K, seed=4)
    cond = mininf_amd.condition(model, y=torch.masked.as_masked_tensor(y, mask),
                                b=torch.masked.as_masked_tensor(b, mask))
    out = []
    for _ in range(steps):
        loss = loss_fn(cond, guide())
        loss.backward()
        out.append((float(loss), [q.grad.clone() for q in guide.parameters()]))
        for q in guide.parameters():
            q.grad = None
    torch.cuda.synchronize()
    return out, loss_fn.last_fusions


def test_masked_model_final_grads_match_the_backward_launch(device, monkeypatch):
    """The forward finishes the fused-draw factor (its backward blocks run inside the forward
    launch) and the one-element mu (the Normal tail over every job's slot): no backward launch."""
    calls = _spy_backward(monkeypatch)
    fused, fusions = _masked_steps(device, monkeypatch, True)
    assert calls == [] and fusions["final_grads"] == 1 and fusions["fused_draws"] == 1
    plain, _ = _masked_steps(device, monkeypatch, False)
    assert len(calls) == 3
    for (lf, gf), (lp, gp) in zip(fused, plain):
        assert lf == lp
        for a, b in zip(gf, gp):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6 * float(b.abs().max()))


@pytest.mark.parametrize("set_to_none", [True, False])
def test_direct_accumulation_matches_autograd(device, monkeypatch, set_to_none):
    """nn._Loss.backward hands the forward's final gradients to the leaf parameters itself
    (MININF_AMD_DIRECT_GRADS, no autograd engine): the same gradients as the engine's
    AccumulateGrad, assigned or accumulated into existing .grad tensors."""
    def run(direct):
        monkeypatch.setenv("MININF_AMD_DIRECT_GRADS", "1" if direct else "0")
        model, guide, loss_fn = _setup(device)
        params = list(guide.parameters())
        out = []
        for _ in range(2):
            if set_to_none:
                for p in params:
                    p.grad = None
            loss = loss_fn(model, {"theta": guide()})
            loss.backward()
            out.append([p.grad.clone() for p in params])
        return out

    direct, engine = run(True), run(False)
    for gd, ge in zip(direct, engine):
        for a, b in zip(gd, ge):
            torch.testing.assert_close(a, b, rtol=0, atol=0)


def test_direct_accumulation_keeps_tensor_hooks(device, monkeypatch):
    """A hook on a parameter sends the backward through the autograd engine (the hook runs)."""
    monkeypatch.setenv("MININF_AMD_DIRECT_GRADS", "1")
    model, guide, loss_fn = _setup(device)
    seen = []
    p0 = next(iter(guide.parameters()))
    p0.register_hook(lambda g: seen.append(1))
    loss = loss_fn(model, {"theta": guide()})
    loss.backward()
    assert seen == [1]
