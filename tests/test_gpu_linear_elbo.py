"""
The ELBO forward run by the linear site's launch (``mi_linear_elbo_forward``, ABI 13): for the
minibatch regression (examples/minibatch.md:76-88 -- one linear site ``y ~ Normal(X @ theta, 1)``
over a device minibatch, the prior ``theta ~ Normal(0, 1)`` folded into the launch, theta the
guide's Normal draw made by the launch) the launch's last blocks reduce its partials and run the
ELBO tail, so the step's forward and backward are ONE kernel (``mi_elbo_forward`` and
``mi_elbo_backward`` are not launched).

* loss and gradients equal the two-launch path (MININF_AMD_LINEAR_ELBO=0) to 1e-6, over several
  Adam steps, for particle counts from one to eight 32-particle tiles and P = 32 / 64;
* the validation words reach the host (an invalid value raises the reference's message), also
  through the mirror of a captured step;
* a non-unit upstream still launches the backward, which reads what the fused launch wrote;
* captured replays (several steps per replay) equal eager steps.
"""
import pytest
import torch
from torch.distributions import Normal

import mininf_amd as mi
from mininf_amd import _native as nat
from mininf_amd.data import DeviceDataLoader
from mininf_amd.graph import StepGraph
from mininf_amd.optim import Adam

pytestmark = pytest.mark.gpu


def _problem(device, n=16384, p=32, seed=3):
    gen = torch.Generator().manual_seed(seed)
    X = torch.randn(n, p, generator=gen)
    y = X @ torch.randn(p, generator=gen) + torch.randn(n, generator=gen)

    def model():
        theta = mi.sample("theta", Normal(0, 1), sample_shape=p)
        with mi.batch(n):
            with mi.no_log_prob():
                Xs = mi.sample("X", Normal(0, 1), sample_shape=(n, p))
            mi.sample("y", Normal(Xs @ theta, 1))

    return model, X.to(device), y.to(device)


def _spy(monkeypatch, name):
    lib = nat.lib()
    real = getattr(lib, name)
    calls = []

    def spy(*args):
        calls.append(1)
        return real(*args)
    monkeypatch.setattr(lib, name, spy)
    return calls


def _run(device, monkeypatch, fused, K=32, p=32, steps=3, batch=2048, minibatch=True):
    monkeypatch.setenv("MININF_AMD_LINEAR_ELBO", "1" if fused else "0")
    n = 16384
    model, X, y = _problem(device, n=n, p=p)
    gen = torch.Generator().manual_seed(1)
    module = mi.nn.ParameterizedDistribution(
        Normal, loc=1e-2 * torch.randn(p, generator=gen),
        scale=(1e-2 * torch.randn(p, generator=gen)).exp()).to(device)
    optimizer = Adam(module.parameters(), lr=0.01)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=5)
    loader = DeviceDataLoader(X, y, batch_size=batch, shuffle=True, drop_last=True, seed=2)
    static = mi.condition(model, X=X, y=y)
    out = []
    for _ in range(steps):
        optimizer.zero_grad(set_to_none=True)
        if minibatch:
            Xb, yb = loader.next()
            cond = mi.condition(model, X=Xb, y=yb)
        else:
            cond = static
        loss = loss_fn(cond, {"theta": module()})
        loss.backward()
        out.append((float(loss), [q.grad.clone() for q in module.parameters()]))
        optimizer.step()
    torch.cuda.synchronize()
    return out, [q.detach().clone() for q in module.parameters()]


@pytest.mark.parametrize("K,p,takes", [(32, 32, True), (64, 32, True), (40, 32, True),
                                       (32, 64, True), (128, 16, True),
                                       (256, 32, False)])   # slab sums exceed the tail's LDS
def test_fused_forward_matches_two_launches(device, monkeypatch, K, p, takes):
    fwd = _spy(monkeypatch, "mi_elbo_forward")
    bwd = _spy(monkeypatch, "mi_elbo_backward")
    fused_lin = _spy(monkeypatch, "mi_linear_elbo_forward")
    fused, params_f = _run(device, monkeypatch, True, K=K, p=p)
    if takes:
        assert fwd == [] and bwd == [] and len(fused_lin) == 3, "one kernel per step expected"
    else:
        assert fused_lin == [] and len(fwd) == 3, "the library declines: two launches"
    fwd.clear()
    plain, params_p = _run(device, monkeypatch, False, K=K, p=p)
    assert len(fwd) == 3
    for (lf, gf), (lp, gp) in zip(fused, plain):
        assert lf == pytest.approx(lp, rel=1e-6, abs=1e-6)
        for a, b in zip(gf, gp):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6 * float(b.abs().max()))
    for a, b in zip(params_f, params_p):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)


def test_fused_forward_without_minibatch(device, monkeypatch):
    """The whole dataset conditioned directly (C3's shape, small): still one launch."""
    fused_lin = _spy(monkeypatch, "mi_linear_elbo_forward")
    fused, _ = _run(device, monkeypatch, True, K=32, minibatch=False, steps=2)
    plain, _ = _run(device, monkeypatch, False, K=32, minibatch=False, steps=2)
    assert len(fused_lin) == 2
    for (lf, gf), (lp, gp) in zip(fused, plain):
        assert lf == pytest.approx(lp, rel=1e-6)
        for a, b in zip(gf, gp):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6 * float(b.abs().max()))


def test_non_unit_upstream_launches_the_backward(device, monkeypatch):
    monkeypatch.setenv("MININF_AMD_LINEAR_ELBO", "1")
    model, X, y = _problem(device, n=4096)
    module = mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(32),
                                             scale=torch.ones(32)).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=64, seed=9)
    bwd = _spy(monkeypatch, "mi_elbo_backward")
    cond = mi.condition(model, X=X, y=y)
    loss = loss_fn(cond, {"theta": module()})
    loss.backward()
    unit = [q.grad.clone() for q in module.parameters()]
    assert bwd == []
    loss_fn._counter.sub_(1)   # the same draws again
    loss = loss_fn(cond, {"theta": module()})
    grads = torch.autograd.grad(loss, list(module.parameters()),
                                grad_outputs=torch.tensor(2.0, device=device))
    assert len(bwd) == 1
    for g, u in zip(grads, unit):
        torch.testing.assert_close(g, 2 * u, rtol=1e-6, atol=1e-6 * float(u.abs().max()))


def test_fused_forward_reports_invalid_values(device, monkeypatch):
    monkeypatch.setenv("MININF_AMD_LINEAR_ELBO", "1")
    model, X, y = _problem(device, n=4096)
    y = y.clone()
    y[17] = float("nan")
    module = mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(32),
                                             scale=torch.ones(32)).to(device)
    fused_lin = _spy(monkeypatch, "mi_linear_elbo_forward")
    with pytest.raises(ValueError, match="not in the support"):
        mi.nn.EvidenceLowerBoundLoss(num_particles=32)(mi.condition(model, X=X, y=y),
                                                       {"theta": module()})
    assert len(fused_lin) == 1


def test_captured_fused_steps_match_eager(device, monkeypatch):
    monkeypatch.setenv("MININF_AMD_LINEAR_ELBO", "1")
    eager, eager_params = _run(device, monkeypatch, True, K=32, steps=9)

    model, X, y = _problem(device)
    gen = torch.Generator().manual_seed(1)
    module = mi.nn.ParameterizedDistribution(
        Normal, loc=1e-2 * torch.randn(32, generator=gen),
        scale=(1e-2 * torch.randn(32, generator=gen)).exp()).to(device)
    optimizer = Adam(module.parameters(), lr=0.01)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=32, seed=5)
    loader = DeviceDataLoader(X, y, batch_size=2048, shuffle=True, drop_last=True, seed=2)

    def step():
        optimizer.zero_grad(set_to_none=True)
        Xb, yb = loader.next()
        loss = loss_fn(mi.condition(model, X=Xb, y=yb), {"theta": module()})
        loss.backward()
        optimizer.step()
        return loss

    graph = StepGraph(step, warmup=3, repeat=3)   # steps 0-2 eager, replays run 3-5 and 6-8
    losses = []
    for _ in range(2):
        losses.append(float(graph()))
    graph.check()
    assert losses[0] == pytest.approx(eager[5][0], rel=1e-6)
    assert losses[1] == pytest.approx(eager[8][0], rel=1e-6)
    for a, b in zip(module.parameters(), eager_params):
        torch.testing.assert_close(a.detach(), b, rtol=1e-6, atol=1e-7)
