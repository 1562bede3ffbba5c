"""
The optimizer step inside the step's last launch (ABI 14): the ELBO forward that writes the final
guide gradients (mi_elbo_forward_adam; the minibatch regression, examples/minibatch.md:76-88, and
the README model, README.md:40-69) is held until the Adam step over its gradients, which then runs
in that launch's last block (csrc/adam_math.hpp, torch's fused-Adam arithmetic).

* parameters and losses are BIT-identical to the held-off path (MININF_AMD_DEFER_STEP=0: the
  finishing launch, then mi_adam_step) over several steps, eager and captured, and mi_adam_step
  is not launched when the step joins;
* any other consumer between the backward and the step (reading a gradient, clipping, torch's own
  Adam, validation) enqueues the launch first: results equal the held-off path.
"""
import pytest
import torch
from torch.distributions import Bernoulli, Beta, Normal

import mininf_amd as mi
from mininf_amd import _native as nat
from mininf_amd import engine
from mininf_amd.data import DeviceDataLoader
from mininf_amd.graph import StepGraph
from mininf_amd.optim import Adam

pytestmark = pytest.mark.gpu


def _spy(monkeypatch, name):
    lib = nat.lib()
    real = getattr(lib, name)
    calls = []

    def spy(*args):
        calls.append(args)
        return real(*args)
    monkeypatch.setattr(lib, name, spy)
    return calls


def _regression(device, validate=False, K=32, p=32, n=16384, batch=2048):
    gen = torch.Generator().manual_seed(3)
    X = torch.randn(n, p, generator=gen)
    y = X @ torch.randn(p, generator=gen) + torch.randn(n, generator=gen)
    X, y = X.to(device), y.to(device)

    def model():
        theta = mi.sample("theta", Normal(0, 1), sample_shape=p)
        with mi.batch(n):
            with mi.no_log_prob():
                Xs = mi.sample("X", Normal(0, 1), sample_shape=(n, p))
            mi.sample("y", Normal(Xs @ theta, 1))

    gen = torch.Generator().manual_seed(1)
    module = mi.nn.ParameterizedDistribution(
        Normal, loc=1e-2 * torch.randn(p, generator=gen),
        scale=(1e-2 * torch.randn(p, generator=gen)).exp()).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=5, validate=validate)
    loader = DeviceDataLoader(X, y, batch_size=batch, shuffle=True, drop_last=True, seed=2)

    def approx():
        return {"theta": module()}

    def conditioned():
        Xb, yb = loader.next()
        return mi.condition(model, X=Xb, y=yb)
    return module, loss_fn, approx, conditioned


def _coin(device, validate=False, n=200_000, K=1024):
    gen = torch.Generator().manual_seed(3)
    x = (torch.rand(n, generator=gen) < 0.3).float().to(device)

    def model():
        theta = mi.sample("theta", Beta(2.0, 2.0))
        mi.sample("x", Bernoulli(theta), sample_shape=[n])

    module = mi.nn.ParameterizedDistribution(Beta, concentration1=3.0,
                                             concentration0=5.0).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=7, validate=validate)
    cond = mi.condition(model, x=x)
    return module, loss_fn, (lambda: {"theta": module()}), (lambda: cond)


def _hierarchical(device, validate=False, n=4096, K=128):
    """The masked hierarchical model's shape (C5, examples/missing-observations.md): mu drawn
    on its own, z ~ q(z) drawn inside the site program (a fused draw), its final gradients
    written by the ELBO forward's final-gradient blocks."""
    gen = torch.Generator().manual_seed(3)
    y = torch.randn(n, generator=gen).to(device)
    b = (torch.rand(n, generator=gen) < 0.4).float().to(device)

    def model():
        mu = mi.sample("mu", Normal(0.0, 1.0))
        z = mi.sample("z", Normal(mu, 1.0), sample_shape=[n])
        mi.sample("y", Normal(z, 0.5))
        mi.sample("b", Bernoulli(logits=z))

    module = mi.nn.ParameterizedFactorizedDistribution(
        mu=mi.nn.ParameterizedDistribution(Normal, loc=0.1, scale=0.7),
        z=mi.nn.ParameterizedDistribution(Normal, loc=torch.linspace(-1, 1, n),
                                          scale=torch.linspace(0.2, 0.9, n))).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=5, validate=validate)
    cond = mi.condition(model, y=y, b=b)
    return module, loss_fn, (lambda: module()), (lambda: cond)


MODELS = {"regression": _regression, "coin": _coin, "hierarchical": _hierarchical}


def _train(device, monkeypatch, name, held, steps=4, between=None, optimizer_cls=Adam,
           validate=False):
    monkeypatch.setenv("MININF_AMD_DEFER_STEP", "1" if held else "0")
    module, loss_fn, approx, conditioned = MODELS[name](device, validate=validate)
    optimizer = optimizer_cls(module.parameters(), lr=0.02)
    losses = []
    for _ in range(steps):
        optimizer.zero_grad(set_to_none=True)
        loss = loss_fn(conditioned(), approx())
        loss.backward()
        if between is not None:
            between(module)
        optimizer.step()
        losses.append(loss.detach())   # (after the step: reading it earlier would enqueue)
    torch.cuda.synchronize()
    assert engine.pending_step() is None
    return torch.stack(losses).cpu(), [q.detach().clone() for q in module.parameters()], \
        loss_fn.last_fusions


@pytest.mark.parametrize("name", ["regression", "coin"])
def test_step_joins_the_held_launch(device, monkeypatch, name):
    adam = _spy(monkeypatch, "mi_adam_step")
    fused = _spy(monkeypatch, "mi_elbo_forward_adam")
    losses, params, fusions = _train(device, monkeypatch, name, held=True)
    assert adam == [], "the optimizer step ran in the held launch"
    assert len(fused) == 4
    assert fusions["optimizer_step"] == 1
    adam.clear()
    fused.clear()
    ref_losses, ref_params, ref_fusions = _train(device, monkeypatch, name, held=False)
    assert len(adam) == 4 and ref_fusions["optimizer_step"] == 0
    assert fused == []
    assert torch.equal(losses, ref_losses)
    for a, b in zip(params, ref_params):
        assert torch.equal(a, b)


@pytest.mark.parametrize("name", ["regression", "coin"])
def test_captured_joined_steps_match_held_off_steps(device, monkeypatch, name):
    ref_losses, ref_params, _ = _train(device, monkeypatch, name, held=False, steps=9)
    monkeypatch.setenv("MININF_AMD_DEFER_STEP", "1")
    module, loss_fn, approx, conditioned = MODELS[name](device, validate=True)
    optimizer = Adam(module.parameters(), lr=0.02)

    def step():
        optimizer.zero_grad(set_to_none=True)
        loss = loss_fn(conditioned(), approx())
        loss.backward()
        optimizer.step()
        return loss

    adam = _spy(monkeypatch, "mi_adam_step")
    graph = StepGraph(step, warmup=3, repeat=3)
    assert adam == []   # warm-up steps and the captured ones: no optimizer launch of their own
    losses = [float(graph()) for _ in range(2)]
    graph.check()
    assert losses[0] == float(ref_losses[5]) and losses[1] == float(ref_losses[8])
    for a, b in zip(module.parameters(), ref_params):
        assert torch.equal(a.detach(), b)


@pytest.mark.parametrize("name", ["regression", "coin"])
def test_consumers_between_backward_and_step(device, monkeypatch, name):
    """Gradient clipping reads the held gradients: the launch runs first, the step on its own."""

    def clip(module):
        torch.nn.utils.clip_grad_norm_(module.parameters(), 0.5)

    adam = _spy(monkeypatch, "mi_adam_step")
    losses, params, _ = _train(device, monkeypatch, name, held=True, between=clip)
    assert len(adam) == 4
    ref_losses, ref_params, _ = _train(device, monkeypatch, name, held=False, between=clip)
    assert torch.equal(losses, ref_losses)
    for a, b in zip(params, ref_params):
        assert torch.equal(a, b)


def test_torch_adam_reads_the_held_gradients(device, monkeypatch):
    losses, params, _ = _train(device, monkeypatch, "regression", held=True,
                               optimizer_cls=torch.optim.Adam)
    ref_losses, ref_params, _ = _train(device, monkeypatch, "regression", held=False,
                                       optimizer_cls=torch.optim.Adam)
    assert torch.equal(losses, ref_losses)
    for a, b in zip(params, ref_params):
        assert torch.equal(a, b)


def test_eager_validation_still_raises(device, monkeypatch):
    monkeypatch.setenv("MININF_AMD_DEFER_STEP", "1")
    module, loss_fn, approx, _ = _coin(device, validate=True, n=10_000, K=256)

    def model():
        theta = mi.sample("theta", Beta(2.0, 2.0))
        mi.sample("x", Bernoulli(theta), sample_shape=[10_000])

    bad = torch.zeros(10_000, device=device)
    bad[77] = 3.0
    with pytest.raises(ValueError, match="not in the support"):
        loss_fn(mi.condition(model, x=bad), approx())
    assert engine.pending_step() is None


def test_gradients_read_before_the_step_are_complete(device, monkeypatch):
    """Reading a held gradient (a copy to the host) enqueues the launch: the values equal the
    held-off path's."""
    seen = []
    _train(device, monkeypatch, "coin", held=True, steps=2,
           between=lambda m: seen.append([q.grad.cpu() for q in m.parameters()]))
    ref = []
    _train(device, monkeypatch, "coin", held=False, steps=2,
           between=lambda m: ref.append([q.grad.cpu() for q in m.parameters()]))
    for a, b in zip(seen, ref):
        for x, y in zip(a, b):
            assert torch.equal(x, y)


@pytest.mark.parametrize("name", ["regression", "coin"])
def test_validated_step_joins_the_held_launch(device, monkeypatch, name):
    """With validation on, the loss reads the step's validation words before returning: that read
    waits for the site launches only -- the held ELBO forward (which writes no word) stays held and
    the optimizer step still joins it. Results equal the held-off path bit for bit."""
    adam = _spy(monkeypatch, "mi_adam_step")
    losses, params, fusions = _train(device, monkeypatch, name, held=True, validate=True)
    assert adam == [] and fusions["optimizer_step"] == 1
    ref_losses, ref_params, _ = _train(device, monkeypatch, name, held=False, validate=True)
    assert torch.equal(losses, ref_losses)
    for a, b in zip(params, ref_params):
        assert torch.equal(a, b)


@pytest.mark.parametrize("name", ["regression", "coin"])
def test_allocator_reuse_between_backward_and_step(device, monkeypatch, name):
    """The round-4 fault's cause, pinned: between loss.backward() and
    optimizer.step() the caching allocator hands out every free block of the sizes the held
    launch's buffers have (the deferred reductions' [K] / [slots, K] outputs, partial slabs,
    workspaces: 512 B .. 16 MB), filled with NaN and kept until after the step. Had the held
    launch dropped one of its buffers, the fill would land in memory it reads, or its stores in a
    NaN tensor: the steps are bit-identical to the held-off path and every NaN tensor is intact."""
    def churn(junk):
        def between(module):
            for nbytes in [1 << j for j in range(9, 25)] * 3:
                junk.append(torch.full((nbytes // 4,), float("nan"), device=device))
        return between

    junk: list = []
    losses, params, fusions = _train(device, monkeypatch, name, held=True, between=churn(junk))
    assert fusions["optimizer_step"] == 1
    torch.cuda.synchronize()
    assert all(bool(torch.isnan(t).all()) for t in junk), "a held launch wrote into freed memory"
    ref_junk: list = []
    ref_losses, ref_params, _ = _train(device, monkeypatch, name, held=False,
                                       between=churn(ref_junk))
    assert torch.equal(losses, ref_losses)
    for a, b in zip(params, ref_params):
        assert torch.equal(a, b)


def test_consumer_on_another_stream_waits_for_the_held_launch(device, monkeypatch):
    """a consumer that reads the held gradients on a side stream after
    side.wait_stream(main) -- recorded before anything flushed the held launch -- is ordered
    after the launch (the flush makes the current stream wait), and an optimizer stepping on that
    stream does not join it: results equal the held-off path."""
    def run(held):
        monkeypatch.setenv("MININF_AMD_DEFER_STEP", "1" if held else "0")
        module, loss_fn, approx, conditioned = _coin(device)
        optimizer = Adam(module.parameters(), lr=0.02)
        side = torch.cuda.Stream()
        grads, losses = [], []
        for _ in range(3):
            optimizer.zero_grad(set_to_none=True)
            loss = loss_fn(conditioned(), approx())
            loss.backward()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                grads.append([q.grad.clone() for q in module.parameters()])
                optimizer.step()
            torch.cuda.current_stream().wait_stream(side)
            losses.append(loss.detach())
        torch.cuda.synchronize()
        assert engine.pending_step() is None
        return torch.stack(losses).cpu(), grads, [q.detach().clone() for q in module.parameters()]

    losses, grads, params = run(True)
    ref_losses, ref_grads, ref_params = run(False)
    assert torch.equal(losses, ref_losses)
    for a, b in zip(grads, ref_grads):
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    for a, b in zip(params, ref_params):
        assert torch.equal(a, b)
