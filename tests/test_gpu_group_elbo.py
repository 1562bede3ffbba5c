"""
The ELBO forward run by the site group's launch (``mi_group_elbo_forward``, ABI 13): for the README
model (README.md:40-69 -- theta ~ Beta(2, 2), x ~ Bernoulli(theta)[n], guide Beta(c1, c0)) the
Bernoulli BCAST launch carries the prior (mi_prior), the Beta draws' implicit-gradient factors
(mi_side) and now the ELBO's reduction and tail, so the step's forward and backward are the guide's
draw plus ONE kernel (``mi_elbo_forward`` / ``mi_elbo_backward`` are not launched).

* loss and gradients equal the two-launch path (MININF_AMD_GROUP_ELBO=0) to 1e-6 over several Adam
  steps, for particle counts within one 256-particle chunk, ragged, and the bench's 4096;
* invalid data raises the reference's message; a non-unit upstream launches the backward, which
  reads the sums the fused launch saved;
* captured replays (several steps per replay) equal eager steps.
"""
import pytest
import torch
from torch.distributions import Bernoulli, Beta

import mininf_amd as mi
from mininf_amd import _native as nat
from mininf_amd.graph import StepGraph
from mininf_amd.optim import Adam

pytestmark = pytest.mark.gpu


def _spy(monkeypatch, name):
    lib = nat.lib()
    real = getattr(lib, name)
    calls = []

    def spy(*args):
        calls.append(1)
        return real(*args)
    monkeypatch.setattr(lib, name, spy)
    return calls


def _setup(device, n, K, seed=3):
    gen = torch.Generator().manual_seed(seed)
    x = (torch.rand(n, generator=gen) < 0.3).float().to(device)

    def model():
        theta = mi.sample("theta", Beta(2.0, 2.0))
        mi.sample("x", Bernoulli(theta), sample_shape=[n])

    module = mi.nn.ParameterizedDistribution(Beta, concentration1=3.0,
                                             concentration0=5.0).to(device)
    return mi.condition(model, x=x), module, mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=7)


def _run(device, monkeypatch, fused, n, K, steps=3):
    monkeypatch.setenv("MININF_AMD_GROUP_ELBO", "1" if fused else "0")
    cond, module, loss_fn = _setup(device, n, K)
    optimizer = Adam(module.parameters(), lr=0.02)
    out = []
    for _ in range(steps):
        optimizer.zero_grad(set_to_none=True)
        loss = loss_fn(cond, {"theta": module()})
        loss.backward()
        out.append((float(loss), [q.grad.clone() for q in module.parameters()]))
        optimizer.step()
    torch.cuda.synchronize()
    return out, [q.detach().clone() for q in module.parameters()], loss_fn.last_fusions


@pytest.mark.parametrize("n,K,takes", [(50_000, 256, True), (123_457, 1000, True),
                                       (1_000_000, 4096, True),
                                       (4096, 64, False)])   # one chunk: no rank-one slot layout
def test_fused_forward_matches_two_launches(device, monkeypatch, n, K, takes):
    fwd = _spy(monkeypatch, "mi_elbo_forward")
    bwd = _spy(monkeypatch, "mi_elbo_backward")
    fused_calls = _spy(monkeypatch, "mi_group_elbo_forward")
    fused, params_f, fusions = _run(device, monkeypatch, True, n, K)
    if takes:
        assert fwd == [] and bwd == [] and len(fused_calls) == 3, "one site kernel per step expected"
        assert fusions["group_elbo"] == 1 and fusions["folded_priors"] == 1
    else:
        assert fused_calls == [] and len(fwd) == 3 and fusions["group_elbo"] == 0
    fwd.clear()
    plain, params_p, _ = _run(device, monkeypatch, False, n, K)
    assert len(fwd) == 3
    for (lf, gf), (lp, gp) in zip(fused, plain):
        assert lf == pytest.approx(lp, rel=1e-6, abs=1e-6)
        for a, b in zip(gf, gp):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6 * float(b.abs().max()))
    for a, b in zip(params_f, params_p):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)


def test_invalid_data_raises(device, monkeypatch):
    monkeypatch.setenv("MININF_AMD_GROUP_ELBO", "1")
    cond, module, loss_fn = _setup(device, 10_000, 256)

    def model():
        theta = mi.sample("theta", Beta(2.0, 2.0))
        mi.sample("x", Bernoulli(theta), sample_shape=[10_000])

    bad = torch.zeros(10_000, device=device)
    bad[123] = 2.0
    fused_calls = _spy(monkeypatch, "mi_group_elbo_forward")
    with pytest.raises(ValueError, match="not in the support"):
        loss_fn(mi.condition(model, x=bad), {"theta": module()})
    assert len(fused_calls) == 1


def test_non_unit_upstream_launches_the_backward(device, monkeypatch):
    monkeypatch.setenv("MININF_AMD_GROUP_ELBO", "1")
    cond, module, loss_fn = _setup(device, 20_000, 512)
    bwd = _spy(monkeypatch, "mi_elbo_backward")
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
        torch.testing.assert_close(g, 2 * u, rtol=1e-6, atol=1e-7)


def test_captured_fused_steps_match_eager(device, monkeypatch):
    monkeypatch.setenv("MININF_AMD_GROUP_ELBO", "1")
    eager, eager_params, _ = _run(device, monkeypatch, True, 100_000, 1024, steps=9)
    cond, module, loss_fn = _setup(device, 100_000, 1024)
    optimizer = Adam(module.parameters(), lr=0.02)

    def step():
        optimizer.zero_grad(set_to_none=True)
        loss = loss_fn(cond, {"theta": module()})
        loss.backward()
        optimizer.step()
        return loss

    graph = StepGraph(step, warmup=3, repeat=3)
    losses = [float(graph()) for _ in range(2)]
    graph.check()
    assert losses[0] == pytest.approx(eager[5][0], rel=1e-6)
    assert losses[1] == pytest.approx(eager[8][0], rel=1e-6)
    for a, b in zip(module.parameters(), eager_params):
        torch.testing.assert_close(a.detach(), b, rtol=1e-6, atol=1e-7)
