"""
The masked hierarchical model's global parameter (examples/missing-observations.md:33-45: mu
~ Normal(0, 1), z ~ Normal(mu, 1)[n]) inside the fused-draw site program:

* mu's prior site is evaluated by the program's block-row flush (mi_group.prior on site 0's
  per-particle parameter) instead of a launch of its own: loss and gradients equal the unfolded
  path (MININF_AMD_FOLD_PRIOR=0) at 1e-6;
* mu's K draws are made by the program (mi_group.pdraw: the mi_normal_rsample normals and fmaf,
  bit-identical) instead of a mi_normal_rsample launch before it: the same loss, gradients and
  written draws as the separate launch (MININF_AMD_DRAW_IN_LINEAR=0 keeps every draw its own
  launch), eager and under graph replay.

Both fusions are checked against the oracle (not only against the unfused path) at full size by
test_gpu_fullsize.py::test_c5_fused_draw_full_size_against_oracle, which asserts that both were
active (last_fusions: program_draws, folded_priors) in the evaluation it compares at 1e-5.
"""
import numpy as np
import pytest
import torch
from torch.distributions import Bernoulli, Normal

import mininf_amd as mi
from mininf_amd import _native as nat
from mininf_amd.graph import StepGraph

pytestmark = pytest.mark.gpu


def _model(device, n=4096, K=64, seed=3):
    gen = torch.Generator().manual_seed(seed)
    y = torch.randn(n, generator=gen).to(device)
    b = (torch.rand(n, generator=gen) < 0.4).float().to(device)
    mask = (torch.rand(n, generator=gen) > 0.2).to(device)

    def model():
        mu = mi.sample("mu", Normal(0.0, 1.0))
        z = mi.sample("z", Normal(mu, 1.0), sample_shape=[n])
        mi.sample("y", Normal(z, 0.5))
        mi.sample("b", Bernoulli(logits=z))

    guide = mi.nn.ParameterizedFactorizedDistribution(
        mu=mi.nn.ParameterizedDistribution(Normal, loc=0.3, scale=0.8),
        z=mi.nn.ParameterizedDistribution(Normal, loc=torch.linspace(-1, 1, n),
                                          scale=torch.linspace(0.2, 0.9, n))).to(device)
    cond = mi.condition(model, y=torch.masked.as_masked_tensor(y, mask),
                        b=torch.masked.as_masked_tensor(b, mask))
    return guide, cond, K


def _spy(monkeypatch, name):
    lib = nat.lib()
    real = getattr(lib, name)
    calls = []

    def spy(*args):
        calls.append(args)
        return real(*args)
    monkeypatch.setattr(lib, name, spy)
    return calls


def _steps(device, steps=3, **env):
    import os
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        guide, cond, K = _model(device)
        loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=11)
        opt = mi.optim.Adam(guide.parameters(), lr=0.05)
        losses, grads = [], []
        for _ in range(steps):
            opt.zero_grad(set_to_none=True)
            loss = loss_fn(cond, guide())
            loss.backward()
            grads.append([p.grad.detach().clone() for p in guide.parameters()])
            opt.step()
            losses.append(float(loss))
        return losses, grads, [p.detach().clone() for p in guide.parameters()], loss_fn.last_fusions
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_program_makes_the_global_draw(device, monkeypatch):
    calls = _spy(monkeypatch, "mi_normal_rsample_exp")
    plain = _spy(monkeypatch, "mi_normal_rsample")
    losses, grads, params, fusions = _steps(device)
    assert calls == [] and plain == [], "mu's draw ran in the site program"
    assert fusions["fused_draws"] == 1 and fusions["folded_priors"] == 1
    assert fusions["program_draws"] == 1
    ref_losses, ref_grads, ref_params, _ = _steps(device, MININF_AMD_DRAW_IN_LINEAR="0")
    assert losses == ref_losses
    for a, b in zip(grads, ref_grads):
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    for a, b in zip(params, ref_params):
        assert torch.equal(a, b)


def test_folded_prior_matches_its_own_launch(device):
    losses, grads, _, fusions = _steps(device, steps=1)
    assert fusions["folded_priors"] == 1
    ref_losses, ref_grads, _, ref_fusions = _steps(device, steps=1, MININF_AMD_FOLD_PRIOR="0")
    assert ref_fusions["folded_priors"] == 0
    assert losses[0] == pytest.approx(ref_losses[0], rel=1e-6)
    for x, y in zip(grads[0], ref_grads[0]):
        np.testing.assert_allclose(x.cpu().numpy(), y.cpu().numpy(), rtol=1e-5, atol=1e-6)


def test_program_draw_under_graph_replay(device):
    """Captured steps (three per replay): the program's draw reads the generator step from the
    device word the ELBO forward advances, so every replay draws anew -- the replayed losses and
    parameters equal eager steps with the separate draw launch."""
    import os
    ref_losses, _, ref_params, _ = _steps(device, steps=6, MININF_AMD_DRAW_IN_LINEAR="0")
    guide, cond, K = _model(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=11)
    opt = mi.optim.Adam(guide.parameters(), lr=0.05)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = loss_fn(cond, guide())
        loss.backward()
        opt.step()
        return loss

    # warm-up: 3 eager steps, then replays of 3 captured steps
    graph = StepGraph(step, warmup=3, repeat=3)
    loss = float(graph())
    graph.check()
    assert loss == pytest.approx(ref_losses[5], rel=1e-6)
    for a, b in zip(guide.parameters(), ref_params):
        torch.testing.assert_close(a.detach(), b, rtol=1e-6, atol=1e-6)
    assert os.environ.get("MININF_AMD_DRAW_IN_LINEAR") is None
