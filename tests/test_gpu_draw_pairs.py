"""
The fused-draw site program's paired loop (MININF_AMD_DRAW_PAIRS=1: two particles per iteration as
two independent generator -> density chains, jit.cpp; opt-in, measured slower) against the default
one-particle loop: the same per-particle values in the same summation order, so the loss, every
gradient and the parameters after Adam steps are bit-identical -- an odd particle count (the last
particle's second copy masked out) and a per-particle mu read from memory (no program draw) included.
"""
import os

import pytest
import torch
from torch.distributions import Bernoulli, Normal

import mininf_amd as mi

pytestmark = pytest.mark.gpu


def _steps(device, K, pairs, program_draw, steps=2, n=4096):
    old = {k: os.environ.get(k) for k in ("MININF_AMD_DRAW_PAIRS", "MININF_AMD_DRAW_IN_LINEAR")}
    os.environ["MININF_AMD_DRAW_PAIRS"] = "1" if pairs else "0"
    if not program_draw:
        os.environ["MININF_AMD_DRAW_IN_LINEAR"] = "0"   # mu drawn by its own launch, read per row
    try:
        gen = torch.Generator().manual_seed(7)
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
        loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=13)
        opt = mi.optim.Adam(guide.parameters(), lr=0.05)
        out = []
        for _ in range(steps):
            opt.zero_grad(set_to_none=True)
            loss = loss_fn(cond, guide())
            loss.backward()
            out.append((float(loss), [p.grad.detach().clone() for p in guide.parameters()]))
            opt.step()
        assert loss_fn.last_fusions["fused_draws"] == 1
        assert loss_fn.last_fusions["program_draws"] == int(program_draw)
        return out, [p.detach().clone() for p in guide.parameters()]
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("K,program_draw", [(64, True), (63, True), (33, False)])
def test_paired_loop_matches_the_default_loop(device, K, program_draw):
    paired, p_params = _steps(device, K, True, program_draw)
    single, s_params = _steps(device, K, False, program_draw)
    for (lp, gp), (ls, gs) in zip(paired, single):
        assert lp == ls
        for a, b in zip(gp, gs):
            assert torch.equal(a, b)
    for a, b in zip(p_params, s_params):
        assert torch.equal(a, b)
