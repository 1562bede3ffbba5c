"""
mininf_amd.optim.Adam (one mi_adam_step launch per step, csrc/adam.hip) against
torch.optim.Adam(fused=True), whose arithmetic it restates: bit-identical parameters and state
after several steps, with weight decay / maximize, more than one launch's worth of tensors, tensors
spread over many blocks (two-level completion counts), grads that skip a parameter, and inside a
captured graph.
"""
import pytest
import torch

from mininf_amd.graph import StepGraph
from mininf_amd.optim import Adam

pytestmark = pytest.mark.gpu


def make(device, shapes, seed=0):
    gen = torch.Generator().manual_seed(seed)
    return [torch.randn(s, generator=gen).to(device).requires_grad_() for s in shapes]


@pytest.mark.parametrize("kwargs", [dict(lr=0.01), dict(lr=0.003, weight_decay=0.1),
                                    dict(lr=0.02, betas=(0.8, 0.99), eps=1e-6, maximize=True)])
def test_matches_torch_fused_adam(device, kwargs):
    shapes = [(), (3,), (1000,), (2048, 3), (5,), (700_001,), (1,), (17, 4), (9,), (300_000,)]
    ours, ref = make(device, shapes), make(device, shapes)
    opt = Adam(ours, **kwargs)
    opt_ref = torch.optim.Adam(ref, fused=True, **kwargs)
    gen = torch.Generator().manual_seed(1)
    for step in range(6):
        grads = [torch.randn(s, generator=gen).to(device) for s in shapes]
        for k, (a, b, g) in enumerate(zip(ours, ref, grads)):
            skip = step == 2 and k == 3   # a parameter without a gradient keeps its step
            a.grad = None if skip else g.clone()
            b.grad = None if skip else g.clone()
        opt.step()
        opt_ref.step()
    for a, b in zip(ours, ref):
        assert torch.equal(a, b)
        sa, sb = opt.state[a], opt_ref.state[b]
        assert torch.equal(sa["exp_avg"], sb["exp_avg"])
        assert torch.equal(sa["exp_avg_sq"], sb["exp_avg_sq"])
        assert float(sa["step"]) == float(sb["step"])


def test_captured_steps_advance(device):
    params = make(device, [(4,), (100_000,)])
    ref = make(device, [(4,), (100_000,)])
    opt = Adam(params, lr=0.01)
    opt_ref = torch.optim.Adam(ref, lr=0.01, fused=True)
    grads = [torch.full_like(p, 0.5) for p in params]

    def step():
        for p, g in zip(params, grads):
            p.grad = g
        opt.step()
    captured = StepGraph(step, warmup=2)
    for _ in range(3):
        captured()
    torch.cuda.synchronize()
    for _ in range(2 + 3):
        for p, g in zip(ref, grads):
            p.grad = g.clone()
        opt_ref.step()
    for a, b in zip(params, ref):
        assert torch.equal(a.detach(), b.detach())
    assert float(opt.state[params[1]]["step"]) == 5.0
