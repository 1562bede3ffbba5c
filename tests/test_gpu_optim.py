"""
mininf_amd.optim.Adam (one mi_adam_step launch per step, csrc/adam.hip) against
torch.optim.Adam(fused=True), whose arithmetic it restates: bit-identical parameters and state
after several steps, with weight decay / maximize, more than one launch's worth of tensors, tensors
spread over many blocks (two-level completion counts), grads that skip a parameter, and inside a
captured graph.
"""
import copy

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


def test_cached_bias_corrections_follow_betas_and_loaded_steps(device):
    """The launch caches the next step's bias corrections in its counter words (keyed by step
    and betas): changed betas, a rewound step count and a reordered tensor list between steps
    still give torch's fused Adam bit for bit."""
    shapes = [(5,), (4096,), (300_000,)]
    ours, ref = make(device, shapes), make(device, shapes)
    opt = Adam(ours, lr=0.01)
    opt_ref = torch.optim.Adam(ref, lr=0.01, fused=True)
    gen = torch.Generator().manual_seed(3)
    for step in range(9):
        if step == 3:
            for o in (opt, opt_ref):
                o.param_groups[0]["betas"] = (0.8, 0.95)
        if step == 5:   # rewind one tensor's step count (as a loaded checkpoint would)
            opt.state[ours[1]]["step"].fill_(1.0)
            opt_ref.state[ref[1]]["step"].fill_(1.0)
        grads = [torch.randn(s, generator=gen).to(device) for s in shapes]
        for k, (a, b, g) in enumerate(zip(ours, ref, grads)):
            skip = step == 6 and k == 0   # the tensor slots shift for one step
            a.grad = None if skip else g.clone()
            b.grad = None if skip else g.clone()
        opt.step()
        opt_ref.step()
        for a, b in zip(ours, ref):
            assert torch.equal(a, b), step
    for a, b in zip(ours, ref):
        assert float(opt.state[a]["step"]) == float(opt_ref.state[b]["step"])


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


@pytest.mark.parametrize("source", ["default", "fused_cpu_mapped"])
def test_loads_a_torch_adam_state_dict(device, source):
    """A torch.optim.Adam state_dict (its default keeps `step` as a host tensor; a checkpoint
    mapped to the CPU moves every state tensor there) loads into this Adam, whose later updates
    stay bit-identical to torch's fused Adam continuing from the same state."""
    shapes = [(), (3,), (1000,), (300_000,)]
    ours, ref, start = make(device, shapes), make(device, shapes), make(device, shapes)
    gen = torch.Generator().manual_seed(2)
    grads = [[torch.randn(s, generator=gen).to(device) for s in shapes] for _ in range(6)]
    opt_start = torch.optim.Adam(start, lr=0.01, fused=source != "default")
    for g in grads[:3]:
        for p, gi in zip(start, g):
            p.grad = gi.clone()
        opt_start.step()
    saved = opt_start.state_dict()
    if source == "fused_cpu_mapped":
        saved = {"state": {k: {n: t.cpu() for n, t in v.items()} for k, v in saved["state"].items()},
                 "param_groups": saved["param_groups"]}
    with torch.no_grad():
        for a, b, s in zip(ours, ref, start):
            a.copy_(s)
            b.copy_(s)
    opt, opt_ref = Adam(ours, lr=0.01), torch.optim.Adam(ref, lr=0.01, fused=True)
    # independent copies: Optimizer.load_state_dict keeps a loaded tensor that already has the
    # parameter's device and dtype (the two optimizers would share their moments)
    opt.load_state_dict(copy.deepcopy(saved))
    # the reference continues as fused Adam (its groups' `fused` comes from the loaded dict)
    ref_saved = copy.deepcopy(saved)
    opt_ref.load_state_dict({"state": ref_saved["state"],
                             "param_groups": [dict(g, fused=True) for g in saved["param_groups"]]})
    for g in grads[3:]:
        for a, b, gi in zip(ours, ref, g):
            a.grad, b.grad = gi.clone(), gi.clone()
        opt.step()
        opt_ref.step()
    for a, b in zip(ours, ref):
        assert torch.equal(a, b)
        sa = opt.state[a]
        assert sa["step"].device == a.device and sa["step"].dtype == torch.float32
        assert float(sa["step"]) == 6.0
