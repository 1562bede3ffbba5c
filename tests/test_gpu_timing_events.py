"""
Timing events around a site kernel (mi_group_forward_deferred / mi_linear_forward_deferred's
`start_event` / `stop_event`) are eager-only (csrc/internal.hpp). Round 5's capture branch recorded
them with hipEventRecordExternal, which returned hipErrorInvalidValue inside a capture and broke
the capture (gpurun_out/dbg1_one.err). Now a launch given events while its stream captures
returns MI_EUNSUPPORTED before enqueuing anything: the step fails to capture with that message,
and the next capture of the same step (no events) replays like the eager step.
"""
import pytest
import torch
from torch.distributions import Bernoulli, Beta, Normal

import mininf_amd as mi
from mininf_amd import engine
from mininf_amd.graph import CaptureError, StepGraph

pytestmark = pytest.mark.gpu


class AlwaysEvents:
    """engine.KERNEL_TIMER that hands out an event pair for every launch, captured or not. torch
    creates an event's hipEvent_t at its first record, so the pool's events are recorded once here,
    outside any capture (as bench.py's EventTimer does)."""
    def __init__(self, count=16):
        self.pool = []
        for _ in range(count):
            start = torch.cuda.Event(enable_timing=True)
            stop = torch.cuda.Event(enable_timing=True)
            start.record()
            stop.record()
            self.pool.append((start, stop))
        torch.cuda.synchronize()
        self.pairs = []

    def pair(self, launcher):
        start, stop = self.pool[len(self.pairs) % len(self.pool)]
        assert start.cuda_event and stop.cuda_event
        self.pairs.append((start, stop))
        return start, stop

    def stamps(self, launcher):
        return None


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


@pytest.mark.parametrize("setup,K", [(coin, 256), (regression, 64)])
def test_events_are_eager_only(device, setup, K):
    conditioned, guide, module = setup(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=5)

    def step():
        module.zero_grad(set_to_none=True)
        loss = loss_fn(conditioned, guide())
        loss.backward()
        return loss

    timer = AlwaysEvents()
    engine.KERNEL_TIMER = timer
    try:
        step()   # eager: the events are recorded around the site kernel
        torch.cuda.synchronize()
        assert timer.pairs
        assert all(s.elapsed_time(e) > 0 for s, e in timer.pairs)
        with pytest.raises(CaptureError, match="unsupported"):
            StepGraph(step, warmup=0)
    finally:
        engine.KERNEL_TIMER = None
    # the failed capture left the process usable: the same step captures and replays
    graph = StepGraph(step, warmup=1)
    graph()
    torch.cuda.synchronize()
    graph.check()
    assert torch.isfinite(graph.output).all()
