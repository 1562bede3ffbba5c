"""
HIP-graph capture of a full training step (mininf_amd.graph.StepGraph): replays must reproduce
eager steps exactly (the guide generator advances through its device counter), and validation
errors found during a replay must surface through check() with the reference's messages.
"""
import pytest
import torch
from torch.distributions import Bernoulli, Beta, Normal

import mininf_amd as mi
from mininf_amd.graph import StepGraph

pytestmark = pytest.mark.gpu


def coin_setup(device, n=5000, K=256):
    gen = torch.Generator().manual_seed(0)
    x = (torch.rand(n, generator=gen) < 0.7).float().to(device)

    def model():
        theta = mi.sample("theta", Beta(2, 2))
        mi.sample("x", Bernoulli(theta), sample_shape=[n])

    module = mi.nn.ParameterizedDistribution(Beta, concentration0=2.0,
                                             concentration1=2.0).to(device)
    optimizer = torch.optim.Adam(module.parameters(), lr=0.02, capturable=True)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=7)
    conditioned = mi.condition(model, x=x)

    def step():
        optimizer.zero_grad(set_to_none=True)
        loss = loss_fn(conditioned, {"theta": module()})
        loss.backward()
        optimizer.step()
        return loss

    return step, module, x


def test_graph_replays_match_eager_steps(device):
    eager_step, eager_module, _ = coin_setup(device)
    graph_body, graph_module, _ = coin_setup(device)
    eager_losses = [float(eager_step()) for _ in range(7)]
    # StepGraph runs 3 eager warm-up steps (steps 0-2); capture records step 3 without executing
    # it; the four replays execute steps 3-6.
    captured = StepGraph(graph_body, warmup=3)
    graph_losses = []
    for _ in range(4):
        graph_losses.append(float(captured()))
    captured.check()
    torch.testing.assert_close(torch.tensor(graph_losses), torch.tensor(eager_losses[3:]),
                               rtol=1e-6, atol=0)
    for a, b in zip(eager_module.parameters(), graph_module.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=0)


def test_failed_capture_leaves_the_process_usable(device):
    """A step that runs an operation a capturing stream refuses (a synchronous copy from pageable
    host memory) raises CaptureError naming the model line; the capture is abandoned, so the
    same process then captures and replays a good step (a failed capture used to
    poison every later test)."""
    from mininf_amd.graph import CaptureError
    step, _, _ = coin_setup(device, n=1000, K=16)
    host = torch.arange(4, dtype=torch.float32)
    calls = []

    def bad_step():
        loss = step()
        if torch.cuda.is_current_stream_capturing():
            calls.append(1)
            host.to(device)   # pageable host-to-device copy: not capturable
        return loss

    with pytest.raises(CaptureError, match="host.to.device"):
        StepGraph(bad_step, warmup=1)
    assert calls == [1]
    assert not torch.cuda.is_current_stream_capturing()
    # the process is usable: plain work, then a fresh capture and replays that match eager steps
    assert float((torch.ones(8, device=device) * 2).sum()) == 16.0
    test_graph_replays_match_eager_steps(device)


def test_multi_step_replays_match_eager_steps(device):
    """StepGraph(repeat=3): each replay runs three full steps (the bench's launch amortisation);
    losses of every third step and the parameters match eager steps."""
    eager_step, eager_module, _ = coin_setup(device)
    graph_body, graph_module, _ = coin_setup(device)
    eager_losses = [float(eager_step()) for _ in range(2 + 3 * 3)]
    captured = StepGraph(graph_body, warmup=2, repeat=3)
    graph_losses = [float(captured()) for _ in range(3)]
    captured.check()
    torch.testing.assert_close(torch.tensor(graph_losses),
                               torch.tensor(eager_losses[2 + 2::3]), rtol=1e-6, atol=0)
    for a, b in zip(eager_module.parameters(), graph_module.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=0)


def test_multi_step_replay_raises_validation_errors(device):
    body, _, x = coin_setup(device)
    captured = StepGraph(body, warmup=2, repeat=2)
    captured()
    captured.check()
    x[3] = 2.0   # outside Bernoulli's support: found by a replay, raised by the next check
    captured()
    with pytest.raises(ValueError, match="is not in the support"):
        captured.check()


def test_graph_defers_validation_errors(device):
    body, _, x = coin_setup(device)
    captured = StepGraph(body, warmup=2)
    captured()
    captured.check()
    x[3] = 2.0            # same storage, now outside the Bernoulli support
    captured()
    with pytest.raises(ValueError, match="is not in the support"):
        captured.check()


def test_graph_regression_minibatch_window(device):
    """
    A captured step that gathers a new device-resident minibatch on every replay (C4 shape).
    """
    n_total, B, p, K = 4096, 256, 8, 32
    gen = torch.Generator().manual_seed(1)
    X = torch.randn(n_total, p, generator=gen).to(device)
    y = (X @ torch.randn(p, generator=gen).to(device)) + 0.1
    counter = torch.zeros(1, dtype=torch.int64, device=device)
    offsets = torch.arange(B, device=device)

    def model():
        theta = mi.sample("theta", Normal(0, 1), sample_shape=p)
        with mi.batch(n_total):
            with mi.no_log_prob():
                Xb = mi.sample("X", Normal(0, 1), sample_shape=(n_total, p))
            mi.sample("y", Normal(Xb @ theta, 1))

    module = mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(p),
                                             scale=torch.ones(p)).to(device)
    optimizer = torch.optim.Adam(module.parameters(), lr=0.05, capturable=True)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=3)

    def step():
        optimizer.zero_grad(set_to_none=True)
        rows = (counter % (n_total // B)) * B + offsets
        counter.add_(1)
        loss = loss_fn(mi.condition(model, X=X.index_select(0, rows), y=y.index_select(0, rows)),
                       {"theta": module()})
        loss.backward()
        optimizer.step()
        return loss

    captured = StepGraph(step, warmup=2)
    first = float(captured())
    for _ in range(200):
        captured()
    captured.check()
    assert float(captured()) < first      # it learns across replays
    assert int(counter) == 2 + 202         # warm-up steps and replays advanced the window (capture
    #                                        records the increment without executing it)


def test_graph_replays_fused_guide_draws(device):
    """
    A hierarchical model whose latent vector is drawn inside the site kernel (mi_draw, the step
    read from the device counter): graph replays must reproduce eager steps.
    """
    n, K = 4096, 16

    def setup():
        gen = torch.Generator().manual_seed(2)
        y = torch.randn(n, generator=gen).to(device)

        def model():
            mu = mi.sample("mu", Normal(0.0, 1.0))
            z = mi.sample("z", Normal(mu, 1.0), sample_shape=[n])
            mi.sample("y", Normal(z, 0.5))

        approx = mi.nn.ParameterizedFactorizedDistribution(
            mu=mi.nn.ParameterizedDistribution(Normal, loc=0.0, scale=1.0),
            z=mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(n), scale=torch.ones(n)),
        ).to(device)
        optimizer = torch.optim.Adam(approx.parameters(), lr=0.01, capturable=True)
        loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=9)
        cond = mi.condition(model, y=y)

        def step():
            optimizer.zero_grad(set_to_none=True)
            loss = loss_fn(cond, approx())
            loss.backward()
            optimizer.step()
            return loss.detach()
        return step, approx

    eager_step, eager_approx = setup()
    graph_body, graph_approx = setup()
    eager = [float(eager_step()) for _ in range(6)]
    captured = StepGraph(graph_body, warmup=2)
    replays = [float(captured()) for _ in range(4)]
    captured.check()
    torch.testing.assert_close(torch.tensor(replays), torch.tensor(eager[2:]), rtol=1e-6, atol=0)
    for a, b in zip(eager_approx.parameters(), graph_approx.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=0)


@pytest.mark.parametrize("family", ["bernoulli_linear", "bernoulli_group"])
@pytest.mark.parametrize("host_looks", [True, False], ids=["polling", "unpolled"])
def test_graph_never_loses_a_transient_violation(device, family, host_looks):
    """
    A rotating device-resident minibatch (C4 shape) where exactly one window holds a value outside
    the Bernoulli support (2.0), replayed without ever blocking: the violation of that one replay
    must still be raised, with the reference's message (core.py:186-188), even though later
    replays evaluate valid windows (sticky validation words).
    """
    n_total, B, p, K = 4096, 256, 8, 32
    windows = n_total // B
    gen = torch.Generator().manual_seed(1)
    X = torch.randn(n_total, p, generator=gen).to(device)
    y = (torch.rand(n_total, generator=gen) < 0.5).float().to(device)
    y[5 * B + 17] = 2.0               # window 5 only
    counter = torch.zeros(1, dtype=torch.int64, device=device)
    offsets = torch.arange(B, device=device)

    def model():
        theta = mi.sample("theta", Normal(0, 1), sample_shape=p)
        if family == "bernoulli_linear":
            Xb = mi.sample("X", Normal(0, 1), sample_shape=(B, p))
            mi.sample("y", Bernoulli(logits=Xb @ theta))
        else:
            mi.sample("y", Bernoulli(logits=theta.sum()), sample_shape=[B])

    module = mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(p),
                                             scale=torch.ones(p)).to(device)
    optimizer = torch.optim.Adam(module.parameters(), lr=0.01, capturable=True)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=3)

    def step():
        optimizer.zero_grad(set_to_none=True)
        rows = (counter % windows) * B + offsets
        counter.add_(1)
        data = dict(y=y.index_select(0, rows))
        if family == "bernoulli_linear":
            data["X"] = X.index_select(0, rows)
        loss = loss_fn(mi.condition(model, **data), {"theta": module()})
        loss.backward()
        optimizer.step()
        return loss

    captured = StepGraph(step, warmup=2)   # windows 0, 1 (eager); capture executes nothing
    poll = captured._check
    if not host_looks:   # the host never inspects a replay before the last one
        captured._check = lambda block: None
    with pytest.raises(ValueError, match="is not in the support"):
        for _ in range(windows - 3):       # replays see windows 2 .. 14: window 5 once
            captured()
        captured._check = poll
        captured.check()
    captured()                             # cleared after raising: valid windows pass again
    captured.check()


def test_captured_step_keeps_its_host_constant_copies(device):
    """
    A torch-evaluated site with host constants (StudentT(3., 0., 1.)) reads cached device copies
    of them (particles.device_copy). StepGraph pins the copies its capture read, so evicting them
    from the cache (more than 64 other copies) and reusing the freed memory leaves the replays
    unchanged (a replay could read memory the caching allocator had handed out again).
    """
    from torch.distributions import StudentT
    from mininf_amd import particles
    x = torch.linspace(-2, 2, 100, device=device)

    def model():
        theta = mi.sample("theta", StudentT(3.0, 0.0, 1.0))
        mi.sample("x", Normal(theta, 1.0), sample_shape=[100])

    module = mi.nn.ParameterizedDistribution(Normal, loc=0.1, scale=0.8).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=64, seed=3)
    cond = mi.condition(model, x=x)

    def step():
        for p in module.parameters():
            p.grad = None
        loss = loss_fn(cond, {"theta": module()})
        loss.backward()
        return loss

    captured = StepGraph(step, warmup=2)
    assert captured._pinned, "the capture should have read device copies of the constants"
    loss_fn._counter.zero_()
    before = float(captured())
    for i in range(200):   # evict every cached copy, then reuse the freed blocks
        particles.device_copy(torch.full((5,), float(i) + 0.5), device)
    particles._HOST_COPIES.clear()
    import gc
    gc.collect()
    junk = [torch.full((64,), 1e30, device=device) for _ in range(256)]
    loss_fn._counter.zero_()
    after = float(captured())
    captured.check()
    del junk
    assert after == before


def test_capture_survives_garbage_with_device_finalizers(device):
    """
    Garbage whose finalizers touch the device -- an earlier StepGraph (its hipGraph executable and
    memory pool), a pinned host buffer written by a non-blocking copy, HIP events -- left in
    reference cycles right before a StepGraph is built, with the collector set to run at every
    allocation (commit 1bb8d71: a collection inside a capture ran such finalizers on the capturing
    stream and aborted a bench run; StepGraph now collects before the capture and keeps the
    collector off during it). Capture and replays succeed and match eager steps, and the
    collector's state is restored afterwards.
    """
    import gc

    class Cycle:
        def __init__(self, payload):
            self.payload = payload
            self.me = self

    eager_step, _, _ = coin_setup(device, n=2000, K=64)
    eager = [float(eager_step()) for _ in range(5)]

    body, _, _ = coin_setup(device, n=2000, K=64)
    old_body, _, _ = coin_setup(device, n=2000, K=64)
    old = StepGraph(old_body, warmup=1)
    old()
    old.check()
    thresholds = gc.get_threshold()
    gc.disable()   # the garbage survives until the StepGraph is built
    try:
        pinned = torch.empty(1024, pin_memory=True)
        pinned.copy_(torch.ones(1024, device=device), non_blocking=True)
        events = [torch.cuda.Event(enable_timing=True) for _ in range(8)]
        for e in events:
            e.record()
        torch.cuda.synchronize()
        Cycle(old)
        Cycle(pinned)
        Cycle(events)
        del old, pinned, events
        gc.set_threshold(1, 1, 1)
        gc.enable()
        captured = StepGraph(body, warmup=3)
        assert gc.isenabled()
    finally:
        gc.set_threshold(*thresholds)
        gc.enable()
    losses = [float(captured()) for _ in range(2)]
    captured.check()
    torch.testing.assert_close(torch.tensor(losses), torch.tensor(eager[3:5]), rtol=1e-6, atol=0)
