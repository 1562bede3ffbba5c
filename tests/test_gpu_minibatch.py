"""
Device-resident minibatches (mininf_amd.data.DeviceDataLoader, csrc/minibatch.hip) on the GPU:

* the rows kernel against its restatement (oracle/minibatch.py), bit for bit, across epochs,
  sequential and shuffled, with a ragged last batch;
* gathered values against torch indexing of the dataset;
* the reference's minibatch regression (examples/minibatch.md:24-33) through the fused linear
  site reading X and y through the row index, against the same model conditioned on plain copies
  of the same rows (identical kernels on identical values: equal losses and gradients);
* a captured training loop drawing a new batch per replay against the eager loop;
* validation: an invalid value is reported with the reference's message.
"""
import pytest
import torch
from torch.distributions import Normal

import mininf_amd as mi
from mininf_amd.data import DeviceDataLoader, Minibatch
from mininf_amd.graph import StepGraph
from oracle import minibatch as oracle

pytestmark = pytest.mark.gpu


def test_rows_match_oracle(device):
    n, batch = 1003, 100
    X = torch.arange(n, dtype=torch.float32, device=device)
    for shuffle in (False, True):
        loader = DeviceDataLoader(X, batch_size=batch, shuffle=shuffle, seed=5)
        batches = len(loader)
        assert batches == 11
        for epoch in range(2):
            seen = []
            for b, (xb,) in enumerate(loader):
                count = min(batch, n - b * batch)
                want = oracle.batch_rows(epoch * batches + b, n, batch, batches, shuffle, 5, count)
                got = xb._mininf_batch.rows.cpu().tolist()
                assert got == want
                # a value-reading op gathers the rows
                assert isinstance(xb, Minibatch)
                assert torch.equal(xb.clone().as_subclass(torch.Tensor).cpu(),
                                   torch.tensor(want, dtype=torch.float32))
                seen += got
            assert sorted(seen) == list(range(n))


def test_next_crosses_epochs_with_drop_last(device):
    n, batch = 1000, 128
    loader = DeviceDataLoader(torch.zeros(n, 4, device=device), batch_size=batch, shuffle=True,
                              drop_last=True, seed=3)
    assert len(loader) == 7
    for c in range(16):
        (xb,) = loader.next()
        want = oracle.batch_rows(c, n, batch, 7, True, 3, batch)
        assert xb._mininf_batch.rows.cpu().tolist() == want
    with pytest.raises(ValueError, match="drop_last"):
        DeviceDataLoader(torch.zeros(n, device=device), batch_size=batch).next()


def regression(device, n=4096, p=8, seed=0):
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


def guide_module(device, p=8):
    gen = torch.Generator().manual_seed(9)
    return mi.nn.ParameterizedDistribution(Normal, loc=1e-3 * torch.randn(p, generator=gen),
                                           scale=torch.ones(p)).to(device)


def test_indexed_linear_site_matches_plain_rows(device):
    model, X, y = regression(device)
    loader = DeviceDataLoader(X, y, batch_size=512, shuffle=True, seed=1)
    Xb, yb = next(iter(loader))
    rows = Xb._mininf_batch.rows.long()
    results = []
    for values in ((Xb, yb), (X[rows].clone(), y[rows].clone())):
        module = guide_module(device)
        loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=64, seed=2)
        loss = loss_fn(mi.condition(model, X=values[0], y=values[1]), {"theta": module()})
        loss.backward()
        results.append((float(loss), [q.grad.clone() for q in module.parameters()]))
    (l0, g0), (l1, g1) = results
    assert l0 == l1
    for a, b in zip(g0, g1):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    # the indexed run never gathered X or y
    assert Xb._mininf_batch.filled == [False, False]


def test_captured_loop_draws_a_batch_per_replay(device):
    model, X, y = regression(device, n=8192)

    def setup():
        loader = DeviceDataLoader(X, y, batch_size=1024, shuffle=True, drop_last=True, seed=4)
        module = guide_module(device)
        optimizer = torch.optim.Adam(module.parameters(), lr=0.01, capturable=True)
        loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=32, seed=6)

        def step():
            optimizer.zero_grad(set_to_none=True)
            Xb, yb = loader.next()
            loss = loss_fn(mi.condition(model, X=Xb, y=yb), {"theta": module()})
            loss.backward()
            optimizer.step()
            return loss.detach()
        return step, module

    eager, eager_module = setup()
    eager_losses = [float(eager()) for _ in range(8)]
    body, graph_module = setup()
    captured = StepGraph(body, warmup=3)
    graph_losses = [float(captured()) for _ in range(4)]
    captured.check()
    torch.testing.assert_close(torch.tensor(graph_losses), torch.tensor(eager_losses[3:7]),
                               rtol=1e-6, atol=0)
    assert len(set(eager_losses)) == len(eager_losses)   # a new batch (and draw) every step


def test_multi_step_replay_with_minibatches_and_hip_adam(device):
    """StepGraph(repeat=4) over the minibatch loop with mininf_amd.optim.Adam: four batches,
    draws and Adam steps per replay, the same losses and parameters as eager steps."""
    model, X, y = regression(device, n=8192)

    def setup():
        loader = DeviceDataLoader(X, y, batch_size=1024, shuffle=True, drop_last=True, seed=4)
        module = guide_module(device)
        optimizer = mi.optim.Adam(module.parameters(), lr=0.01)
        loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=32, seed=6)

        def step():
            optimizer.zero_grad(set_to_none=True)
            Xb, yb = loader.next()
            loss = loss_fn(mi.condition(model, X=Xb, y=yb), {"theta": module()})
            loss.backward()
            optimizer.step()
            return loss.detach()
        return step, module

    eager, eager_module = setup()
    eager_losses = [float(eager()) for _ in range(2 + 4 * 3)]
    body, graph_module = setup()
    captured = StepGraph(body, warmup=2, repeat=4)
    graph_losses = [float(captured()) for _ in range(3)]
    captured.check()
    torch.testing.assert_close(torch.tensor(graph_losses),
                               torch.tensor(eager_losses[2 + 3::4]), rtol=1e-6, atol=0)
    for a, b in zip(eager_module.parameters(), graph_module.parameters()):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-6, atol=0)


def test_invalid_values_raise_reference_message(device):
    model, X, y = regression(device)
    y = y.clone()
    y[17] = float("nan")
    loader = DeviceDataLoader(X, y, batch_size=4096, seed=1)
    Xb, yb = next(iter(loader))
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=8)
    with pytest.raises(ValueError, match="is not in the support"):
        loss_fn(mi.condition(model, X=Xb, y=yb), {"theta": guide_module(device)()})
    X = X.clone()
    X[5, 1] = float("nan")
    loader = DeviceDataLoader(X, y, batch_size=64, seed=1)
    Xb, yb = next(iter(loader))
    with pytest.raises(ValueError, match="is not in the support"):
        loss_fn(mi.condition(model, X=Xb, y=yb), {"theta": guide_module(device)()})


def test_view_outlives_the_yielded_tensor(device):
    """A view of a minibatch keeps its batch alive on its own: reading it after the yielded tensor
    is gone still gathers the batch's rows."""
    import gc
    n, batch = 1000, 64
    X = torch.arange(n * 2, dtype=torch.float32, device=device).reshape(n, 2)
    loader = DeviceDataLoader(X, batch_size=batch, shuffle=True, drop_last=True, seed=9)
    (xb,) = loader.next()
    rows = xb._mininf_batch.rows.cpu()
    view = xb.reshape(-1, 1)
    assert isinstance(view, Minibatch)
    del xb
    gc.collect()
    got = view.clone().as_subclass(torch.Tensor).reshape(batch, 2).cpu()
    assert torch.equal(got, X.cpu()[rows.long()])


def test_linear_kernel_draws_the_batch_rows(device, monkeypatch):
    """The linear site kernel draws the rows of the batch it reads (mi_linear.rows: no
    mi_minibatch_rows launch): the rows it writes are the oracle's order, and the losses and
    gradients of several eager steps equal those with the rows kernel (MININF_AMD_FUSE_ROWS=0)."""
    model, X, y = regression(device, n=8192)
    n, batch = 8192, 1024

    def run():
        loader = DeviceDataLoader(X, y, batch_size=batch, shuffle=True, drop_last=True, seed=4)
        module = guide_module(device)
        loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=32, seed=6)
        out = []
        for step in range(10):   # crosses an epoch (8 batches per epoch)
            Xb, yb = loader.next()
            b = Xb._mininf_batch
            loss = loss_fn(mi.condition(model, X=Xb, y=yb), {"theta": module()})
            loss.backward()
            taken_by_kernel = not b.pending
            rows = b.rows.cpu().tolist()
            assert rows == oracle.batch_rows(step, n, batch, 8, True, 4, batch)
            out.append((float(loss), [q.grad.clone() for q in module.parameters()],
                        taken_by_kernel))
            for q in module.parameters():
                q.grad = None
        return out, int(loader.counter[0])

    fused, c0 = run()
    monkeypatch.setenv("MININF_AMD_FUSE_ROWS", "0")
    plain, c1 = run()
    assert c0 == c1 == 10
    for (l0, g0, _), (l1, g1, _) in zip(fused, plain):
        assert l0 == l1
        for a, b in zip(g0, g1):
            torch.testing.assert_close(a, b, rtol=0, atol=0)


def test_unsupported_linear_draw_takes_the_batch_rows_once(device, monkeypatch):
    """
    The linear launch cannot draw theta for P = 64 features and K = 128 particles (its staging
    buffer is too small for four particle tiles of two feature tiles) but can draw the batch's
    rows: the draw falls back to the guide's own launch, and the rows are still drawn exactly once
    per step -- the loader counter advances by one and every batch is the oracle's (ADVICE r03,
    high: the fallback drew them twice, skipping every other batch).
    """
    from mininf_amd import guide as guide_mod
    n, p, batch, K = 8192, 64, 1024, 128
    X, y = regression(device, n=n, p=p)[1:]
    launches = []
    real = guide_mod.PendingDraw.launch

    def spy(self):
        if not self.done:
            launches.append(tuple(self.z.shape))
        return real(self)
    monkeypatch.setattr(guide_mod.PendingDraw, "launch", spy)

    def model():
        theta = mi.sample("theta", Normal(0, 1), sample_shape=p)
        with mi.batch(n):
            with mi.no_log_prob():
                Xs = mi.sample("X", Normal(0, 1), sample_shape=(n, p))
            mi.sample("y", Normal(Xs @ theta, 1))

    loader = DeviceDataLoader(X, y, batch_size=batch, shuffle=True, drop_last=True, seed=9)
    module = mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(p),
                                             scale=torch.ones(p)).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=2)
    for step in range(3):
        Xb, yb = loader.next()
        b = Xb._mininf_batch
        loss = loss_fn(mi.condition(model, X=Xb, y=yb), {"theta": module()})
        loss.backward()
        assert int(loader.counter[0]) == step + 1
        assert b.rows.cpu().tolist() == oracle.batch_rows(step, n, batch, n // batch, True, 9,
                                                          batch)
        for q in module.parameters():
            q.grad = None
    assert launches == [(K, p)] * 3, launches   # the guide's own draw, once per step
