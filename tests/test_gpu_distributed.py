"""
Particle sharding on the device path: two ranks (gloo, both on cuda:0 -- the pool's boxes have
one GPU; the driver's 8-GPU runs use RCCL) each evaluate their half of the particles with the HIP
kernels; the all-reduced loss and gradients must equal a single process evaluating all particles,
because the guide generator is keyed by the global particle index.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch.distributions import Bernoulli, Beta, Normal

pytestmark = pytest.mark.gpu

K_TOTAL = 64


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def setup(device):
    import mininf_amd as mi
    n = 3000
    gen = torch.Generator().manual_seed(0)
    x = (torch.rand(n, generator=gen) < 0.3).float().to(device)
    y = torch.randn(n, generator=gen).to(device)

    def model():
        theta = mi.sample("theta", Beta(2.0, 2.0))
        mu = mi.sample("mu", Normal(0.0, 1.0))
        mi.sample("x", Bernoulli(theta), sample_shape=[n])
        mi.sample("y", Normal(mu, 1.0), sample_shape=[n])

    torch.manual_seed(0)
    guide = mi.nn.ParameterizedFactorizedDistribution(
        theta=mi.nn.ParameterizedDistribution(Beta, concentration1=1.5, concentration0=2.5),
        mu=mi.nn.ParameterizedDistribution(Normal, loc=0.3, scale=0.8),
    ).to(device)
    return mi.condition(model, x=x, y=y), guide


def run(process_group):
    import mininf_amd as mi
    from mininf_amd.distributed import all_reduce_gradients
    device = torch.device("cuda", 0)
    cond, guide = setup(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K_TOTAL, seed=11,
                                           process_group=process_group)
    loss = loss_fn(cond, guide())
    loss.backward()
    params = list(guide.parameters())
    if process_group is not None:
        total = all_reduce_gradients(params, process_group, loss=loss)
    else:
        total = loss.detach()
    return float(total), [p.grad.detach().cpu().reshape(-1).tolist() for p in params]


def worker(rank, world, port, queue):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        queue.put((rank,) + run(dist.group.WORLD))
    finally:
        dist.destroy_process_group()


def test_two_ranks_match_one_process():
    world = 2
    ctx = mp.get_context("spawn")
    queue = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, queue)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(queue.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single_total, single_grads = run(None)
    for _, total, grads in results:
        assert total == pytest.approx(single_total, rel=1e-5)
        for got, want in zip(grads, single_grads):
            assert got == pytest.approx(want, rel=1e-5, abs=1e-6)


# ------------------------------------------------------------------------------------------------
# Data sharding: ranks own element slices of the hierarchical model
# (examples/missing-observations.md:33-45 restated as C5), all particles on every rank.
# ------------------------------------------------------------------------------------------------
N_DATA, K_DATA = 4096, 64


def hierarchical(device, shard=None):
    import mininf_amd as mi
    gen = torch.Generator().manual_seed(4)
    mu_true = torch.randn((), generator=gen)
    z_true = mu_true + torch.randn(N_DATA, generator=gen)
    y = z_true + 0.5 * torch.randn(N_DATA, generator=gen)
    b = (torch.rand(N_DATA, generator=gen) < torch.sigmoid(z_true)).float()
    mask = torch.rand(N_DATA, generator=gen) > 0.2
    loc0 = 0.1 * torch.randn(N_DATA, generator=gen)
    sl = slice(None) if shard is None else shard.slice
    n = N_DATA if shard is None else shard.size
    ym = torch.masked.as_masked_tensor(y[sl].to(device), mask[sl].to(device))
    bm = torch.masked.as_masked_tensor(b[sl].to(device), mask[sl].to(device))

    def model():
        mu = mi.sample("mu", Normal(0, 1))
        z = mi.sample("z", Normal(mu, 1), sample_shape=[n])
        mi.sample("y", Normal(z, 0.5))
        mi.sample("b", Bernoulli(logits=z))

    guide = mi.nn.ParameterizedFactorizedDistribution(
        mu=mi.nn.ParameterizedDistribution(Normal, loc=0.2, scale=0.9),
        z=mi.nn.ParameterizedDistribution(Normal, loc=loc0[sl], scale=torch.full((n,), 0.8)),
    ).to(device)
    return mi.condition(model, y=ym, b=bm), guide


def run_data(process_group, rank=0, world=1):
    import mininf_amd as mi
    from mininf_amd.distributed import GradientBucket, element_shard
    device = torch.device("cuda", 0)
    shard = None if process_group is None else element_shard(N_DATA, process_group,
                                                              shared=("mu",))
    cond, guide = hierarchical(device, shard)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K_DATA, seed=3,
                                           process_group=process_group, data_shard=shard)
    loss = loss_fn(cond, guide())
    loss.backward()
    if process_group is not None:
        bucket = GradientBucket(guide["mu"].parameters(), process_group, with_loss=True)
        bucket.pack(loss)
        bucket.all_reduce()
        bucket.bind()
        total = bucket.loss()
    else:
        total = loss.detach()
    grads = {name: p.grad.detach().cpu().reshape(-1) for name, p in guide.named_parameters()}
    return float(total), grads, (0, N_DATA) if shard is None else (shard.start, shard.stop)


def data_worker(rank, world, port, queue):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        total, grads, span = run_data(dist.group.WORLD, rank, world)
        queue.put((rank, total, {k: v.tolist() for k, v in grads.items()}, span))
    finally:
        dist.destroy_process_group()


def test_data_sharded_ranks_match_one_process():
    """Two ranks, each with half of the elements and all 64 particles: the all-reduced loss and
    the shared (mu) gradients equal one process's; each rank's z gradients equal the single
    process's on its slice (the z draws are keyed by the global element index)."""
    world = 2
    ctx = mp.get_context("spawn")
    queue = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=data_worker, args=(r, world, port, queue)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(queue.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single_total, single_grads, _ = run_data(None)
    for _, total, grads, (start, stop) in results:
        assert total == pytest.approx(single_total, rel=1e-5)
        for name, got in grads.items():
            want = single_grads[name]
            if name.startswith("z."):
                want = want[start:stop]
            got = torch.tensor(got)
            assert got.shape == want.shape, name
            torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6, msg=name)
