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
