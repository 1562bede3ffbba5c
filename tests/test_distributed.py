"""
Particle sharding across ranks exercised with the gloo backend on the CPU
(world size 2): rank particle ranges, the single flat all-reduce of gradients + loss, and the
identity "sum of rank shares == single-process value" for the ELBO's linear structure.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mininf_amd.distributed import GradientBucket, all_reduce_gradients
from mininf_amd.nn import EvidenceLowerBoundLoss


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, queue):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        loss = EvidenceLowerBoundLoss(num_particles=8 * world, process_group=dist.group.WORLD)
        shard = loss._shard()
        # A linear "loss share" per rank, as the ELBO produces: sum over the rank's particles / K.
        K = loss.num_particles
        w = torch.nn.Parameter(torch.tensor([1.0, -2.0]))
        offset, local = shard[3], shard[2]
        particles = torch.arange(offset, offset + local, dtype=torch.float32)
        share = (w[0] * particles.sum() + w[1] * particles.square().sum()) / K
        share.backward()
        total = all_reduce_gradients([w], dist.group.WORLD, loss=share)
        queue.put((rank, shard, w.grad.tolist(), float(total)))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_and_all_reduce():
    world = 2
    ctx = mp.get_context("spawn")
    queue = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, queue)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(queue.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    K = 16
    k = torch.arange(K, dtype=torch.float32)
    want_grad = [float(k.sum() / K), float(k.square().sum() / K)]
    want_total = float((k.sum() - 2 * k.square().sum()) / K)
    for rank, shard, grad, total in results:
        assert shard == (world, rank, K // world, rank * (K // world))
        assert grad == pytest.approx(want_grad)
        assert total == pytest.approx(want_total)


def test_indivisible_particles_rejected():
    class Group:
        pass

    loss = EvidenceLowerBoundLoss(num_particles=5)
    loss.process_group = Group()
    import unittest.mock as um
    with um.patch.object(dist, "get_world_size", return_value=2), \
            um.patch.object(dist, "get_rank", return_value=0):
        with pytest.raises(ValueError, match="not divisible"):
            loss._shard()


def bucket_worker(rank, world, port, queue):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        a = torch.nn.Parameter(torch.randn(3, 2))
        b = torch.nn.Parameter(torch.randn(()))
        bucket = GradientBucket([a, b], dist.group.WORLD)
        out = []
        for step in range(2):   # twice: the second backward runs with grads bound to the bucket
            for p in (a, b):
                p.grad = None
            ((rank + 1) * (a.square().sum() + step * b * a.sum())).backward()
            bucket.pack()
            bucket.all_reduce()
            bucket.bind()
            got = [a.grad.clone(), b.grad.clone()]
            for p in (a, b):
                p.grad = None
            ((rank + 1) * (a.square().sum() + step * b * a.sum())).backward()
            all_reduce_gradients([a, b], dist.group.WORLD)
            out.append([torch.equal(x, y) for x, y in zip(got, [a.grad, b.grad])])
        # the loss share rides in the same flat buffer: one all-reduce gives the global loss
        lossy = GradientBucket([a, b], dist.group.WORLD, with_loss=True)
        for p in (a, b):
            p.grad = None
        share = (rank + 1) * (a.square().sum() + b)
        share.backward()
        lossy.pack(share)
        lossy.all_reduce()
        lossy.bind()
        want = 3 * (a.detach().square().sum() + b.detach())   # ranks 0 and 1: (1 + 2) * ...
        out.append([torch.allclose(lossy.loss(), want), torch.equal(a.grad, 6 * a.detach())])
        queue.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_gradient_bucket_matches_all_reduce_gradients():
    """
    The split step bench.py captures for N > 1 (pack in the backward graph, one all-reduce,
    gradients bound to the reduced buffer) gives the same sums as all_reduce_gradients.
    """
    world = 2
    ctx = mp.get_context("spawn")
    queue = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=bucket_worker, args=(r, world, port, queue)) for r in range(world)]
    for p in procs:
        p.start()
    results = [queue.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out in results:
        assert all(all(step) for step in out), (rank, out)


# ------------------------------------------------------------------------------------------------
# Data sharding (DataShard): the element slices and the loss's replicated-site bookkeeping
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n", [9, 10, 4097, 1_000_000])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_element_shards_tile_the_data_axis(n, world):
    from mininf_amd.distributed import element_shard
    shards = [element_shard(n, world=world, rank=r, shared=("mu",)) for r in range(world)]
    assert shards[0].start == 0 and shards[-1].stop == n
    for a, b in zip(shards, shards[1:]):
        assert a.stop == b.start
    for s in shards:
        assert s.size == 0 or s.start % 4 == 0   # one Philox block per element quad
        assert s.shared == ("mu",) and s.world == world


def test_data_shard_validation():
    from mininf_amd.distributed import DataShard
    with pytest.raises(ValueError, match="multiple of 4"):
        DataShard(6, 10)
    with pytest.raises(ValueError, match="stop >= start"):
        DataShard(8, 4)
    shard = DataShard(8, 20, ["mu"], world=4)
    assert shard.shared == ("mu",) and shard.slice == slice(8, 20) and shard.size == 12
    with pytest.raises(ValueError, match="process_group"):
        EvidenceLowerBoundLoss(num_particles=4, data_shard=DataShard(0, 8))
    loss = EvidenceLowerBoundLoss(num_particles=16, data_shard=DataShard(0, 8, ("mu",), world=4))
    # every rank evaluates every particle; the loss knows the world from the shard
    assert loss._shard() == (4, 0, 16, 0)
    assert loss._element_offsets({"mu": None, "z": None}) == {"z": 0}


@pytest.mark.parametrize("offset", [0, 500])
def test_sharded_non_normal_factor_is_rejected_on_every_rank(offset):
    """A data-sharded Beta factor is rejected by the rank whose slice starts at element 0 as well
    (rank 0 accepted it and went on to the collective while the others raised)."""
    from torch.distributions import Beta
    from mininf_amd import _native as nat, guide
    factor = Beta(torch.full((1000,), 2.0), torch.full((1000,), 3.0))
    with pytest.raises(nat.NativeError, match="must be a Normal"):
        guide.draw_all({"p": factor}, 4, 0, 0, 0, element_offsets={"p": offset})
