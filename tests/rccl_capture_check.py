"""
Run as a child process by tests/test_gpu_dist_graph.py: the sharded training step -- zero_grad,
ELBO forward and backward, packing the gradients and the loss share into the flat bucket, the
RCCL all-reduce, binding the reduced gradients and the HIP Adam -- captured as ONE hipGraph with
several steps per replay (bench.py's N > 1 path over RCCL), against the same steps run eagerly.

A one-rank ``nccl`` process group bootstraps a communicator of our own (mininf_amd.rccl: RCCL
called directly) on the box's single GPU: the collective is a real ncclAllReduce inside the
capture. The model is the reference's minibatch regression
(examples/minibatch.md:24-33) on a device-resident loader, so every replay draws a new batch and
new particles. Prints one JSON line.
"""
import json
import os
import socket
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import mininf_amd as mi  # noqa: E402
import mininf_amd.optim  # noqa: E402
from mininf_amd.distributed import GradientBucket  # noqa: E402
from mininf_amd.graph import StepGraph  # noqa: E402
from mininf_amd.rccl import Communicator  # noqa: E402
from torch.distributions import Normal  # noqa: E402

N_ROWS, P, BATCH, K = 16384, 8, 2048, 32
WARMUP, REPEAT = 2, 4


def setup(device, group, comm):
    gen = torch.Generator().manual_seed(0)
    X = torch.randn(N_ROWS, P, generator=gen)
    y = X @ torch.randn(P, generator=gen) + torch.randn(N_ROWS, generator=gen)
    loader = mi.DeviceDataLoader(X.to(device), y.to(device), batch_size=BATCH, shuffle=True,
                                 drop_last=True, seed=0)

    def model():
        theta = mi.sample("theta", Normal(0, 1), sample_shape=P)
        with mi.batch(N_ROWS):
            with mi.no_log_prob():
                Xs = mi.sample("X", Normal(0, 1), sample_shape=(N_ROWS, P))
            mi.sample("y", Normal(Xs @ theta, 1))

    guide = mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(P),
                                            scale=torch.ones(P)).to(device)
    optimizer = mininf_amd.optim.Adam(guide.parameters(), lr=0.01)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=1, process_group=group)
    bucket = GradientBucket(guide.parameters(), group, with_loss=True, communicator=comm)

    def step():
        optimizer.zero_grad(set_to_none=True)
        Xb, yb = loader.next()
        loss = loss_fn(mi.condition(model, X=Xb, y=yb), {"theta": guide()})
        loss.backward()
        bucket.pack(loss)
        bucket.all_reduce()
        bucket.bind()
        optimizer.step()
        return bucket.loss()
    return step, guide


def main():
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    with socket.socket() as sock:
        sock.bind(("127.0.0.1", 0))
        port = sock.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=device)
    group = dist.group.WORLD
    comm = Communicator(group, device)
    try:
        eager_step, eager_guide = setup(device, group, comm)
        eager = [float(eager_step()) for _ in range(WARMUP + 2 * REPEAT)]

        graph_body, graph_guide = setup(device, group, comm)
        captured = StepGraph(graph_body, warmup=WARMUP, repeat=REPEAT,
                             capture_error_mode="thread_local")
        losses = []
        for _ in range(2):
            out = captured()
            torch.cuda.synchronize()
            losses.append(float(out))
        captured.check()
        # replay r ends with step WARMUP + (r + 1) * REPEAT
        want = [eager[WARMUP + REPEAT - 1], eager[WARMUP + 2 * REPEAT - 1]]
        param_diff = max(float((a - b).abs().max()) for a, b in
                         zip(eager_guide.parameters(), graph_guide.parameters()))
        print(json.dumps({"graph_losses": losses, "eager_losses": want,
                          "param_max_abs_diff": param_diff, "eager_all": eager}), flush=True)
    finally:
        comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
