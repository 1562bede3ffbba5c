"""Capture a C5-shaped step with the fused guide draw at a given particle count / size."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mininf_amd as mi  # noqa: E402
from mininf_amd.graph import StepGraph  # noqa: E402
from torch.distributions import Bernoulli, Normal  # noqa: E402

n, K, masked = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3] == "1"
dev = torch.device("cuda", 0)
gen = torch.Generator().manual_seed(0)
y = torch.randn(n, generator=gen).to(dev)
b = (torch.rand(n, generator=gen) < 0.5).float().to(dev)
mask = (torch.rand(n, generator=gen) > 0.2).to(dev)


def model():
    mu = mi.sample("mu", Normal(0, 1))
    z = mi.sample("z", Normal(mu, 1), sample_shape=[n])
    mi.sample("y", Normal(z, 0.5))
    mi.sample("b", Bernoulli(logits=z))


approx = mi.nn.ParameterizedFactorizedDistribution(
    mu=mi.nn.ParameterizedDistribution(Normal, loc=0.0, scale=1.0),
    z=mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(n), scale=torch.ones(n))).to(dev)
opt = torch.optim.Adam(approx.parameters(), lr=0.01, capturable=True)
loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=1)
data = dict(y=torch.masked.as_masked_tensor(y, mask), b=torch.masked.as_masked_tensor(b, mask)) \
    if masked else dict(y=y, b=b)
cond = mi.condition(model, **data)


def step():
    opt.zero_grad(set_to_none=True)
    loss = loss_fn(cond, approx())
    loss.backward()
    opt.step()
    return loss.detach()


for _ in range(2):
    step()
torch.cuda.synchronize()
print("eager ok", flush=True)
g = StepGraph(step, warmup=2)
print("captured", flush=True)
for _ in range(3):
    g()
g.check()
torch.cuda.synchronize()
print("replayed ok", flush=True)
