"""
Which part of the GP example's step (examples/missing-observations.md:28-45) goes wrong under
StepGraph replay: forward only, forward + backward, then the full step, each replay compared with
the same computation run eagerly. Prints one line per stage.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import mininf_amd as mi  # noqa: E402
from mininf_amd.graph import StepGraph  # noqa: E402
from torch.distributions import Gamma, Normal  # noqa: E402
from tests import example_models as ex  # noqa: E402

device = torch.device("cuda", 0)


def setup():
    n = ex.MISSING_N
    q = mi.nn.ParameterizedFactorizedDistribution(
        z=mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(n), scale=torch.ones(n)),
        sigma=mi.nn.ParameterizedDistribution(Gamma, concentration=2, rate=2),
        length_scale=mi.nn.ParameterizedDistribution(Gamma, concentration=2, rate=2),
    ).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=16, seed=5)
    y = torch.linspace(-1, 1, n, device=device)
    cond = mi.condition(ex.missing_model, {"kappa": torch.tensor(0.1, device=device)}, y=y)
    return q, loss_fn, cond


def stage(name, make_body, read):
    q, loss_fn, cond = setup()
    eager_body = make_body(q, loss_fn, cond)
    eager = [read(eager_body(), q) for _ in range(WARMUP + 2)]
    q2, loss_fn2, cond2 = setup()
    body = make_body(q2, loss_fn2, cond2)
    g = StepGraph(body, warmup=WARMUP)
    got = []
    for _ in range(2):
        out = g()
        torch.cuda.synchronize()
        got.append(read(out, q2))
    print(name, os.environ.get("GP_DEBUG_TAG", ""), "eager", eager[WARMUP:], "graph", got,
          flush=True)


def fwd(q, loss_fn, cond):
    return lambda: loss_fn(cond, q()).detach()


def fwd_bwd(q, loss_fn, cond):
    def body():
        for p in q.parameters():
            p.grad = None
        loss = loss_fn(cond, q())
        loss.backward()
        return torch.cat([p.grad.reshape(-1)[:3] for p in q.parameters()])
    return body


WARMUP = int(os.environ.get("GP_DEBUG_WARMUP", "2"))
stage("forward", fwd, lambda out, q: float(out))
if os.environ.get("GP_DEBUG_BWD", "1") == "1":
    stage("forward+backward", fwd_bwd, lambda out, q: out.cpu().tolist())
