"""
Host cost of the primitives an eager step is made of (microseconds per call, GPU box): torch
allocations and small launches, ctypes launches, the Beta guide's construction pieces.

    python tools/host_micro.py
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import mininf_amd as mi  # noqa: E402
from mininf_amd import nn  # noqa: E402


def timed(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round(1e6 * (time.perf_counter() - t0) / n, 2)


def main():
    device = torch.device("cuda", 0)
    x = torch.ones(4096, device=device)
    module = nn.ParameterizedDistribution(torch.distributions.Beta, concentration1=2.0,
                                          concentration0=2.0).to(device)
    u1 = module.distribution_parameters["concentration1"]
    u0 = module.distribution_parameters["concentration0"]
    conc = torch.ones(2, device=device)
    out = {
        "torch.empty": timed(lambda: torch.empty(4096, device=device)),
        "x > 0": timed(lambda: x > 0),
        "(x > 0).all()": timed(lambda: (x > 0).all()),
        "bool(x.amin() > 0)": timed(lambda: bool(x.amin() > 0)),
        "torch._is_all_true((x>0).all())": timed(lambda: torch._is_all_true((x > 0).all())),
        "x2.tolist()": timed(lambda: conc.tolist()),
        "x2.cpu()": timed(lambda: conc.cpu()),
        "torch.zeros(8, int32)": timed(lambda: torch.zeros(8, dtype=torch.int32, device=device)),
        "current_stream": timed(lambda: torch.cuda.current_stream(device).cuda_stream),
        "raw stream": timed(lambda: torch._C._cuda_getCurrentRawStream(0)),
        "os.environ.get": timed(lambda: os.environ.get("MININF_AMD_X", "1")),
        "ExpStackFn.apply (no defer)": timed(lambda: nn._ExpStackFn.apply(u1, u0, False)),
        "ExpStackFn.apply (defer)": timed(lambda: nn._ExpStackFn.apply(u1, u0, True)),
        "Dirichlet(validate_args=False)": timed(
            lambda: torch.distributions.Dirichlet(conc, validate_args=False)),
        "module() (validated)": timed(lambda: module()),
    }
    torch.distributions.Distribution.set_default_validate_args(False)
    out["module() (unvalidated)"] = timed(lambda: module())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
