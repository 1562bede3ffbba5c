"""
Time mininf_amd.optim.Adam alone on C5's guide parameters (z loc and scale, 1e6 floats each):
HIP events around graph replays of 50 steps each (MININF_AMD_LIB selects a variant build):

    python tools/adam_probe.py [elements per tensor]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import mininf_amd as mi  # noqa: E402
import mininf_amd.optim  # noqa: E402,F401


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(n, device=dev, generator=gen)) for _ in range(2)]
    for p in params:
        p.grad = torch.randn(n, device=dev, generator=gen)
    opt = mi.optim.Adam(params, lr=1e-3)
    for _ in range(20):
        opt.step()
    torch.cuda.synchronize()
    # 50 steps per captured graph: the launches back to back, no host dispatch between them
    per = 50
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph):
            for _ in range(per):
                opt.step()
    torch.cuda.current_stream().wait_stream(side)
    graph.replay()
    torch.cuda.synchronize()
    replays = 8
    steps = per * replays
    start, stop = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record()
    for _ in range(replays):
        graph.replay()
    stop.record()
    torch.cuda.synchronize()
    us = start.elapsed_time(stop) * 1e3 / steps
    moved = 28.0 * 2 * n   # read param, grad, m, v; write param, m, v (fp32)
    print(json.dumps({"lib": os.environ.get("MININF_AMD_LIB", "default"), "n": n,
                      "us_per_step": round(us, 2), "TB_s": round(moved / us / 1e6, 3)}),
          flush=True)


if __name__ == "__main__":
    main()
