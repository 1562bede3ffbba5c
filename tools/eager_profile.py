"""
cProfile of the README training loop run eagerly (bench workload, HIP Adam): the host functions
behind each step's ~1 ms, by own time and by cumulative time.

    python tools/eager_profile.py [c2|c3|c4|c5] [steps] > out.txt
"""
import cProfile
import io
import os
import pstats
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import mininf_amd  # noqa: E402
import mininf_amd.optim  # noqa: E402


def main():
    config = sys.argv[1] if len(sys.argv) > 1 else "c2"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    device = torch.device("cuda", 0)
    w = bench.workload(config, device, 1, 0)
    optimizer = mininf_amd.optim.Adam(w["module"].parameters(), lr=w["lr"])
    loss_fn = mininf_amd.nn.EvidenceLowerBoundLoss(num_particles=w["k_local"], seed=1)

    def step():
        optimizer.zero_grad(set_to_none=True)
        loss = loss_fn(w["conditioned"](), w["guide"]())
        loss.backward()
        optimizer.step()

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    prof = cProfile.Profile()
    prof.enable()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    prof.disable()
    for key in ("tottime", "cumtime"):
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats(key).print_stats(70)
        print(buf.getvalue(), flush=True)
    for pattern in filter(None, os.environ.get("CALLEES", "").split(",")):
        buf = io.StringIO()   # what the named functions spend their time in
        pstats.Stats(prof, stream=buf).sort_stats("cumtime").print_callees(pattern)
        print(buf.getvalue(), flush=True)


if __name__ == "__main__":
    main()
