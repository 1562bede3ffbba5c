"""
List the aten ops and device kernels of one eager training step of a bench config, in order
(torch.profiler): where the small launches of a step come from.

Usage (GPU box): python tools/op_profile.py [c2|c3|c4|c5]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mininf_amd  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    w = bench.workload(cfg, device, 1, 0)
    module = w["module"]
    optimizer = torch.optim.Adam(module.parameters(), lr=w["lr"], capturable=True, fused=True)
    loss_fn = mininf_amd.nn.EvidenceLowerBoundLoss(num_particles=w["k_local"], seed=1)

    def step():
        optimizer.zero_grad(set_to_none=True)
        loss = loss_fn(w["conditioned"](), w["guide"]())
        loss.backward()
        optimizer.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        step()
        torch.cuda.synchronize()
    events = [e for e in prof.events() if e.device_type.name == "CUDA"]
    events.sort(key=lambda e: e.time_range.start)
    for e in events:
        parent = e.cpu_parent
        chain = []
        while parent is not None and len(chain) < 4:
            chain.append(parent.name)
            parent = parent.cpu_parent
        print(f"{e.name[:70]:70s} <- {' <- '.join(chain)}")
    print(len(events), "device kernels")


if __name__ == "__main__":
    main()
