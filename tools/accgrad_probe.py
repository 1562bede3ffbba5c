"""
Which objects keep an eager step's autograd graph alive after the step (the source of torch's
"AccumulateGrad node's stream does not match" warning when a later step runs on another stream):
runs a few eager bench steps, then lists live tensors that carry a grad_fn, with two levels of
referrers.

    python tools/accgrad_probe.py [c3|c4|c2|c5]
"""
import gc
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import mininf_amd  # noqa: E402
import mininf_amd.optim  # noqa: E402


def describe(obj):
    if isinstance(obj, torch.Tensor):
        return f"Tensor{tuple(obj.shape)} grad_fn={type(obj.grad_fn).__name__}"
    if isinstance(obj, dict):
        return "dict keys=" + ",".join(str(k)[:30] for k in list(obj)[:6])
    if isinstance(obj, (list, tuple)):
        return f"{type(obj).__name__}[{len(obj)}]"
    return type(obj).__module__ + "." + type(obj).__qualname__


def main():
    config = sys.argv[1] if len(sys.argv) > 1 else "c3"
    device = torch.device("cuda", 0)
    w = bench.workload(config, device, 1, 0)
    optimizer = mininf_amd.optim.Adam(w["module"].parameters(), lr=w["lr"])
    loss_fn = mininf_amd.nn.EvidenceLowerBoundLoss(num_particles=w["k_local"], seed=1)

    def step():
        optimizer.zero_grad(set_to_none=True)
        loss = loss_fn(w["conditioned"](), w["guide"]())
        loss.backward()
        optimizer.step()
        return loss.detach()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    gc.collect()
    nodes = [o for o in gc.get_objects() if isinstance(o, torch.autograd.function.BackwardCFunction)]
    print(f"{config}: {len(nodes)} live custom-Function nodes", flush=True)
    for n in nodes[:8]:
        print(" ", describe(n))
        for r in gc.get_referrers(n)[:4]:
            print("    <-", describe(r))
            for r2 in gc.get_referrers(r)[:3]:
                print("       <-", describe(r2))
    live = [o for o in gc.get_objects()
            if isinstance(o, torch.Tensor) and getattr(o, "grad_fn", None) is not None]
    print(f"{config}: {len(live)} live tensors with grad_fn", flush=True)
    for t in live[:12]:
        print(" ", describe(t))
        for r in gc.get_referrers(t)[:6]:
            if r is live:
                continue
            print("    <-", describe(r))
            for r2 in gc.get_referrers(r)[:4]:
                if r2 is live:
                    continue
                print("       <-", describe(r2))
    # the step's warm-up on a side stream (StepGraph), the warning raised where it happens
    import traceback
    import warnings
    from mininf_amd.graph import StepGraph
    warnings.filterwarnings("error", message=".*AccumulateGrad node's stream.*")
    real_begin = torch.cuda.CUDAGraph.capture_begin

    def begin(self, *args, **kwargs):   # what the warm-up left alive, just before the capture
        gc.collect()
        nodes = [o for o in gc.get_objects()
                 if isinstance(o, torch.autograd.function.BackwardCFunction)]
        tensors = [o for o in gc.get_objects()
                   if isinstance(o, torch.Tensor) and getattr(o, "grad_fn", None) is not None]
        print(f"before capture: {len(nodes)} custom-Function nodes, {len(tensors)} tensors with "
              "grad_fn", flush=True)
        for o in (nodes + tensors)[:10]:
            print(" ", describe(o))
            for r in gc.get_referrers(o)[:5]:
                print("    <-", describe(r))
                for r2 in gc.get_referrers(r)[:3]:
                    print("       <-", describe(r2))
        return real_begin(self, *args, **kwargs)
    torch.cuda.CUDAGraph.capture_begin = begin
    try:
        graph = StepGraph(step, warmup=2)
        graph()
        torch.cuda.synchronize()
        print("StepGraph: no warning", flush=True)
        graph2 = StepGraph(step, warmup=2)   # a second capture after the first (bench: C2 floor)
        graph2()
        torch.cuda.synchronize()
        print("second StepGraph: no warning", flush=True)
    except Exception:
        traceback.print_exc()


if __name__ == "__main__":
    main()
