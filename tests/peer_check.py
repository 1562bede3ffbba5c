"""
Child of tests/test_gpu_peer.py, one process per rank under torch.distributed.run (two or three
ranks on the one GPU). Prints one JSON line on rank 0.

    peer_check.py sum       mininf_amd.peer's all-reduce against gloo's, eager and from a captured
                            graph (world > 2 runs the kernel's multi-peer write and wait loops)
    peer_check.py missing   the last rank never calls: every other rank's call must time out
                            bounded, poison its bucket with NaN, and raise PeerTimeout at the next
                            host read (eager calls and StepGraph replays), without advancing its
                            call counter
"""
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mininf_amd.graph import StepGraph  # noqa: E402
from mininf_amd.peer import PeerCommunicator, PeerTimeout  # noqa: E402


def capture(fn):
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        graph.capture_begin()
        fn()
        graph.capture_end()
    torch.cuda.current_stream().wait_stream(stream)
    return graph


def check_sum(comm, rank, device):
    gen = torch.Generator().manual_seed(100 + rank)
    eager_equal = True
    for n in (1, 65, 300):
        for _ in range(3):
            x = torch.randn(n, generator=gen)
            want = x.clone()
            dist.all_reduce(want)
            got = x.to(device)
            comm.all_reduce(got)
            torch.cuda.synchronize()
            eager_equal &= bool(torch.allclose(got.cpu(), want, rtol=0, atol=1e-6))
            if dist.get_world_size() == 2:   # one addition: the same rounding as any SUM
                eager_equal &= bool(torch.equal(got.cpu(), want))
    # captured: the kernel is one graph node; each replay reduces the buffer's current contents
    buf = torch.zeros(65, device=device)
    graph = capture(lambda: comm.all_reduce(buf))
    graph_equal = True
    for _ in range(4):
        x = torch.randn(65, generator=gen)
        want = x.clone()
        dist.all_reduce(want)
        buf.copy_(x.to(device))
        dist.barrier()
        graph.replay()
        torch.cuda.synchronize()
        graph_equal &= bool(torch.allclose(buf.cpu(), want, rtol=0, atol=1e-6))
    comm.check()
    return {"eager_equal": eager_equal, "graph_equal": graph_equal,
            "error_word": int(comm.error[0])}


def check_missing(comm, rank, world, device):
    if rank == world - 1:   # the rank that never calls
        return {}
    out = {}
    # a StepGraph replay of the all-reduce: the kernel times out, the bucket is NaN, the graph
    # raises at its check
    buf = torch.ones(33, device=device)
    step_graph = StepGraph(lambda: comm.all_reduce(buf) or buf, warmup=0)
    t0 = time.perf_counter()
    step_graph()
    torch.cuda.synchronize()
    out["wait_s"] = time.perf_counter() - t0
    out["graph_nan"] = bool(torch.isnan(buf).all())
    try:
        step_graph.check()
        out["graph_raised"] = False
    except PeerTimeout:
        out["graph_raised"] = True
    # eager: the next call raises before enqueuing anything
    x = torch.ones(8, device=device)
    try:
        comm.all_reduce(x)
        out["eager_raised"] = False
    except PeerTimeout:
        out["eager_raised"] = True
    torch.cuda.synchronize()
    out["eager_untouched"] = bool((x == 1).all())
    # the sticky word also poisons a launch that bypasses the host check (a graph captured before
    # the failure), and the kernel did not advance the call counter
    counter_before = comm.call_counter()
    step_graph.graph.replay()
    torch.cuda.synchronize()
    out["sticky_nan"] = bool(torch.isnan(buf).all())
    out["counter"] = [counter_before, comm.call_counter()]
    out["error_word"] = int(comm.error[0])
    return out


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "sum"
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    comm = PeerCommunicator(device=device, max_floats=300)
    if mode == "sum":
        result = check_sum(comm, rank, device)
    else:
        result = check_missing(comm, rank, world, device)
    results = [None] * world
    dist.all_gather_object(results, result)
    comm.close()
    if rank == 0:
        print(json.dumps({"mode": mode, "world": world, "ranks": results},
                         default=lambda v: None if isinstance(v, float) and math.isnan(v) else v),
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
