"""
Child of tests/test_gpu_peer.py, one process per rank under torch.distributed.run (two ranks on
the one GPU): mininf_amd.peer's all-reduce against gloo's, eager and from a captured graph.
Prints one JSON line on rank 0.
"""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mininf_amd.peer import PeerCommunicator  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    comm = PeerCommunicator(device=device, max_floats=300)
    gen = torch.Generator().manual_seed(100 + rank)
    eager_equal = True
    for n in (1, 65, 300):
        for _ in range(3):
            x = torch.randn(n, generator=gen)
            want = x.clone()
            dist.all_reduce(want)
            got = x.to(device)
            comm.all_reduce(got)
            eager_equal &= bool(torch.equal(got.cpu(), want))
    # captured: the kernel is one graph node; each replay reduces the buffer's current contents
    buf = torch.zeros(65, device=device)
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        graph.capture_begin()
        comm.all_reduce(buf)
        graph.capture_end()
    torch.cuda.current_stream().wait_stream(stream)
    graph_equal = True
    for _ in range(4):
        x = torch.randn(65, generator=gen)
        want = x.clone()
        dist.all_reduce(want)
        buf.copy_(x.to(device))
        dist.barrier()
        graph.replay()
        torch.cuda.synchronize()
        graph_equal &= bool(torch.equal(buf.cpu(), want))
    error = int(comm.error.item())
    dist.barrier()
    comm.close()
    flags = torch.tensor([int(eager_equal), int(graph_equal), -error])
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)   # (every rank equal; any rank's error word)
    if rank == 0:
        print(json.dumps({"eager_equal": bool(flags[0]), "graph_equal": bool(flags[1]),
                          "error_word": -int(flags[2]), "world": world}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
