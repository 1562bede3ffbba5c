"""
One-shot peer-write all-reduce for the sharded step's small gradient bucket (C2's and
C4's buckets are a few hundred bytes; a ring collective pays a latency per hop for them).

Each rank allocates one receive region of fine-grained device memory (``mi_peer_alloc``), the
ranks exchange its IPC handle over the process group once, and every rank maps its peers' regions
(``mi_peer_open``; over xGMI between GPUs, or the same card for ranks sharing one). Then
:meth:`PeerCommunicator.all_reduce` is ONE kernel on the current stream (``mi_peer_allreduce``):
the bucket is written into every peer's region, a flag with the call number follows, and each rank
sums the slots in rank order once its peers' flags arrived -- capturable into the step's hipGraph,
like :class:`mininf_amd.rccl.Communicator`, whose interface it shares (``all_reduce``, ``close``).

Opt-in (``bench.py --allreduce peer``); unmeasured on multi-GPU hardware: the tests run two ranks
sharing one GPU. A rank whose peer never arrives stops waiting after about a second and records it
in :attr:`PeerCommunicator.error` (device word; :meth:`check` reads it).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import torch
import torch.distributed as dist

from . import _native as native


class PeerCommunicator:
    """
    The ranks of ``group`` (one process per rank; ranks may share a GPU), buckets of at most
    ``max_floats`` float32 values.
    """
    def __init__(self, group=None, device: Optional[torch.device] = None,
                 max_floats: int = 1024) -> None:
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > native.PEER_MAX_RANKS:
            raise ValueError(f"at most {native.PEER_MAX_RANKS} ranks")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.max_floats = int(max_floats)
        lib = native.lib()
        size = ctypes.c_size_t()
        native.check(lib.mi_peer_region_bytes(self.max_floats, ctypes.byref(size)),
                     "mi_peer_region_bytes")
        self.region = ctypes.c_void_p()
        handle = (ctypes.c_ubyte * native.PEER_HANDLE_BYTES)()
        with torch.cuda.device(self.device):
            native.check(lib.mi_peer_alloc(size, ctypes.byref(self.region), handle),
                         "mi_peer_alloc")
        handles: List[Optional[bytes]] = [None] * self.world
        dist.all_gather_object(handles, bytes(handle), group=group)
        self.peers: List[ctypes.c_void_p] = []
        self.desc = native.Peer()
        self.desc.rank, self.desc.world, self.desc.max_floats = self.rank, self.world, self.max_floats
        with torch.cuda.device(self.device):
            for q, h in enumerate(handles):
                if q == self.rank:
                    self.desc.regions[q] = self.region.value
                    continue
                buf = (ctypes.c_ubyte * native.PEER_HANDLE_BYTES).from_buffer_copy(h)
                mapped = ctypes.c_void_p()
                native.check(lib.mi_peer_open(buf, ctypes.byref(mapped)), "mi_peer_open")
                self.peers.append(mapped)
                self.desc.regions[q] = mapped.value
        self.error = torch.zeros(1, dtype=torch.int32, device=self.device)
        # every rank's region is mapped before any rank's first write into it
        dist.barrier(group=group)

    def all_reduce(self, tensor: torch.Tensor) -> None:
        """In-place SUM of a contiguous float32 device tensor of at most ``max_floats`` values."""
        if not tensor.is_contiguous() or tensor.device != self.device or \
                tensor.dtype != torch.float32 or tensor.numel() > self.max_floats:
            raise ValueError(f"all_reduce takes a contiguous float32 tensor of at most "
                             f"{self.max_floats} values on {self.device}")
        # (through the launch hook: a held step-finishing launch writing `tensor` runs first)
        stream = native.stream_handle(self.device)
        native.check(native.lib().mi_peer_allreduce(ctypes.byref(self.desc), tensor.data_ptr(),
                                                    tensor.data_ptr(), tensor.numel(),
                                                    self.error.data_ptr(), stream),
                     "mi_peer_allreduce")

    def check(self) -> None:
        """Raise if a call's wait for a peer timed out (a host synchronisation)."""
        if int(self.error.item()) != 0:
            raise RuntimeError("peer all-reduce: a peer's flag did not arrive (timed out)")

    def close(self) -> None:
        lib = native.lib()
        torch.cuda.synchronize(self.device)
        for mapped in self.peers:
            lib.mi_peer_close(mapped)
        self.peers = []
        if self.region:
            lib.mi_peer_free(self.region)
            self.region = ctypes.c_void_p()
