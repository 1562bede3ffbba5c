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

Opt-in (``bench.py --allreduce peer``); unmeasured on multi-GPU hardware: the tests run two and
three ranks sharing one GPU. A rank whose peer never arrives stops waiting after about a second,
writes NaN into the bucket instead of a sum of stale slots, and sets :attr:`PeerCommunicator.error`
(a word of pinned host memory, sticky: every later call of the kernel skips its peer writes and
poisons its bucket too). The host raises :class:`PeerTimeout` at its next read of the word:
:meth:`PeerCommunicator.all_reduce` reads it before enqueuing (no synchronisation), a
:class:`mininf_amd.graph.StepGraph` that captured the all-reduce reads it at each replay and
:meth:`~mininf_amd.graph.StepGraph.check`, and :meth:`PeerCommunicator.check` after a device wait.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import torch
import torch.distributed as dist

from . import _native as native
from . import graph


class PeerTimeout(RuntimeError):
    """A peer's flag did not arrive within the bounded wait: the communicator has failed."""


class PeerCommunicator:
    """
    The ranks of ``group`` (one process per rank; ranks may share a GPU), buckets of at most
    ``max_floats`` float32 values.
    """
    def __init__(self, group=None, device: Optional[torch.device] = None,
                 max_floats: int = 1024) -> None:
        self.group = group
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
        # the peers' slot offsets are computed from this rank's layout: every rank must agree on it
        layout = (self.world, self.max_floats, int(size.value))
        gathered: List[Optional[tuple]] = [None] * self.world
        dist.all_gather_object(gathered, (layout, bytes(handle)), group=group)
        mismatch = [q for q, (other, _) in enumerate(gathered) if tuple(other) != layout]
        if mismatch:
            with torch.cuda.device(self.device):
                lib.mi_peer_free(self.region)
            raise ValueError(f"peer all-reduce: ranks {mismatch} built their regions with another "
                             f"layout (world, max_floats, bytes) than rank {self.rank}'s {layout}: "
                             f"{[tuple(g[0]) for g in gathered]}")
        handles = [h for _, h in gathered]
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
        # the sticky error word, in pinned host memory: the kernel ORs into it, the host polls it
        self.error = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        # every rank's region is mapped before any rank's first write into it
        dist.barrier(group=group)

    def all_reduce(self, tensor: torch.Tensor) -> None:
        """In-place SUM of a contiguous float32 device tensor of at most ``max_floats`` values."""
        if not tensor.is_contiguous() or tensor.device != self.device or \
                tensor.dtype != torch.float32 or tensor.numel() > self.max_floats:
            raise ValueError(f"all_reduce takes a contiguous float32 tensor of at most "
                             f"{self.max_floats} values on {self.device}")
        self.raise_if_failed()
        # a StepGraph capturing this call reads the word after each replay
        graph.register_host_check(self.raise_if_failed)
        # (through the launch hook: a held step-finishing launch writing `tensor` runs first)
        stream = native.stream_handle(self.device)
        native.check(native.lib().mi_peer_allreduce(ctypes.byref(self.desc), tensor.data_ptr(),
                                                    tensor.data_ptr(), tensor.numel(),
                                                    self.error.data_ptr(), stream),
                     "mi_peer_allreduce")

    def call_counter(self) -> int:
        """Calls this rank has completed (diagnostics; synchronous)."""
        count = ctypes.c_uint64()
        with torch.cuda.device(self.device):
            native.check(native.lib().mi_peer_call_count(ctypes.byref(self.desc),
                                                         ctypes.byref(count)), "mi_peer_call_count")
        return int(count.value)

    def raise_if_failed(self) -> None:
        """Raise :class:`PeerTimeout` if a call that has completed timed out (no synchronisation:
        the word is pinned host memory the kernel writes)."""
        if int(self.error[0]) != 0:
            raise PeerTimeout(f"peer all-reduce (rank {self.rank} of {self.world}): a peer's flag "
                              "did not arrive within the bounded wait; the call's bucket was "
                              "filled with NaN and the communicator has failed")

    def check(self) -> None:
        """Wait for the device, then raise if any call's wait for a peer timed out."""
        torch.cuda.synchronize(self.device)
        self.raise_if_failed()

    def close(self) -> None:
        lib = native.lib()
        torch.cuda.synchronize(self.device)
        # no rank frees its region while a lagging peer's kernel may still write into it
        dist.barrier(group=self.group)
        for mapped in self.peers:
            lib.mi_peer_close(mapped)
        self.peers = []
        if self.region:
            lib.mi_peer_free(self.region)
            self.region = ctypes.c_void_p()
