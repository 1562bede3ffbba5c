"""
RCCL called directly (``ncclCommInitRank`` / ``ncclAllReduce`` over xGMI), for the ONE all-reduce
of the sharded ELBO step inside a captured hipGraph.

``torch.distributed``'s RCCL process group tracks every collective with events that its watchdog
thread polls; an all-reduce captured into a graph leaves such events on a capturing stream, which
the watchdog then queries (``hipErrorCapturedEvent`` aborts the process). A communicator of our
own has no watchdog: ``ncclAllReduce`` is enqueued on the caller's stream like any kernel, so a
capture records it as a graph node and every replay runs it. The process group is still used to
bootstrap the communicator (rank 0's unique id is broadcast over it) and for host barriers.

The library is the ``librccl.so`` torch itself loaded (the same copy, so one RCCL per process).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch
import torch.distributed as dist

from . import _native as native

NCCL_UNIQUE_ID_BYTES = 128
NCCL_SUM = 0                                      # ncclRedOp_t (rccl.h)
_DTYPES = {torch.float32: 7, torch.float64: 8}    # ncclFloat32, ncclFloat64


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_ubyte * NCCL_UNIQUE_ID_BYTES)]


_LIB: Optional[ctypes.CDLL] = None


def library() -> ctypes.CDLL:
    """librccl.so: torch's own copy (already mapped), else ROCm's."""
    global _LIB
    if _LIB is None:
        candidates = [os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"),
                      "/opt/rocm/lib/librccl.so"]
        path = next((p for p in candidates if os.path.exists(p)), None)
        if path is None:
            raise RuntimeError("librccl.so not found (torch/lib or /opt/rocm/lib)")
        lib = ctypes.CDLL(path)
        vp = ctypes.c_void_p
        lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        lib.ncclCommInitRank.argtypes = [ctypes.POINTER(vp), ctypes.c_int, _UniqueId, ctypes.c_int]
        lib.ncclAllReduce.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, vp, vp]
        lib.ncclCommDestroy.argtypes = [vp]
        lib.ncclGetErrorString.argtypes = [ctypes.c_int]
        lib.ncclGetErrorString.restype = ctypes.c_char_p
        for name in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclCommDestroy"):
            getattr(lib, name).restype = ctypes.c_int
        _LIB = lib
    return _LIB


def _check(code: int, what: str) -> None:
    if code != 0:
        message = library().ncclGetErrorString(code)
        raise RuntimeError(f"{what} failed: {message.decode() if message else code}")


class Communicator:
    """
    An RCCL communicator over the ranks of ``group`` (one rank per GPU, the current device), built
    once; :meth:`all_reduce` sums a device buffer in place on the current stream (capturable).
    """
    def __init__(self, group=None, device: Optional[torch.device] = None) -> None:
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        lib = library()
        uid = _UniqueId()
        if self.rank == 0:
            _check(lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        # the 128 opaque bytes (NULs included) from rank 0 to every rank
        box = [ctypes.string_at(ctypes.addressof(uid), NCCL_UNIQUE_ID_BYTES)
               if self.rank == 0 else None]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group or dist.group.WORLD, 0),
                                   group=group)
        uid = _UniqueId()
        ctypes.memmove(ctypes.addressof(uid), box[0], NCCL_UNIQUE_ID_BYTES)
        self.comm = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _check(lib.ncclCommInitRank(ctypes.byref(self.comm), self.world, uid, self.rank),
                   "ncclCommInitRank")

    def all_reduce(self, tensor: torch.Tensor) -> None:
        """In-place SUM of a contiguous float32/float64 device tensor over the ranks."""
        if not tensor.is_contiguous() or tensor.device != self.device or \
                tensor.dtype not in _DTYPES:
            raise ValueError("all_reduce takes a contiguous float32/float64 tensor on the "
                             f"communicator's device {self.device}")
        # through the launch hook: a held step-finishing launch (engine._PendingStep) that writes
        # `tensor` -- a guide gradient passed here directly -- is enqueued before the collective
        stream = native.stream_handle(self.device)
        _check(library().ncclAllReduce(tensor.data_ptr(), tensor.data_ptr(), tensor.numel(),
                                       _DTYPES[tensor.dtype], NCCL_SUM, self.comm, stream),
               "ncclAllReduce")

    def close(self) -> None:
        if self.comm:
            library().ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()
