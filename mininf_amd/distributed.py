"""
Particle sharding across GPUs (one process per GPU, ``torch.distributed`` over RCCL/xGMI).

Monte-Carlo particles are independent, so the only exchange the ELBO step has is ONE all-reduce of
the guide gradients (plus the loss value) per step. ``EvidenceLowerBoundLoss(
num_particles=K, process_group=g)`` gives rank r the global particles [r K/W, (r+1) K/W) -- the
Philox counter uses the global particle index, so the union of draws does not depend on W -- and
returns the rank's share of the loss (its particles' sum / K plus entropy / W). Summing the shares'
gradients over ranks gives the full-K gradient, which every rank then applies with an identical
optimizer step, so the guide parameters stay in sync without a broadcast.
"""
from __future__ import annotations

import dataclasses
from typing import Iterable, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import engine


@dataclasses.dataclass(frozen=True)
class DataShard:
    """
    Data sharding of one ELBO over the ranks of a process group (the C5 row):
    instead of splitting the particles, rank r owns the elements ``[start, stop)`` of the data
    axis -- its slice of the observations and of every guide factor over them -- for ALL
    particles. The rank's model and guide are written for its slice (``stop - start`` elements);
    the factors and sites named in ``shared`` (global latents such as the hierarchical mean) are
    replicated: every rank draws them identically and counts their log density and entropy with
    weight 1/W, so the ranks' losses sum to the full ELBO. Only the shared parameters' gradients
    (and the loss) need the all-reduce; each rank's optimizer updates its own slice.

    The guide generator keys a sharded factor's draws by the GLOBAL element index
    (``mi_draw.element_offset``), so the union of the slices draws exactly what one process drawing
    every element would: ``start`` is a multiple of 4 (one Philox block per element quad).
    """
    start: int
    stop: int
    shared: Tuple[str, ...] = ()
    world: Optional[int] = None   # ranks sharing the data axis (default: the group's size)

    def __post_init__(self) -> None:
        if self.start < 0 or self.stop < self.start or (self.start % 4 and self.stop > self.start):
            raise ValueError(f"invalid data shard [{self.start}, {self.stop}): start must be a "
                             "non-negative multiple of 4 and stop >= start")
        object.__setattr__(self, "shared", tuple(self.shared))

    @property
    def size(self) -> int:
        return self.stop - self.start

    @property
    def slice(self) -> slice:
        return slice(self.start, self.stop)


def element_shard(n: int, group=None, shared: Sequence[str] = (), *, world: Optional[int] = None,
                  rank: Optional[int] = None) -> DataShard:
    """
    This rank's :class:`DataShard` of ``n`` elements: contiguous slices of ``ceil(n / W)``
    elements rounded up to a multiple of 4 (the last rank takes the remainder). ``world`` and
    ``rank`` default to the group's.
    """
    if world is None:
        world = dist.get_world_size(group) if dist.is_initialized() else 1
    if rank is None:
        rank = dist.get_rank(group) if dist.is_initialized() else 0
    per = -(-n // world)
    per = -(-per // 4) * 4
    return DataShard(min(n, rank * per), min(n, (rank + 1) * per), tuple(shared), world)


def all_reduce_gradients(parameters: Iterable[torch.nn.Parameter], group=None,
                         loss: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """
    Sum the gradients (and optionally the loss share) of all ranks with one flat all-reduce.

    Args:
        parameters: Parameters whose ``.grad`` to reduce in place.
        group: Process group (default: the world).
        loss: This rank's loss share; if given, the global loss is returned.

    Returns:
        The summed loss if ``loss`` was given, else ``None``.
    """
    engine.flush_pending_step()   # (a held finishing launch writes the gradients)
    grads = [p.grad for p in parameters if p.grad is not None]
    parts = [g.reshape(-1) for g in grads]
    if loss is not None:
        parts.append(loss.detach().reshape(1).to(grads[0].dtype if grads else torch.float32))
    if not parts:
        return None
    bucket = torch.cat(parts)
    dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=group)
    offset = 0
    for g in grads:
        n = g.numel()
        g.copy_(bucket[offset:offset + n].view_as(g))
        offset += n
    return bucket[offset] if loss is not None else None


class GradientBucket:
    """
    The guide gradients of one rank as ONE flat fp32 buffer, for a step split around the
    all-reduce: ``pack()`` (one concatenation kernel, capturable) after the backward,
    ``all_reduce()`` (one RCCL call), then ``bind()`` points every ``param.grad`` at its slice of the
    reduced buffer -- no copy back -- so the optimizer step (also capturable) reads the sums.
    The result equals :func:`all_reduce_gradients` (the gloo tests check this). Clear the
    gradients with ``zero_grad(set_to_none=True)`` before each backward, so that the backward
    does not accumulate into the bound views.

    With ``with_loss`` the buffer carries one more element, the rank's loss share (``pack(loss)``),
    so the same single all-reduce also yields the global loss (:meth:`loss`).

    Args:
        parameters: The parameters whose gradients to reduce (all of them must receive one).
        group: Process group (default: the world).
        with_loss: Reserve the loss element.
        communicator: A :class:`mininf_amd.rccl.Communicator` to run the all-reduce on (RCCL
            called directly: capturable into a hipGraph); default: ``torch.distributed`` over
            ``group``.
    """
    def __init__(self, parameters: Iterable[torch.nn.Parameter], group=None,
                 with_loss: bool = False, communicator=None) -> None:
        self.params = [p for p in parameters if p.requires_grad]
        if not self.params:
            raise ValueError("no parameters to reduce")
        dtypes = {p.dtype for p in self.params}
        if len(dtypes) != 1:
            raise ValueError(f"parameters of one dtype expected, got {dtypes}")
        self.group = group
        self.with_loss = with_loss
        self.communicator = communicator
        self.flat = torch.zeros(sum(p.numel() for p in self.params) + int(with_loss),
                                dtype=dtypes.pop(), device=self.params[0].device)
        self.views = []
        offset = 0
        for p in self.params:
            self.views.append(self.flat[offset:offset + p.numel()].view_as(p))
            offset += p.numel()

    def pack(self, loss: Optional[torch.Tensor] = None) -> None:
        """Copy this rank's gradients (and loss share, with ``with_loss``) into the flat buffer."""
        engine.flush_pending_step()
        grads = []
        for p in self.params:
            if p.grad is None:
                raise RuntimeError("a parameter of the bucket has no gradient")
            grads.append(p.grad.reshape(-1))
        if self.with_loss:
            if loss is None:
                raise ValueError("this bucket carries the loss: pack(loss)")
            grads.append(loss.detach().reshape(1).to(self.flat.dtype))
        torch.cat(grads, out=self.flat)

    def loss(self) -> torch.Tensor:
        """The loss element (after :meth:`all_reduce`: the global loss)."""
        if not self.with_loss:
            raise ValueError("this bucket does not carry the loss")
        return self.flat[-1]

    def all_reduce(self) -> None:
        """Sum the flat buffer over the ranks (in place)."""
        if self.communicator is not None:
            self.communicator.all_reduce(self.flat)
        else:
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)

    def bind(self) -> None:
        """Make every ``param.grad`` the view of its slice of the flat buffer."""
        for p, v in zip(self.params, self.views):
            p.grad = v
