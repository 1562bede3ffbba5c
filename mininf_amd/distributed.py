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

from typing import Iterable, Optional

import torch
import torch.distributed as dist


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
