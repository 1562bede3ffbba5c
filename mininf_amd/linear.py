"""
Deferred linear predictors: ``X @ theta`` inside a traced model without the [N, K] product.

The reference's regression models compute ``Normal(X @ theta, sigma)`` (``tests/test_mininf.py:13-18``,
``examples/minibatch.md:24-33``). Traced over K particles that matmul is a [N, K] GEMM whose output is
only ever read by the site's log density. While :func:`mininf_amd.particles.trace_particles` runs the
model, :class:`DeferredMatmul` (a ``TorchFunctionMode``) intercepts ``matmul(X, theta)`` for an
observed 2-D ``X`` and a per-particle 1-D ``theta`` and returns a *placeholder*: a batched tensor of
the right shape backed by a zero-stride zero, costing no memory and no kernel. The particle tracer
turns a Normal / Bernoulli-logits site whose location / logits is such a placeholder into a fused
linear site (``mi_linear_forward``: the product is evaluated inside the site kernel).

Semantics are preserved for every other use: any torch operation that reads a placeholder's values
(anything but shape queries and broadcasting views) first *materialises* it -- the real
``torch.matmul(X, theta)`` is computed at that point, exactly as the model wrote it -- and the
operation runs on the real tensor. A placeholder therefore never leaks a wrong value into the model.
"""
from __future__ import annotations

import dataclasses
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch
from torch.overrides import TorchFunctionMode
from torch.utils._pytree import tree_map

from . import guide as _guide
from .guide import lazy_of

_functorch = torch._C._functorch

_MATMULS = {torch.matmul, torch.Tensor.matmul, torch.Tensor.__matmul__, torch.mv, torch.Tensor.mv}

# Operations that only read metadata (never values) pass a placeholder through unchanged.
_METADATA = {
    torch.Tensor.size, torch.Tensor.dim, torch.Tensor.ndimension, torch.Tensor.numel,
    torch.Tensor.__len__, torch.Tensor.is_floating_point, torch.Tensor.is_complex,
    torch.Tensor.stride, torch.Tensor.element_size,
    torch.Tensor.shape.__get__, torch.Tensor.dtype.__get__, torch.Tensor.device.__get__,
    torch.Tensor.ndim.__get__, torch.Tensor.requires_grad.__get__, torch.Tensor.is_cuda.__get__,
    torch.Tensor.layout.__get__, torch.Tensor.is_sparse.__get__, torch.Tensor.grad_fn.__get__,
    torch.Tensor.is_leaf.__get__, torch.Tensor.names.__get__,
}

# Broadcasting views of a placeholder are placeholders of the broadcast shape.
_BROADCASTS = {torch.broadcast_tensors, torch.Tensor.expand, torch.Tensor.expand_as,
               torch.Tensor.broadcast_to, torch.broadcast_to}


class NeedsDraws(Exception):
    """
    Raised while tracing when the model uses a lazy guide draw (:class:`mininf_amd.guide.LazyDraw`)
    in an operation other than a site parameter / value: the loss then re-traces with real draws.
    """



def _leaves(args, kwargs):
    """The tensors of a torch function call's arguments (lists, tuples and dicts walked; the
    pytree machinery costs tens of microseconds per call on this path)."""
    stack = [args, kwargs]
    while stack:
        x = stack.pop()
        if isinstance(x, torch.Tensor):
            yield x
        elif isinstance(x, (list, tuple)):
            stack.extend(x)
        elif isinstance(x, dict):
            stack.extend(x.values())

@dataclasses.dataclass
class Deferred:
    """
    ``root``: the deferred ``X @ theta`` (``X`` [N, P] observed, ``theta`` batched [P]); a derived
    placeholder is ``root`` broadcast to ``shape``.
    """
    X: torch.Tensor
    theta: torch.Tensor
    shape: torch.Size
    root: Optional["Deferred"] = None
    real: Optional[torch.Tensor] = None


class DeferredMatmul(TorchFunctionMode):
    """
    Active while a model is traced over particles (inside ``vmap``); see the module docstring.
    """
    require_device = True   # defer only device matmuls (the fused kernel's operands)

    def __init__(self, K: int, defer_matmul: bool = True) -> None:
        super().__init__()
        self.K = K
        self.defer_matmul = defer_matmul
        self.deferred: Dict[int, Deferred] = {}
        self._keep: List[torch.Tensor] = []   # placeholders stay alive: ids are never reused
        self._bypass = False

    # ---- helpers ---------------------------------------------------------------------------
    def lookup(self, tensor: Any) -> Optional[Deferred]:
        if isinstance(tensor, torch.Tensor):
            return self.deferred.get(id(tensor))
        return None

    def _eligible(self, args, kwargs) -> bool:
        if kwargs or len(args) != 2:
            return False
        X, theta = args
        if not (isinstance(X, torch.Tensor) and isinstance(theta, torch.Tensor)):
            return False
        if self.lookup(X) is not None or self.lookup(theta) is not None:
            return False
        if not self.defer_matmul or lazy_of(X) is not None or lazy_of(theta) is not None:
            return False
        return (not _functorch.is_batchedtensor(X) and X.dim() == 2 and
                (X.is_cuda or not self.require_device) and
                X.dtype == torch.float32 and not X.requires_grad and
                _functorch.is_batchedtensor(theta) and theta.dim() == 1 and
                theta.dtype == torch.float32 and theta.shape[0] == X.shape[1] and
                X.shape[1] <= 64 and X.shape[0] > 0)

    def _placeholder(self, like: torch.Tensor, shape: torch.Size, info: Deferred) -> torch.Tensor:
        level = _functorch.maybe_get_level(like)
        # never read (any value-reading use materialises the product): no initialising kernel
        base = torch.empty((), dtype=torch.float32, device=info.X.device)
        base = base.expand((self.K,) + tuple(shape))
        out = _functorch._add_batch_dim(base, 0, level)
        self.deferred[id(out)] = info
        self._keep.append(out)
        return out

    def materialize(self, tensor: torch.Tensor) -> torch.Tensor:
        """
        The real value of a placeholder (computed once), or ``tensor`` itself.
        """
        info = self.lookup(tensor)
        if info is None:
            return tensor
        root = info.root or info
        if root.real is None:
            _guide.flush_draws()   # theta may be a guide draw not launched yet
            self._bypass = True
            try:
                root.real = torch.matmul(root.X, root.theta)
            finally:
                self._bypass = False
        if info.root is None:
            return root.real
        if info.real is None:
            self._bypass = True
            try:
                info.real = root.real.expand(info.shape)
            finally:
                self._bypass = False
        return info.real

    # ---- the mode ----------------------------------------------------------------------------
    def __torch_function__(self, func: Callable, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if self._bypass:
            return func(*args, **kwargs)
        if func in _MATMULS and self._eligible(args, kwargs):
            X, theta = args
            info = Deferred(X=X, theta=theta, shape=torch.Size([X.shape[0]]))
            return self._placeholder(theta, info.shape, info)
        if not self.deferred and not _guide._LAZY and \
                (not _guide._PENDING_DRAWS or func in _METADATA or func in _BROADCASTS):
            # no placeholder exists, and no pending draw is read by this call: nothing to do
            return func(*args, **kwargs)
        touched = []
        lazy = []
        for x in _leaves(args, kwargs):
            info = self.lookup(x)
            if info is not None:
                touched.append(info)
            elif lazy_of(x) is not None:
                lazy.append(x)
            elif func not in _METADATA and func not in _BROADCASTS and \
                    _guide.pending_draw(x) is not None:
                # the model reads a guide draw whose launch was left to the loss's planning
                _guide.flush_draws()
        if not touched and not lazy:
            return func(*args, **kwargs)
        if func in _METADATA:
            return func(*args, **kwargs)
        if lazy and func not in _BROADCASTS:
            raise NeedsDraws(getattr(func, "__name__", str(func)))
        if not touched:
            return func(*args, **kwargs)
        if func in _BROADCASTS:
            out = func(*args, **kwargs)
            inputs = args[0] if func is torch.broadcast_tensors and len(args) == 1 and \
                isinstance(args[0], (list, tuple)) else args
            if func is torch.broadcast_tensors:
                outs = list(out)
                for src, dst in zip(inputs, outs):
                    self._derive(src, dst)
            else:
                self._derive(args[0], out)
            return out
        args, kwargs = tree_map(lambda x: self.materialize(x) if self.lookup(x) else x,
                                (args, kwargs))
        return func(*args, **kwargs)

    def _derive(self, src: Any, dst: torch.Tensor) -> None:
        info = self.lookup(src)
        if info is None or not isinstance(dst, torch.Tensor):
            return
        root = info.root or info
        self.deferred[id(dst)] = Deferred(X=root.X, theta=root.theta,
                                          shape=torch.Size(dst.shape), root=root)
        self._keep.append(dst)
