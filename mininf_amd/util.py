"""
Small helpers shared by the tracing layer and the ELBO engine.

Host-side mirror of ``mininf/util.py`` (reference). Names, signatures and error behaviour follow
the reference so that models and tests written against it keep working:

* ``IN_CI``                        -- reference ``mininf/util.py:8``
* ``_normalize_shape``             -- reference ``mininf/util.py:15-25``
* ``_format_dict_compact``         -- reference ``mininf/util.py:28-40``
* ``check_constraint``             -- reference ``mininf/util.py:43-66``
* ``get_masked_data_with_dense_grad`` -- reference ``mininf/util.py:69-92``
* ``maybe_as_tensor``              -- reference ``mininf/util.py:95-107``
"""
from __future__ import annotations

import numbers
import os
from typing import Any, Dict, TypeVar

import torch
from torch.distributions.constraints import Constraint


IN_CI = "CI" in os.environ

OptionalSize = torch.Size | torch.Tensor | int | None
TensorDict = Dict[str, torch.Tensor]
T = TypeVar("T", bound=torch.Tensor)


def _normalize_shape(shape: OptionalSize) -> torch.Size:
    """
    Turn ``None``, an int, a 0-d tensor, a sequence or a 1-d tensor into a :class:`torch.Size`.
    """
    if shape is None:
        return torch.Size()
    if isinstance(shape, torch.Size):
        return shape
    scalar_tensor = torch.is_tensor(shape) and shape.ndim == 0
    if isinstance(shape, int) or scalar_tensor:
        return torch.Size([int(shape)])
    return torch.Size([int(size) for size in shape])


def _describe(element: Any) -> str:
    if isinstance(element, torch.Tensor):
        return f"{element.__class__.__name__}(shape={tuple(element.shape)})"
    return str(type(element))


def _format_dict_compact(value: Dict[str, Any], id_: int | None = None,
                         name: str | None = None) -> str:
    """
    Compact ``repr`` of a mapping that shows tensor shapes (or types) instead of values, e.g.
    ``<State at 0x... comprising {'x': Tensor(shape=(3,))}>``.
    """
    body = ", ".join(f"'{key}': {_describe(element)}" for key, element in value.items())
    return f"<{name or value.__class__.__name__} at {hex(id_ or id(value))} comprising {{{body}}}>"


def check_constraint(constraint: Constraint, value: T) -> T:
    """
    Evaluate ``constraint.check`` and respect masks of :class:`torch.masked.MaskedTensor` values.

    For a masked value the check runs on the underlying data and the result is masked with the
    value's mask reduced (``all``) over the constraint's event dimensions.

    Args:
        constraint: Constraint to check.
        value: Plain or masked tensor.

    Returns:
        Elementwise indicator (aggregated over event dimensions) whether the constraint holds.
    """
    if not isinstance(value, torch.masked.MaskedTensor):
        if isinstance(constraint, _PositiveDefinite):
            return _positive_definite(value)
        return constraint.check(value)

    mask = value.get_mask()
    for _ in range(constraint.event_dim):
        mask = mask.all(-1)
    with torch.no_grad():
        checked = constraint.check(value.get_data())
    return torch.masked.as_masked_tensor(checked, mask)


class _DenseGradData(torch.autograd.Function):
    """
    Expose the data of a masked tensor while routing dense gradients back to it. Masked-out
    elements receive a zero gradient (reference ``mininf/util.py:78-90``).
    """
    @staticmethod
    def forward(ctx, value):  # type: ignore[override]
        ctx.mask = value._masked_mask
        return value._masked_data

    @staticmethod
    def backward(ctx, grad):  # type: ignore[override]
        if torch.masked.is_masked_tensor(grad):
            grad = grad._masked_data
        return torch.where(ctx.mask, grad, 0)


def get_masked_data_with_dense_grad(value: torch.masked.MaskedTensor) -> torch.Tensor:
    """
    Return the data of a masked tensor such that gradients flowing back to it are dense tensors
    (zero where masked) instead of sparse or masked tensors.

    Args:
        value: Masked tensor.

    Returns:
        Underlying data with a dense gradient path.
    """
    return _DenseGradData.apply(value)


def maybe_as_tensor(value: Any) -> torch.Tensor | None:
    """
    Convert plain Python numbers to tensors and pass everything else through unchanged.
    """
    if value is not None and isinstance(value, numbers.Number):
        return torch.as_tensor(value)
    return value


from torch.distributions.constraints import _PositiveDefinite  # noqa: E402


def _positive_definite(value: torch.Tensor) -> torch.Tensor:
    """
    ``constraints.positive_definite.check`` (torch constraints.py) without its host branch
    (``if not sym_check.all()``), so that it also runs per particle under ``vmap``: symmetric
    within torch's tolerance AND a successful Cholesky factorisation -- the same result.
    """
    from . import mvn
    # torch.isclose(value, value.mT, atol=1e-6) spelled out (isclose has no vmap batching rule:
    # its fallback launches per particle)
    other = value.mT
    close = (value == other) | ((value - other).abs() <= 1e-6 + 1e-5 * other.abs())
    symmetric = close.all(-2).all(-1)
    if mvn.cholesky_supported(value):   # mi_cholesky: no host sync, capturable
        return symmetric & mvn.cholesky_ex(value.detach())[1].eq(0)
    return symmetric & torch.linalg.cholesky_ex(value).info.eq(0)
