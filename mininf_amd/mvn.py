"""
MultivariateNormal site densities on the HIP kernel ``mi_mvn_tril_forward`` (``csrc/mvn.hip``).

Replaces ``MultivariateNormal.log_prob`` (torch ``multivariate_normal.py:255-262``, with
``_batch_mahalanobis`` at ``:80-102``) for the reference's Gaussian-process sites
(``examples/missing-observations.md:42``): the covariance is factorised by torch (rocSOLVER,
float64 -- the example's GP covariance is too ill-conditioned for float32), the two triangular
solves, the Mahalanobis term and the log-determinant run in one wave per particle, and the
kernel's ``w = L^-1 r`` and ``u = L^-T w`` give the gradients without a second solve:
d/dvalue = -u, d/dloc = u, d/dL = tril(u w^T) - diag(1 / L_ii).

The density is an ``autograd.Function`` with a vmap rule: inside the particle trace
(``torch.func.vmap`` over particles) it launches once for all particles on the physical tensors.
"""
from __future__ import annotations

import math
import os
from typing import Tuple

import torch
from torch.distributions import MultivariateNormal

from . import _native as nat

MAX_N = 1024   # MI_MVN_MAX_N


def enabled(distribution: MultivariateNormal) -> bool:
    """Whether ``distribution``'s density runs on the kernel (float64 on the device, n <= MAX_N)."""
    L = distribution._unbroadcasted_scale_tril
    return os.environ.get("MININF_AMD_MVN_KERNEL", "1") != "0" and L.dtype == torch.float64 \
        and L.device.type == "cuda" and 1 <= L.shape[-1] <= MAX_N


def _launch(value: torch.Tensor, loc: torch.Tensor,
            scale_tril: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(log_prob [...], w [..., n], u [..., n]) over the broadcast batch of the three operands."""
    n = scale_tril.shape[-1]
    if value.shape[-1] != n or loc.shape[-1] != n or scale_tril.shape[-2] != n:
        raise ValueError(f"MultivariateNormal operands disagree on the event size {n}: value "
                         f"{tuple(value.shape)}, loc {tuple(loc.shape)}, scale_tril "
                         f"{tuple(scale_tril.shape)}")
    batch = torch.broadcast_shapes(value.shape[:-1], loc.shape[:-1], scale_tril.shape[:-2])
    B = math.prod(batch)
    device = scale_tril.device
    v = value.to(torch.float64).expand(*batch, n).reshape(B, n).contiguous()
    m = loc.to(torch.float64).expand(*batch, n).reshape(B, n).contiguous()
    L = scale_tril.to(torch.float64).expand(*batch, n, n).reshape(B, n, n).contiguous()
    lp = torch.empty(B, dtype=torch.float64, device=device)
    w = torch.empty((B, n), dtype=torch.float64, device=device)
    u = torch.empty((B, n), dtype=torch.float64, device=device)
    nat.check(nat.lib().mi_mvn_tril_forward(v.data_ptr(), m.data_ptr(), L.data_ptr(), B, n,
                                            lp.data_ptr(), w.data_ptr(), u.data_ptr(),
                                            nat.stream_handle(device)), "mi_mvn_tril_forward")
    return lp.reshape(batch), w.reshape(*batch, n), u.reshape(*batch, n)


class _MvnTrilLogProb(torch.autograd.Function):
    @staticmethod
    def forward(value, loc, scale_tril):  # type: ignore[override]
        return _launch(value, loc, scale_tril)

    @staticmethod
    def setup_context(ctx, inputs, output):  # type: ignore[override]
        value, loc, scale_tril = inputs
        _, w, u = output
        ctx.mark_non_differentiable(w, u)
        ctx.save_for_backward(scale_tril, w, u)
        ctx.shapes = (value.shape, loc.shape, scale_tril.shape)

    @staticmethod
    def backward(ctx, g, _gw, _gu):  # type: ignore[override]
        scale_tril, w, u = ctx.saved_tensors
        vshape, lshape, Lshape = ctx.shapes
        g = g.to(torch.float64)
        gu = g[..., None] * u
        dvalue = dloc = dL = None
        if ctx.needs_input_grad[0]:
            dvalue = (-gu).sum_to_size(vshape)
        if ctx.needs_input_grad[1]:
            dloc = gu.sum_to_size(lshape)
        if ctx.needs_input_grad[2]:
            diag = scale_tril.to(torch.float64).diagonal(dim1=-2, dim2=-1)
            dL = torch.tril(gu[..., :, None] * w[..., None, :]) - \
                torch.diag_embed(g[..., None] / diag)
            dL = dL.sum_to_size(Lshape)
        return dvalue, dloc, dL

    @staticmethod
    def vmap(info, in_dims, value, loc, scale_tril):  # type: ignore[override]
        # physical tensors with the particle axis first and the logical batch dimensions aligned
        # from the right (as the per-particle broadcast aligns them)
        events = (1, 1, 2)
        tensors = (value, loc, scale_tril)
        logical = [t.dim() - e - (d is not None) for t, d, e in zip(tensors, in_dims, events)]
        depth = max(logical)
        phys = []
        for t, d, e, lb in zip(tensors, in_dims, events, logical):
            t = t.movedim(d, 0) if d is not None else t.expand(info.batch_size, *t.shape)
            phys.append(t.reshape(t.shape[0], *([1] * (depth - lb)), *t.shape[1:]))
        return _MvnTrilLogProb.apply(*phys), (0, 0, 0)


def log_prob(distribution: MultivariateNormal, value: torch.Tensor) -> torch.Tensor:
    """``distribution.log_prob(value)`` on the kernel (float64; see :func:`enabled`)."""
    lp, _, _ = _MvnTrilLogProb.apply(value.to(torch.float64), distribution.loc,
                                     distribution._unbroadcasted_scale_tril)
    return lp
