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


def _cholesky_launch(A: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(L, info) of mi_cholesky over the leading batch dimensions of A [..., n, n]."""
    n = A.shape[-1]
    if A.shape[-2] != n or A.dtype not in (torch.float32, torch.float64):
        raise ValueError(f"cholesky of a float32/float64 [..., n, n] tensor, got "
                         f"{tuple(A.shape)} {A.dtype}")
    batch = A.shape[:-2]
    B = math.prod(batch)
    a = A.reshape(B, n, n).contiguous()
    wide = n > 80 and A.dtype == torch.float32   # larger factors are formed in float64
    L = torch.empty((B, n, n), dtype=torch.float64 if wide else A.dtype, device=A.device)
    info = torch.empty(B, dtype=torch.int32, device=A.device)
    nat.check(nat.lib().mi_cholesky(a.data_ptr(), a.element_size(), B, n, L.data_ptr(),
                                    L.element_size(), info.data_ptr(),
                                    nat.stream_handle(A.device)), "mi_cholesky")
    if wide:
        L = L.to(A.dtype)
    return L.reshape(A.shape), info.reshape(batch)


class _CholeskyFn(torch.autograd.Function):
    """``torch.linalg.cholesky_ex(A)`` on mi_cholesky, with torch's backward
    (FunctionsManual linalg_cholesky_backward restated: gA = sym(L^-T phi(L^T gL) L^-1), phi the
    lower triangle with the diagonal halved) and a vmap rule for the particle trace."""
    @staticmethod
    def forward(A):  # type: ignore[override]
        return _cholesky_launch(A)

    @staticmethod
    def setup_context(ctx, inputs, output):  # type: ignore[override]
        L, info = output
        ctx.mark_non_differentiable(info)
        ctx.save_for_backward(L)

    @staticmethod
    def backward(ctx, gL, _ginfo):  # type: ignore[override]
        (L,) = ctx.saved_tensors
        if gL is None:
            return None
        P = (L.mT @ gL.tril()).tril()
        P = P - 0.5 * torch.diag_embed(P.diagonal(dim1=-2, dim2=-1))
        X = torch.linalg.solve_triangular(L.mT, P, upper=True, left=True)     # L^-T phi
        gA = torch.linalg.solve_triangular(L, X, upper=False, left=False)     # ... L^-1
        return 0.5 * (gA + gA.mT)

    @staticmethod
    def vmap(info, in_dims, A):  # type: ignore[override]
        (d,) = in_dims
        A = A.movedim(d, 0) if d is not None else A.expand(info.batch_size, *A.shape)
        return _CholeskyFn.apply(A), (0, 0)


def cholesky_ex(A: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """``torch.linalg.cholesky_ex(A)`` (lower) on the HIP kernel: (L, info), no host sync."""
    return _CholeskyFn.apply(A)


def cholesky_supported(A: torch.Tensor) -> bool:
    return os.environ.get("MININF_AMD_CHOLESKY_KERNEL", "1") != "0" and A.is_cuda and \
        A.dtype in (torch.float32, torch.float64) and A.dim() >= 2 and \
        A.shape[-1] == A.shape[-2] and 1 <= A.shape[-1] <= MAX_N


def log_prob(distribution: MultivariateNormal, value: torch.Tensor) -> torch.Tensor:
    """``distribution.log_prob(value)`` on the kernel (float64; see :func:`enabled`)."""
    lp, _, _ = _MvnTrilLogProb.apply(value.to(torch.float64), distribution.loc,
                                     distribution._unbroadcasted_scale_tril)
    return lp
