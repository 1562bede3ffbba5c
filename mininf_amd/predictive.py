"""
Predictive draws on the HIP samplers: the sites ``broadcast_samples`` (reference
``core.py:548-584``) has to simulate -- ``SampleTracer.sample`` draws them with the distribution's
own ``sample`` (``core.py:192-204``) -- come from the same counter-based Philox generator as the
guide draws (``mi_normal_rsample`` / ``mi_gamma_rsample`` / ``mi_beta_rsample``), so a predictive
run is reproducible from one seed and independent of how the samples are batched or sharded.

Inside the vmapped predictive trace (:func:`mininf_amd.particles.broadcast_particles`) a site's
parameters are batched over the S samples. :class:`_DrawFn` carries a vmap rule: it receives the
physical ``[S, ...]`` parameters, broadcasts them to ``[S, *sample_shape, *batch_shape]`` and draws
all S samples in one launch. The generator counter of element j of sample s is
(seed, stream = the site's draw index, element s * M + j) with M the per-sample element count.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence, Tuple

import torch
from torch.distributions import Beta, Distribution, Gamma, Normal

from . import _native as nat

NORMAL, GAMMA, BETA = 0, 1, 2
# stream ids of predictive draws: apart from the guide factors' (their factor index)
STREAM_BASE = 0x50000


def _params(distribution: Distribution) -> Optional[Tuple[int, Sequence[torch.Tensor]]]:
    cls = type(distribution)
    if cls is Normal:
        return NORMAL, (distribution.loc, distribution.scale)
    if cls is Gamma:
        return GAMMA, (distribution.concentration, distribution.rate)
    if cls is Beta:
        return BETA, (distribution.concentration1, distribution.concentration0)
    return None


def supported(distribution: Distribution) -> bool:
    """Whether the HIP samplers draw this distribution (Normal / Gamma / Beta, float32 device)."""
    found = _params(distribution)
    if found is None:
        return False
    return all(isinstance(t, torch.Tensor) and t.dtype == torch.float32 and t.is_cuda
               for t in found[1])


def _launch(family: int, params: Sequence[torch.Tensor], N: int, seed: int,
            stream_id: int) -> torch.Tensor:
    """One launch drawing N values with per-element parameters (flat, contiguous)."""
    device = params[0].device
    out = torch.empty(N, dtype=torch.float32, device=device)
    a, b = (p.contiguous() for p in params)
    stream = nat.stream_handle(device)
    lib = nat.lib()
    seed &= 0xFFFFFFFFFFFFFFFF
    if family == NORMAL:
        nat.check(lib.mi_normal_rsample(a.data_ptr(), 1, b.data_ptr(), 1, 1, N, seed, 0, None,
                                        stream_id, 0, 0, None, out.data_ptr(), stream),
                  "mi_normal_rsample")
    elif family == GAMMA:
        g = torch.empty(N, dtype=torch.float32, device=device)
        nat.check(lib.mi_gamma_rsample(a.data_ptr(), 1, b.data_ptr(), 1, 1, N, seed, 0, None,
                                       stream_id, 0, None, g.data_ptr(), out.data_ptr(), stream),
                  "mi_gamma_rsample")
    else:
        nat.check(lib.mi_beta_rsample(a.data_ptr(), 1, b.data_ptr(), 1, 1, N, seed, 0, None,
                                      stream_id, 0, None, out.data_ptr(), stream),
                  "mi_beta_rsample")
    return out


class _DrawFn(torch.autograd.Function):
    """draw(index, a, b): one draw per sample; `index` (the sample number, batched under vmap)
    forces the batched rule even when no parameter depends on the sample."""
    @staticmethod
    def forward(index, a, b, family, shape, seed, stream_id):  # type: ignore[override]
        # unbatched call (one sample): the sample's own counter block
        target = tuple(shape) + tuple(torch.broadcast_shapes(a.shape, b.shape))
        M = max(1, math.prod(target))
        flat = [p.expand(target).reshape(M) for p in (a, b)]
        return _launch(family, flat, M, seed, stream_id).reshape(target)

    @staticmethod
    def setup_context(ctx, inputs, output):  # type: ignore[override]
        ctx.mark_non_differentiable(output)

    @staticmethod
    def vmap(info, in_dims, index, a, b, family, shape, seed, stream_id):  # type: ignore[override]
        S = info.batch_size
        logical = []
        phys = []
        for t, d in zip((a, b), in_dims[1:3]):
            t = t.movedim(d, 0) if d is not None else t.expand(S, *t.shape)
            phys.append(t)
            logical.append(tuple(t.shape[1:]))
        batch = tuple(torch.broadcast_shapes(*logical))
        target = (S,) + tuple(shape) + batch
        M = max(1, math.prod(target[1:]))
        flat = []
        for t, lg in zip(phys, logical):
            t = t.reshape(S, *([1] * (len(shape) + len(batch) - len(lg))), *lg)
            flat.append(t.expand(target).reshape(S * M))
        out = _launch(family, flat, S * M, seed, stream_id).reshape(target)
        # the samples in the order of `index` (broadcast_particles passes arange(S))
        return out, 0


def draw(distribution: Distribution, sample_shape: torch.Size, index: torch.Tensor, seed: int,
         stream_id: int) -> torch.Tensor:
    """``distribution.sample(sample_shape)`` inside the predictive vmap, on the HIP samplers."""
    found = _params(distribution)
    assert found is not None
    family, (a, b) = found
    with torch.no_grad():
        return _DrawFn.apply(index, a.detach(), b.detach(), family, tuple(sample_shape), seed,
                             STREAM_BASE + stream_id)
