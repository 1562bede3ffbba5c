"""
Reparameterised guide sampling over K particles (replaces ``FactorizedDistribution.rsample``,
reference ``mininf/nn.py:133-145``, with ONE draw per call at ``nn.py:217``).

Normal, Beta and Gamma factors are drawn by HIP kernels from a counter-based Philox generator keyed
by (seed, step, factor index, global particle index, element), so that K particles split over W GPUs
draw exactly the union of what one GPU would draw. Other families (MultivariateNormal, ...) use
their own ``torch.distributions`` ``rsample`` on the device.

Parity mode: ``noise[name]`` injects host-drawn standard normals (Normal factors, [K, *shape]),
the draws themselves (Beta factors) or the standard Gamma draws g with x = g / rate (Gamma
factors), exactly as the oracle's sample-injection protocol does.
"""
from __future__ import annotations

import ctypes
import dataclasses
import os
from typing import Dict, Optional, Tuple

import torch
from torch.distributions import Beta, Distribution, Gamma, Normal

from . import _native as nat


@dataclasses.dataclass
class DrawConfig:
    K: int
    seed: int
    step: int
    stream_id: int
    particle_offset: int
    noise: Optional[torch.Tensor] = None
    step_device: Optional[torch.Tensor] = None   # uint64 word added to `step` on the device
    # The word holding this evaluation's step once the forward has advanced `step_device`
    # (mi_elbo.step_snapshot): read by every kernel that runs after the ELBO forward.
    step_snapshot: Optional[torch.Tensor] = None
    # global index of element 0 (data-sharded factors, mininf_amd.distributed.DataShard)
    element_offset: int = 0
    # the factor is data-sharded (every rank draws its slice), also on the rank whose slice
    # starts at element 0
    sharded: bool = False
    # small Normal factors: leave the launch to the loss's planning (PendingDraw), which may hand
    # the draw to the linear site kernel that reads it (mi_linear.draw)
    defer: bool = False


def backward_step(cfg: DrawConfig) -> Optional[torch.Tensor]:
    """The device step word of a draw's backward (regenerated noise)."""
    return cfg.step_snapshot if cfg.step_snapshot is not None else cfg.step_device


def use_snapshot(cfg: DrawConfig) -> None:
    """Re-evaluate a forward after its ELBO advanced the generator: draw from the snapshot."""
    if cfg.step_snapshot is not None:
        cfg.step_device = cfg.step_snapshot


def _flat_param(t: torch.Tensor, N: int) -> Tuple[torch.Tensor, int]:
    """
    View a parameter of the factor's batch shape as [N] with a single stride (0 for broadcast
    scalars, 1 for contiguous), materialising it otherwise.
    """
    if t.dtype != torch.float32:
        raise nat.NativeError(f"guide parameters must be float32, got {t.dtype}")
    if t.numel() == 1:
        flat = t.reshape(1).expand(N)
        return flat, 0
    flat = t.reshape(N)
    if flat.stride(0) not in (0, 1):
        flat = flat.contiguous()
    return flat, flat.stride(0)


def _philox_key(cfg: DrawConfig) -> Tuple[int, int]:
    return cfg.seed & 0xFFFFFFFFFFFFFFFF, cfg.step & 0xFFFFFFFFFFFFFFFF


class _NormalRsampleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg: DrawConfig, loc: torch.Tensor, loc_s: int, scale: torch.Tensor,
                scale_s: int):  # type: ignore[override]
        N = loc.shape[0]
        K = cfg.K
        z = torch.empty((K, N), dtype=torch.float32, device=loc.device)
        draw = PendingDraw(cfg, z, loc, loc_s, scale, scale_s, exp_source(scale))
        if cfg.defer and cfg.noise is None and (N % 4 == 0 or N == 1) and N <= DEFER_MAX_N and \
                os.environ.get("MININF_AMD_DRAW_IN_LINEAR", "1") != "0":
            _PENDING_DRAWS[_storage_of(z)] = draw   # launched by flush_draws, or taken
        else:
            draw.launch()
        ctx.cfg = cfg
        ctx.N = N
        ctx.save_for_backward(scale)
        ctx.scale_s = scale_s
        return z

    @staticmethod
    def backward(ctx, dz: torch.Tensor):  # type: ignore[override]
        cfg: DrawConfig = ctx.cfg
        (scale,) = ctx.saved_tensors
        N, K = ctx.N, cfg.K
        device = dz.device
        size = ctypes.c_size_t()
        lib = nat.lib()
        nat.check(lib.mi_normal_rsample_backward_workspace_bytes(K, N, ctypes.byref(size)),
                  "mi_normal_rsample_backward_workspace_bytes")
        workspace = torch.empty(max(1, size.value), dtype=torch.uint8, device=device)
        dloc = torch.empty(N, dtype=torch.float32, device=device)
        deps_scale = torch.empty(N, dtype=torch.float32, device=device)
        seed, step = _philox_key(cfg)
        nat.check(lib.mi_normal_rsample_backward(
            dz.data_ptr(), dz.stride(0), dz.stride(1), K, N, seed, step,
            nat.ptr(backward_step(cfg)), cfg.stream_id, cfg.particle_offset, cfg.element_offset,
            nat.ptr(cfg.noise), workspace.data_ptr(), size.value,
            dloc.data_ptr(), deps_scale.data_ptr(), nat.stream_handle(device)),
            "mi_normal_rsample_backward")
        # dz/dscale = eps: the kernel returns sum_k dz * eps directly.
        return None, dloc, None, deps_scale, None


def beta_concentration(distribution: Beta, N: int) -> torch.Tensor:
    """
    The [N, 2] (concentration1, concentration0) array torch's Beta keeps for its Dirichlet
    (beta.py:36-40), as one contiguous fp32 tensor: the sampler, its backward and the entropy read
    and write both parameters interleaved, so autograd needs no select/stack kernels.
    """
    dirichlet = getattr(distribution, "_dirichlet", None)
    conc = dirichlet.concentration if dirichlet is not None else \
        torch.stack([distribution.concentration1, distribution.concentration0], -1)
    if conc.dtype != torch.float32:
        raise nat.NativeError(f"guide parameters must be float32, got {conc.dtype}")
    conc = conc.reshape(N, 2)
    return conc if conc.is_contiguous() else conc.contiguous()


# ---- deferred exp transforms of Beta guides ---------------------------------------------------
# ParameterizedDistribution.forward of a Beta guide returns its [.., 2] concentration array
# before anything reads it; the guide's draw (mi_beta_rsample_exp) then computes exp(u) and
# writes the array itself, so the transform needs no launch of its own. Any other reader (torch
# argument validation, .mean, a user's own use) launches the transform first (mi_transform_params).

@dataclasses.dataclass(eq=False)
class _PendingExp:
    out: "weakref.ReferenceType"
    u1: torch.Tensor
    u0: Optional[torch.Tensor]   # None: a single positive parameter (a Normal guide's scale)
    params: object          # the mi_params of the transform launch
    filled: bool = False


_PENDING_EXP: Dict[int, _PendingExp] = {}


def _storage_of(tensor) -> Optional[int]:
    if not isinstance(tensor, torch.Tensor):
        return None
    try:
        return tensor.untyped_storage().data_ptr()
    except (RuntimeError, NotImplementedError):
        return None


def pending_exp(tensor) -> Optional[_PendingExp]:
    """The pending transform a concentration array (or a view of it) waits for, or None."""
    if not _PENDING_EXP:
        return None
    rec = _PENDING_EXP.get(_storage_of(tensor))
    if rec is None or rec.filled or rec.out() is None:
        return None
    return rec


def exp_source(scale) -> Optional[Tuple[_PendingExp, int]]:
    """
    For a Normal guide scale still waiting for its exp transform: the record and the address of
    the unconstrained parameter element that becomes ``scale``'s first element, so a kernel can
    read exp(u) at ``scale``'s own offset and strides and write it (mi_normal_rsample_exp,
    mi_draw.scale_exp). None when nothing is pending or the layouts differ.
    """
    rec = pending_exp(scale)
    out = rec.out() if rec is not None else None
    if out is None or rec.u0 is not None or not rec.u1.is_contiguous() or \
            not out.is_contiguous() or tuple(rec.u1.shape) != tuple(out.shape):
        return None
    # u has the layout of the (contiguous) transform output: same offset, same strides
    return rec, rec.u1.data_ptr() + (scale.data_ptr() - out.data_ptr())


def fill_exp(tensor) -> None:
    """Launch a pending transform (mi_transform_params) before its array is read."""
    rec = pending_exp(tensor)
    if rec is None:
        return
    out = rec.out()
    nat.check(nat.lib().mi_transform_params(ctypes.byref(rec.params), out.data_ptr(),
                                            nat.stream_handle(out.device)), "mi_transform_params")
    rec.filled = True


def _forget_exp(ptr: int, rec: _PendingExp) -> None:
    if _PENDING_EXP.get(ptr) is rec:
        del _PENDING_EXP[ptr]


def defer_exp(out: torch.Tensor, u1: torch.Tensor, u0: Optional[torch.Tensor],
              params) -> torch.Tensor:
    """Register `out` (a PendingConcentration) as the pending exp-stack of (u1, u0). The record
    lives as long as `out` does; views of it keep `out` alive."""
    import weakref
    ptr = _storage_of(out)
    rec = _PendingExp(weakref.ref(out), u1, u0, params)
    _PENDING_EXP[ptr] = rec
    weakref.finalize(out, _forget_exp, ptr, rec)
    return out


_PENDING_METADATA = {
    torch.Tensor.size, torch.Tensor.dim, torch.Tensor.ndimension, torch.Tensor.numel,
    torch.Tensor.__len__, torch.Tensor.is_floating_point, torch.Tensor.stride,
    torch.Tensor.element_size, torch.Tensor.data_ptr, torch.Tensor.untyped_storage,
    torch.Tensor.storage_offset, torch.Tensor.is_contiguous, torch.Tensor.shape.__get__,
    torch.Tensor.dtype.__get__, torch.Tensor.device.__get__, torch.Tensor.ndim.__get__,
    torch.Tensor.requires_grad.__get__, torch.Tensor.is_cuda.__get__, torch.Tensor.layout.__get__,
    torch.Tensor.grad_fn.__get__, torch.Tensor.is_leaf.__get__, torch.Tensor.__hash__,
    torch.Tensor._version.__get__, torch.Tensor.reshape, torch.Tensor.view,
}


# views (no value read): the results stay pending
_PENDING_VIEWS = {torch.Tensor.reshape, torch.Tensor.view, torch.Tensor.expand,
                  torch.Tensor.expand_as, torch.broadcast_to, torch.Tensor.broadcast_to,
                  torch.broadcast_tensors, torch.functional.broadcast_tensors}


class PendingConcentration(torch.Tensor):
    """A guide parameter array whose exp transform has not run yet (a Beta guide's concentrations,
    a Normal guide's scale; see above): shape queries, views and pointer reads pass through;
    anything else launches the transform first."""
    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        copies = func is torch.Tensor.reshape and args and isinstance(args[0], torch.Tensor) and \
            not args[0].is_contiguous()   # a reshape that copies reads the values
        if (func not in _PENDING_METADATA and func not in _PENDING_VIEWS) or copies:
            stack = [args, kwargs]
            while stack:
                x = stack.pop()
                if isinstance(x, PendingConcentration):
                    fill_exp(x)
                elif isinstance(x, (list, tuple)):
                    stack.extend(x)
                elif isinstance(x, dict):
                    stack.extend(x.values())
        with torch._C.DisableTorchFunctionSubclass():
            out = func(*args, **kwargs)
        if func in _PENDING_VIEWS:
            roots = [x for x in _flat_args(args) if isinstance(x, PendingConcentration)]

            def rewrap(t):
                if isinstance(t, torch.Tensor) and pending_exp(t) is not None:
                    t = t.as_subclass(PendingConcentration)
                    t._pending_root = roots   # keeps the pending records' tensors alive
                return t
            if isinstance(out, (tuple, list)):
                out = type(out)(rewrap(t) for t in out)
            else:
                out = rewrap(out)
        return out


def _flat_args(args):
    stack, flat = [args], []
    while stack:
        x = stack.pop()
        if isinstance(x, (list, tuple)):
            stack.extend(x)
        else:
            flat.append(x)
    return flat


class _BetaRsampleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg: DrawConfig, conc: torch.Tensor):  # type: ignore[override]
        N = conc.shape[0]
        K = cfg.K
        x = torch.empty((K, N), dtype=torch.float32, device=conc.device)
        seed, step = _philox_key(cfg)
        base = conc.data_ptr()
        pending = pending_exp(conc)
        if pending is not None:   # the guide's exp transform and the draw in one launch
            u1, u0 = pending.u1.reshape(-1), pending.u0.reshape(-1)
            nat.check(nat.lib().mi_beta_rsample_exp(
                u1.data_ptr(), u1.stride(0) if u1.numel() > 1 else 0, u0.data_ptr(),
                u0.stride(0) if u0.numel() > 1 else 0, base, K, N, seed, step,
                nat.ptr(cfg.step_device), cfg.stream_id, cfg.particle_offset, nat.ptr(cfg.noise),
                x.data_ptr(), nat.stream_handle(conc.device)), "mi_beta_rsample_exp")
            pending.filled = True
        else:
            nat.check(nat.lib().mi_beta_rsample(
                base, 2, base + 4, 2, K, N, seed, step, nat.ptr(cfg.step_device), cfg.stream_id,
                cfg.particle_offset, nat.ptr(cfg.noise), x.data_ptr(),
                nat.stream_handle(conc.device)), "mi_beta_rsample")
        ctx.save_for_backward(x, conc)
        ctx.K, ctx.N = K, N
        return x

    @staticmethod
    def backward(ctx, dx: torch.Tensor):  # type: ignore[override]
        x, conc = ctx.saved_tensors
        K, N = ctx.K, ctx.N
        device = dx.device
        size = ctypes.c_size_t()
        lib = nat.lib()
        nat.check(lib.mi_beta_rsample_backward_workspace_bytes(K, N, ctypes.byref(size)),
                  "mi_beta_rsample_backward_workspace_bytes")
        workspace = torch.empty(max(1, size.value), dtype=torch.uint8, device=device)
        dconc = torch.empty((N, 2), dtype=torch.float32, device=device)
        base, out = conc.data_ptr(), dconc.data_ptr()
        nat.check(lib.mi_beta_rsample_backward(
            dx.data_ptr(), dx.stride(0), dx.stride(1), x.data_ptr(), base, 2, base + 4, 2, K, N,
            workspace.data_ptr(), size.value, out, 2, out + 4, 2, nat.stream_handle(device)),
            "mi_beta_rsample_backward")
        return None, dconc


def gamma_params(distribution: Gamma, N: int) -> Tuple[torch.Tensor, int, torch.Tensor, int]:
    """(concentration, stride, rate, stride) of a Gamma factor viewed as [N]."""
    conc, conc_s = _flat_param(distribution.concentration, N)
    rate, rate_s = _flat_param(distribution.rate, N)
    return conc, conc_s, rate, rate_s


class _GammaRsampleFn(torch.autograd.Function):
    """
    Gamma.rsample (gamma.py:80-88) over K particles: mi_gamma_rsample, and its backward through
    torch._standard_gamma_grad restated in fp64 (mi_gamma_rsample_backward). ``cfg.noise`` injects
    the standard Gamma draws g (x = g / rate), the oracle's protocol for Gamma factors.
    """
    @staticmethod
    def forward(ctx, cfg: DrawConfig, conc: torch.Tensor, conc_s: int, rate: torch.Tensor,
                rate_s: int):  # type: ignore[override]
        N, K = conc.shape[0], cfg.K
        # a deferred exp transform of the guide's parameters runs before the sampler reads them
        # (no validation read has forced it when torch's argument validation is off, e.g. in a
        # captured step)
        fill_exp(conc)
        fill_exp(rate)
        x = torch.empty((K, N), dtype=torch.float32, device=conc.device)
        g = torch.empty((K, N), dtype=torch.float32, device=conc.device)
        seed, step = _philox_key(cfg)
        nat.check(nat.lib().mi_gamma_rsample(
            conc.data_ptr(), conc_s, rate.data_ptr(), rate_s, K, N, seed, step,
            nat.ptr(cfg.step_device), cfg.stream_id, cfg.particle_offset, nat.ptr(cfg.noise),
            g.data_ptr(), x.data_ptr(), nat.stream_handle(conc.device)), "mi_gamma_rsample")
        ctx.save_for_backward(g, conc, rate)
        ctx.strides = (conc_s, rate_s)
        ctx.K, ctx.N = K, N
        return x

    @staticmethod
    def backward(ctx, dx: torch.Tensor):  # type: ignore[override]
        g, conc, rate = ctx.saved_tensors
        conc_s, rate_s = ctx.strides
        K, N = ctx.K, ctx.N
        device = dx.device
        lib = nat.lib()
        size = ctypes.c_size_t()
        nat.check(lib.mi_gamma_rsample_backward_workspace_bytes(K, N, ctypes.byref(size)),
                  "mi_gamma_rsample_backward_workspace_bytes")
        workspace = torch.empty(max(1, size.value), dtype=torch.uint8, device=device)
        dconc = torch.empty(N, dtype=torch.float32, device=device)
        drate = torch.empty(N, dtype=torch.float32, device=device)
        nat.check(lib.mi_gamma_rsample_backward(
            dx.data_ptr(), dx.stride(0), dx.stride(1), g.data_ptr(), conc.data_ptr(), conc_s,
            rate.data_ptr(), rate_s, K, N, workspace.data_ptr(), size.value, dconc.data_ptr(), 1,
            drate.data_ptr(), 1, nat.stream_handle(device)), "mi_gamma_rsample_backward")
        # per element; a broadcast parameter's expand backward sums them
        return None, dconc, None, drate, None


# ---- deferred small Normal draws ---------------------------------------------------------------
# A small Normal factor's [K, N] draw (the regression's theta, N = P features) is made by the loss's
# planning instead of when the guide is drawn: when the only kernel that reads it is one linear
# site, that launch draws it (mi_linear.draw, one launch less per step); otherwise flush_draws
# launches mi_normal_rsample before anything reads it (the particle trace's torch operations flush
# through mininf_amd.linear.DeferredMatmul).
DEFER_MAX_N = 64   # MI_LINEAR_MAX_P

@dataclasses.dataclass(eq=False)
class PendingDraw:
    cfg: DrawConfig
    z: torch.Tensor
    loc: torch.Tensor
    loc_s: int
    scale: torch.Tensor
    scale_s: int
    source: Optional[Tuple["_PendingExp", int]]   # exp_source(scale) at draw time
    done: bool = False
    claimed: bool = False   # a planned linear launch will make it (engine.claim_linear_draws)

    def launch(self) -> None:
        """mi_normal_rsample (or _exp with the guide's pending exp transform) into z."""
        if self.done:
            return
        self.done = True
        cfg, loc, scale, z = self.cfg, self.loc, self.scale, self.z
        K, N = z.shape
        seed, step = _philox_key(cfg)
        if self.source is not None:
            # the guide's exp transform and the draw in one launch
            pending, u_ptr = self.source
            nat.check(nat.lib().mi_normal_rsample_exp(
                loc.data_ptr(), self.loc_s, u_ptr, self.scale_s, scale.data_ptr(), K, N, seed,
                step, nat.ptr(cfg.step_device), cfg.stream_id, cfg.particle_offset,
                cfg.element_offset, nat.ptr(cfg.noise), z.data_ptr(),
                nat.stream_handle(loc.device)), "mi_normal_rsample_exp")
            pending.filled = True
        else:
            fill_exp(scale)
            nat.check(nat.lib().mi_normal_rsample(
                loc.data_ptr(), self.loc_s, scale.data_ptr(), self.scale_s, K, N, seed, step,
                nat.ptr(cfg.step_device), cfg.stream_id, cfg.particle_offset, cfg.element_offset,
                nat.ptr(cfg.noise), z.data_ptr(), nat.stream_handle(loc.device)),
                "mi_normal_rsample")

    def describe(self, D) -> None:
        """Fill an mi_draw descriptor for the linear site kernel that takes this draw over."""
        cfg = self.cfg
        seed, step = _philox_key(cfg)
        D.operand, D.stream_id = 1, cfg.stream_id
        D.loc, D.loc_stride = self.loc.data_ptr(), self.loc_s
        D.scale, D.scale_stride = self.scale.data_ptr(), self.scale_s
        D.scale_exp = self.source[1] if self.source is not None else None
        D.seed, D.step, D.step_device = seed, step, nat.ptr(cfg.step_device)
        D.particle_offset, D.element_offset = cfg.particle_offset, cfg.element_offset

    def taken(self) -> None:
        """The linear launch made the draw (and the pending exp transform of its scale)."""
        self.done = True
        if self.source is not None:
            self.source[0].filled = True


_PENDING_DRAWS: Dict[Optional[int], PendingDraw] = {}


def pending_draw(tensor) -> Optional[PendingDraw]:
    """The not yet launched draw whose storage `tensor` (or a batched view of it) reads, or None."""
    if not _PENDING_DRAWS or not isinstance(tensor, torch.Tensor):
        return None
    functorch = torch._C._functorch
    base = tensor
    while functorch.is_batchedtensor(base):
        base = functorch.get_unwrapped(base)
    rec = _PENDING_DRAWS.get(_storage_of(base))
    return rec if rec is not None and not rec.done else None


def flush_draws(claimed: bool = False) -> None:
    """Launch every deferred draw no linear launch has claimed (with ``claimed``, those too)
    before anything reads them."""
    for key, rec in list(_PENDING_DRAWS.items()):
        if claimed or not rec.claimed:
            del _PENDING_DRAWS[key]
            rec.launch()


def take_draw(rec: PendingDraw) -> None:
    rec.taken()
    _PENDING_DRAWS.pop(_storage_of(rec.z), None)


@dataclasses.dataclass(eq=False)   # identity semantics: used in sets
class LazyDraw:
    r"""
    A Normal factor's K draws left to the site kernels (``mi_draw``): the model is traced with
    ``placeholder`` -- a [K, *shape] zero-stride view of a private one-element buffer, recognised
    by its data pointer -- and site groups that read it compute ``loc + eps * scale`` in registers
    (the same Philox eps as :class:`_NormalRsampleFn`). Any other use of the draw in the model
    makes the loss re-trace with :meth:`materialize`\ d draws.
    """
    cfg: DrawConfig
    loc: torch.Tensor
    loc_s: int
    scale: torch.Tensor
    scale_s: int
    N: int
    shape: torch.Size
    placeholder: torch.Tensor
    real: Optional[torch.Tensor] = None

    def materialize(self) -> torch.Tensor:
        if self.real is None:
            z = _NormalRsampleFn.apply(self.cfg, self.loc, self.loc_s, self.scale, self.scale_s)
            self.real = z.reshape((self.cfg.K,) + tuple(self.shape))
            _DRAWN[self.real.data_ptr()] = Drawn(NORMAL_FAMILY, self.cfg, z, self.N)
        return self.real


# data pointer of a live placeholder -> its draw (reset by every lazy draw_all)
_LAZY: Dict[int, LazyDraw] = {}

NORMAL_FAMILY, BETA_FAMILY = "normal", "beta"


@dataclasses.dataclass(eq=False)
class Drawn:
    """
    A materialised guide draw of the last draw_all: ``base`` is the [K, N] output of the sampler's
    autograd node (Normal: :class:`_NormalRsampleFn`, Beta: :class:`_BetaRsampleFn`), from which
    the ELBO can take over the draw's backward (``mi_factor`` absorbed draws).
    """
    family: str
    cfg: DrawConfig
    base: torch.Tensor
    N: int
    dgrad: Optional[torch.Tensor] = None   # Beta: mi_beta_dgrad factors [K, N, 2] (side stream)
    conc: Optional[torch.Tensor] = None    # Beta: the interleaved [N, 2] concentration drawn from


# data pointer of a materialised draw -> its record (reset by every draw_all)
_DRAWN: Dict[int, Drawn] = {}

# Work launched on a side stream by the draws (Beta implicit-gradient factors) that the main
# stream has not joined yet: joined by join_side() before the ELBO reads it, and always before a
# captured step ends.
_SIDE_STREAMS: Dict[int, torch.cuda.Stream] = {}
_PENDING: list = []
# fp64 [K, N, 2] factors up to this many draws (64 MiB); larger Beta factors are evaluated inside
# mi_elbo_forward as before
BETA_DGRAD_MAX = 1 << 22


def _side_stream(device: torch.device) -> torch.cuda.Stream:
    index = device.index if device.index is not None else torch.cuda.current_device()
    stream = _SIDE_STREAMS.get(index)
    if stream is None:
        stream = _SIDE_STREAMS[index] = torch.cuda.Stream(device=device)
    return stream


def join_side() -> None:
    """Make the current stream wait for the side-stream work of the last draws."""
    if not _PENDING:
        return
    current = torch.cuda.current_stream()
    for event in _PENDING:
        current.wait_event(event)
    _PENDING.clear()


def _beta_dgrad(x: torch.Tensor, conc: torch.Tensor, K: int, N: int) -> Optional[torch.Tensor]:
    """
    Launch mi_beta_dgrad for the draws x on the side stream (MININF_AMD_BETA_DGRAD=1): its fp64
    chains depend only on the draws, so they can run beside the site kernels instead of inside
    mi_elbo_forward. Off by default: measured on MI355X (C2, hipGraph replay) the two-queue graph
    cost more per node than the overlap saved (0.17 -> 0.24 ms per step).
    """
    if not (torch.is_grad_enabled() and conc.requires_grad) or K * N > BETA_DGRAD_MAX or \
            os.environ.get("MININF_AMD_BETA_DGRAD", "0") != "1":
        return None
    main = torch.cuda.current_stream()
    side = _side_stream(x.device)
    out = torch.empty((K, N, 2), dtype=torch.float64, device=x.device)
    side.wait_stream(main)
    base = conc.data_ptr()
    nat.check(nat.lib().mi_beta_dgrad(x.data_ptr(), base, 2, base + 4, 2, K, N, out.data_ptr(),
                                      side.cuda_stream), "mi_beta_dgrad")
    event = torch.cuda.Event()
    event.record(side)
    # main-stream tensors used on the side stream: not reused before the side work is done
    for t in (x, conc, out):
        t.record_stream(side)
    _PENDING.append(event)
    return out


def release_lazy() -> None:
    """
    Forget the placeholders and draw records of the last draw_all (the loss has planned its
    kernels; holding them would keep the step's autograd graph alive).
    """
    _LAZY.clear()
    _DRAWN.clear()
    flush_draws(claimed=True)


def drawn_of(tensor) -> Optional[Drawn]:
    """The materialised draw a sample tensor (or a view sharing its storage start) is, or None."""
    if not _DRAWN or not isinstance(tensor, torch.Tensor):
        return None
    try:
        return _DRAWN.get(tensor.data_ptr())
    except RuntimeError:
        return None


def lazy_of(tensor) -> Optional[LazyDraw]:
    """
    The lazy draw a tensor (a placeholder, a broadcast view of one, or a batched view inside the
    particle vmap) stands for, or None.
    """
    if not _LAZY or not isinstance(tensor, torch.Tensor):
        return None
    functorch = torch._C._functorch
    base = tensor
    while functorch.is_batchedtensor(base):
        base = functorch.get_unwrapped(base)
    try:
        return _LAZY.get(base.data_ptr())
    except RuntimeError:  # tensors without storage
        return None


def _fusable_normal(distribution: Normal, N: int) -> bool:
    return (N >= 512 and N % 4 == 0 and distribution.loc.is_cuda and
            distribution.loc.dtype == torch.float32 and distribution.scale.dtype == torch.float32
            and os.environ.get("MININF_AMD_FUSE_DRAWS", "1") != "0")


def draw(distribution: Distribution, cfg: DrawConfig, lazy: bool = False) -> torch.Tensor:
    """
    K reparameterised draws of one guide factor: shape [K, *batch_shape, *event_shape].
    """
    cls = type(distribution)
    if (cfg.sharded or cfg.element_offset) and cls is not Normal:
        raise nat.NativeError(f"a data-sharded guide factor must be a Normal (got {cls.__name__}): "
                              "only the Normal sampler draws element slices of a global draw")
    if cfg.element_offset % 4:
        raise ValueError(f"element offset {cfg.element_offset} of a data-sharded factor is not a "
                         "multiple of 4 (mininf_amd.distributed.DataShard aligns slices)")
    if cls is Normal:
        shape = distribution.batch_shape
        N = max(1, int(shape.numel()))
        nat.require_device(distribution.loc, "guide Normal.loc")
        loc, loc_s = _flat_param(distribution.loc, N)
        scale, scale_s = _flat_param(distribution.scale, N)
        if cfg.noise is not None:
            cfg.noise = cfg.noise.to(device=loc.device, dtype=torch.float32).reshape(cfg.K, N) \
                .contiguous()
        elif lazy and _fusable_normal(distribution, N):
            # never read (recognised by its address; other uses re-trace with real draws)
            buffer = torch.empty(1, dtype=torch.float32, device=loc.device)
            placeholder = buffer.expand((cfg.K,) + tuple(shape))
            _LAZY[buffer.data_ptr()] = LazyDraw(cfg, loc, loc_s, scale, scale_s, N,
                                                torch.Size(shape), placeholder)
            return placeholder
        z = _NormalRsampleFn.apply(cfg, loc, loc_s, scale, scale_s)
        _DRAWN[z.data_ptr()] = Drawn(NORMAL_FAMILY, cfg, z, N)
        return z.reshape((cfg.K,) + tuple(shape))
    if cls is Beta:
        shape = distribution.batch_shape
        N = max(1, int(shape.numel()))
        conc = beta_concentration(distribution, N)
        nat.require_device(conc, "guide Beta concentration")
        if cfg.noise is not None:
            cfg.noise = cfg.noise.to(device=conc.device, dtype=torch.float32).reshape(cfg.K, N) \
                .contiguous()
        x = _BetaRsampleFn.apply(cfg, conc)
        _DRAWN[x.data_ptr()] = Drawn(BETA_FAMILY, cfg, x, N, _beta_dgrad(x, conc, cfg.K, N),
                                     conc)
        return x.reshape((cfg.K,) + tuple(shape))
    if cls is Gamma:
        shape = distribution.batch_shape
        N = max(1, int(shape.numel()))
        nat.require_device(distribution.concentration, "guide Gamma concentration")
        conc, conc_s, rate, rate_s = gamma_params(distribution, N)
        if cfg.noise is not None:   # injected standard draws g, [K, *shape]
            cfg.noise = cfg.noise.to(device=conc.device, dtype=torch.float32).reshape(cfg.K, N) \
                .contiguous()
        x = _GammaRsampleFn.apply(cfg, conc, conc_s, rate, rate_s)
        return x.reshape((cfg.K,) + tuple(shape))
    if cfg.noise is not None:
        return cfg.noise
    return distribution.rsample(torch.Size([cfg.K]))


def draw_all(approximation: Dict[str, Distribution], K: int, seed: int, step: int,
             particle_offset: int, noise: Optional[Dict[str, torch.Tensor]] = None,
             step_device: Optional[torch.Tensor] = None,
             lazy: bool = False,
             step_snapshot: Optional[torch.Tensor] = None,
             element_offsets: Optional[Dict[str, int]] = None) -> Dict[str, torch.Tensor]:
    """
    Draw every factor of a factorised guide (dict order = stream id order). With ``lazy``, large
    Normal factors become :class:`LazyDraw` placeholders evaluated inside the site kernels.
    ``element_offsets``: global index of element 0 of data-sharded factors (multiples of 4).
    """
    _LAZY.clear()
    _DRAWN.clear()
    flush_draws(claimed=True)
    samples = {}
    for stream_id, (name, factor) in enumerate(approximation.items()):
        cfg = DrawConfig(K=K, seed=seed, step=step, stream_id=stream_id,
                         particle_offset=particle_offset,
                         noise=None if noise is None else noise.get(name),
                         step_device=step_device, step_snapshot=step_snapshot,
                         element_offset=(element_offsets or {}).get(name, 0),
                         sharded=element_offsets is not None and name in element_offsets,
                         defer=lazy)
        samples[name] = draw(factor, cfg, lazy)
    return samples
