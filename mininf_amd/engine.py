"""
ELBO engine: turns a :class:`~mininf_amd.particles.ParticleTrace` into HIP site-kernel launches and
wires them into autograd.

Per step (one ``EvidenceLowerBoundLoss.forward``):

1. sites that share their element space and a dense operand are grouped (at most 4 sites, 6
   operands) so the operand is streamed from HBM once and its gradient written once;
2. each group runs ``mi_group_forward`` (``include/mininf_amd.h``), which returns the per-particle
   totals ``T_k`` and -- speculatively, because the ELBO is linear in ``T`` -- the gradients of all
   operands, pre-multiplied by the upstream gradient the ELBO will send (``g0 = -1/K``);
3. in backward, ``mi_scale_rows`` leaves those buffers untouched when the upstream really is
   ``g0`` (every thread block exits after one comparison) and rescales them otherwise.

Gradient modes per operand: DENSE (one value per particle and element: written in the operand's
own layout), PARTICLE (one scalar per particle: reduced over elements inside the kernel).
"""
from __future__ import annotations

import collections
import ctypes
import dataclasses
import functools
import os
import sys
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _native as nat
from . import data, graph, guide, particles
from .particles import ParticleTrace, SiteRecord


# Optional instrumentation (bench.py): an object with `pair(launcher) -> (start, stop)` returning
# torch.cuda.Event pairs (already created, or None) that mi_group_forward_deferred /
# mi_linear_forward_deferred record around the main site kernel of each launch, and
# `stamps(launcher) -> device address or None` of a (min start, max end) clock-stamp pair the
# kernel's workgroups fold their span into (mi_group.stamps).
KERNEL_TIMER = None

FAMILY_CODES = {
    "normal": nat.NORMAL,
    "bernoulli_logits": nat.BERNOULLI_LOGITS,
    "bernoulli_probs": nat.BERNOULLI_PROBS,
    "beta": nat.BETA,
    "gamma": nat.GAMMA,
    "poisson": nat.POISSON,
    "inverse_gamma": nat.INVERSE_GAMMA,
}


def _collapse(t: torch.Tensor, K: int, shape: torch.Size) -> "_View":
    """
    Describe a [K, *R] tensor (R broadcastable to ``shape``) over the logical [K, N] element space
    (N = numel(shape)). Per-particle scalars stay [K, 1] tensors with element stride 0 (their
    gradient is reduced in the kernel); broadcast and collapsible dims stay views; anything else is
    materialised by ``reshape``.
    """
    if t.dim() == 0:
        t = t.expand(K)
    R = tuple(t.shape[1:])
    N = int(torch.Size(shape).numel())
    if int(torch.Size(R).numel()) == 1:
        base = t.reshape(K, 1)
        return _View(base, base.stride(0), 0)
    if R == tuple(shape):   # already [K, *shape]: no broadcast view needed
        flat = t if len(R) == 1 else t.reshape(K, N)
        return _View(flat, flat.stride(0), flat.stride(1) if N > 1 else 1)
    full = t.reshape((K,) + (1,) * (len(shape) - len(R)) + R).expand((K,) + tuple(shape))
    flat = full.reshape(K, N)
    return _View(flat, flat.stride(0), flat.stride(1) if N > 1 else 1)


_DEVICE_CACHE: "collections.OrderedDict[Tuple, Tuple[torch.Tensor, torch.Tensor]]" = \
    collections.OrderedDict()


def _to_device(t: torch.Tensor, K: int, device: torch.device, what: str,
               allow_constant: bool = True) -> Tuple[Optional[torch.Tensor], Optional[float]]:
    """
    Bring a site tensor to the engine's device. Models written against the reference build
    distributions from Python numbers and CPU data (e.g. ``Beta(2, 2)``): such unbatched host values
    become kernel constants (scalars) or cached device copies (tensors, keyed on storage and
    version). Returns (tensor, None) or (None, constant).
    """
    if t.device == device:
        if allow_constant and not t.requires_grad and (t.dim() == 0 or t.stride(0) == 0):
            # a number of a distribution built in a captured step (mininf_amd.graph)
            value = graph.CONSTANT_VALUES.get(t.data_ptr())
            if value is not None and (t.dim() == 0 or t[0].numel() == 1):
                return None, value
        return t, None
    if t.device.type != "cpu":
        raise nat.NativeError(f"{what} lives on {t.device}, expected {device}")
    if t.requires_grad:
        raise nat.NativeError(f"{what} requires grad but lives on the CPU; move it to {device}")
    unbatched = t.dim() > 0 and t.stride(0) == 0
    base = t[0] if unbatched else t
    if allow_constant and unbatched and base.numel() == 1:
        return None, float(base.reshape(()))
    key = (base.data_ptr(), tuple(base.shape), tuple(base.stride()), base.dtype, base._version,
           str(device))
    hit = _DEVICE_CACHE.get(key)
    if hit is None:
        hit = (base, base.to(device))
        _DEVICE_CACHE[key] = hit
        while len(_DEVICE_CACHE) > 64:
            _DEVICE_CACHE.popitem(last=False)
    else:
        _DEVICE_CACHE.move_to_end(key)
    moved = hit[1]
    return (moved.expand((K,) + tuple(moved.shape)) if unbatched else moved), None


def _float(t: torch.Tensor, what: str) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise nat.NativeError(f"{what}: the HIP site kernels compute in float32 (the reference's "
                              f"default dtype); got {t.dtype}.")
    return t


@dataclasses.dataclass
class _View:
    tensor: Optional[torch.Tensor]  # autograd input ([K, N] view, or [K, 1] per-particle scalars)
    sk: int                         # element strides over the logical [K, N] space
    si: int
    constant: Optional[float] = None  # host scalar (e.g. the 2.0 of `Beta(2, 2)`): no operand
    draw: Optional[guide.LazyDraw] = None  # a guide draw computed inside the kernel (mi_draw)

    @functools.cached_property
    def key(self) -> Tuple:
        """Identity of the operand (views are not modified after construction: computed once)."""
        if self.constant is not None:
            return ("constant", self.constant)
        if self.draw is not None:
            return ("draw", id(self.draw))
        t = self.tensor
        return (t.data_ptr(), tuple(t.shape), tuple(t.stride()), self.sk, self.si,
                t.requires_grad)

    @property
    def dense(self) -> bool:
        return self.constant is None and self.sk != 0 and self.si != 0

    @property
    def per_particle(self) -> bool:
        """One scalar per particle: the gradient is reduced over elements inside the kernel."""
        return self.constant is None and self.draw is None and self.tensor.shape[1] == 1 and \
            self.si == 0

    @property
    def requires_grad(self) -> bool:
        if self.draw is not None:
            return self.draw.loc.requires_grad or self.draw.scale.requires_grad
        return self.tensor.requires_grad


@dataclasses.dataclass
class _Operand:
    view: _View
    mode: int
    slot: int = -1


class _GroupLauncher:
    """
    Owns the ctypes descriptor of one site group and launches ``mi_group_forward``.
    """
    def __init__(self, K: int, N: int, g0: float, device: torch.device,
                 per_site: bool = False) -> None:
        self.K, self.N, self.g0, self.device = K, N, g0, device
        self.per_site = per_site  # also return each site's log density per particle (diagnostics)
        self.operands: List[_Operand] = []
        self.keys: Dict[Tuple, int] = {}
        self.sites: List[Tuple[SiteRecord, List[int], Optional[torch.Tensor]]] = []
        self.num_slots = 0
        # the fused draw's dloc / dscale partials stay in the workspace for the ELBO backward
        # (MI_GROUP_DRAW_PARTIALS); set by the ELBO plan when it absorbs the draw
        self.draw_partials = False
        self.exp_pending = None
        self.workspace: Optional[torch.Tensor] = None   # of the last run
        # Beta implicit-gradient factors carried as extra workgroups of this launch (mi_side):
        # (draws x [K, N], concentration [N, 2]) set by the ELBO plan; side_out is the [K, N, 2]
        # result of the last run, or None when the group's kernel cannot carry the job
        self.side: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
        self.side_out: Optional[torch.Tensor] = None
        # a one-element prior site folded into this launch (mi_prior, fold_priors): (site, family
        # code, (constant, constant)); its validation word follows the group's own
        self.prior: Optional[Tuple[SiteRecord, int, Tuple[float, float]]] = None
        # a deferred one-element Normal guide draw this launch makes itself (mi_group.pdraw,
        # claim_group_draws): (the draw, the operand index that reads it)
        self.pdraw: Optional[Tuple[guide.PendingDraw, int]] = None
        self.made_pdraw = False   # the last launch made that draw (EvidenceLowerBoundLoss.last_fusions)

    @property
    def flag_sites(self) -> List[SiteRecord]:
        """The sites whose validation words this launch writes, in word order."""
        return [site for site, _, _ in self.sites] + ([self.prior[0]] if self.prior else [])

    def try_add(self, site: SiteRecord, views: List[_View], mask: Optional[_View]) -> bool:
        constants = [v.constant for v in views]
        views_in = views
        views = [v for v in views if v.constant is None]
        new = {v.key for v in views if v.key not in self.keys}
        if len(self.sites) >= nat.MAX_SITES or len(self.operands) + len(new) > nat.MAX_OPERANDS:
            return False
        draws = {id(op.view.draw) for op in self.operands if op.view.draw is not None} | \
            {id(v.draw) for v in views if v.draw is not None}
        if len(draws) > 1:   # one fused draw per group
            return False
        grad_on = torch.is_grad_enabled()
        slots = len({v.key for v in views if v.key not in self.keys and v.per_particle
                     and v.requires_grad and grad_on})
        if self.num_slots + slots > nat.MAX_SLOTS:
            return False
        indices = []
        for v in views:
            if v.key not in self.keys:
                mode, slot = nat.GRAD_NONE, -1
                if v.requires_grad and grad_on:
                    if v.per_particle:
                        mode, slot = nat.GRAD_PARTICLE, self.num_slots
                        self.num_slots += 1
                    else:
                        mode = nat.GRAD_DENSE
                self.keys[v.key] = len(self.operands)
                self.operands.append(_Operand(v, mode, slot))
            indices.append(self.keys[v.key])
        it = iter(indices)
        roles = [(-1, c) if c is not None else (next(it), 0.0) for c in constants]
        assert len(roles) == len(views_in)
        self.sites.append((site, roles, mask))
        return True

    def shares_dense_operand(self, views: List[_View]) -> bool:
        return any(v.key in self.keys and v.dense for v in views)

    def inputs(self, skip: Sequence[int] = ()) -> List[Optional[torch.Tensor]]:
        """
        Autograd inputs: one per operand, two (loc, scale) for a fused draw; None for the operands
        in ``skip`` (draws whose backward the ELBO absorbs).
        """
        out: List[Optional[torch.Tensor]] = []
        for index, op in enumerate(self.operands):
            if op.view.draw is not None:
                out.extend([None, None] if index in skip else [op.view.draw.loc,
                                                               op.view.draw.scale])
            else:
                out.append(None if index in skip else op.view.tensor)
        return out

    @property
    def draw(self) -> Optional["guide.LazyDraw"]:
        return next((op.view.draw for op in self.operands if op.view.draw is not None), None)

    def draw_supported(self) -> bool:
        """
        Python mirror of sites.hip draw_supported (plus the specialiser being enabled): whether
        the group's fused draw can run, or has to be materialised before launching.
        """
        if self.draw is None:
            return True
        if os.environ.get("MININF_AMD_JIT", "1") == "0" or self.N % 4 or self.N < 512:
            return False
        for op in self.operands:
            v = op.view
            if v.draw is not None or v.constant is not None:
                continue
            if v.si != 0 and v.si != 1:
                return False
        for _, _, mask in self.sites:
            if mask is not None and (mask.sk != 0 or mask.si not in (0, 1)):
                return False
        return True

    def describe(self, compute_grads: bool, fuse_exp: bool = False, query: bool = False):
        """
        The ctypes ``mi_group`` descriptor of this group plus freshly allocated dense gradient
        buffers (one per DENSE operand, None otherwise). ``fuse_exp``: a fused draw whose guide
        scale still waits for its exp transform reads the unconstrained parameter instead
        (``mi_draw.scale_exp``); otherwise the transform is launched first. ``query``: for a plan
        query only (``mi_group_prior_supported``): nothing is launched or allocated -- no pending
        transform or gather runs, and dense gradients get a placeholder address.
        """
        device = self.device
        K, N = self.K, self.N
        group = nat.Group()
        group.K, group.N = K, N
        group.num_sites = len(self.sites)
        group.num_operands = len(self.operands)
        group.num_slots = self.num_slots if compute_grads else 0
        group.compute_grads = int(compute_grads)
        group.grad_scale = self.g0
        grads: List[Optional[torch.Tensor]] = []
        for index, op in enumerate(self.operands):
            desc = group.operands[index]
            view = op.view
            grad = None
            mode = op.mode if compute_grads else nat.GRAD_NONE
            if view.draw is not None:
                d = view.draw
                desc.data = None
                desc.stride_k, desc.stride_i = N, 1
                desc.grad_mode = mode
                dw = group.draw
                dw.operand = index + 1
                dw.stream_id = d.cfg.stream_id
                dw.loc, dw.loc_stride = d.loc.data_ptr(), d.loc_s
                dw.scale, dw.scale_stride = d.scale.data_ptr(), d.scale_s
                source = guide.exp_source(d.scale) if fuse_exp else None
                if source is not None:
                    # the guide's deferred exp transform runs inside the site program, which
                    # writes the scale for the autograd of the transform (run() marks it filled)
                    self.exp_pending, dw.scale_exp = source
                elif not query:
                    guide.fill_exp(d.scale)   # a deferred transform runs before the kernel reads it
                dw.seed, dw.step = guide._philox_key(d.cfg)
                dw.step_device = nat.ptr(d.cfg.step_device)
                dw.particle_offset = d.cfg.particle_offset
                dw.element_offset = d.cfg.element_offset
                if mode == nat.GRAD_DENSE and self.draw_partials:
                    group.options |= nat.GROUP_DRAW_PARTIALS
                elif mode == nat.GRAD_DENSE and query:
                    dw.dloc = dw.dscale = _QUERY_ADDRESS
                elif mode == nat.GRAD_DENSE:
                    dloc = torch.empty(N, dtype=torch.float32, device=device)
                    dscale = torch.empty(N, dtype=torch.float32, device=device)
                    dw.dloc, dw.dscale = dloc.data_ptr(), dscale.data_ptr()
                    grad = (dloc, dscale)
                grads.append(grad)
                continue
            if not query:
                data.ensure_filled(view.tensor)   # a minibatch read directly: gather its rows
            desc.data = view.tensor.data_ptr()
            desc.stride_k, desc.stride_i = view.sk, view.si
            if mode == nat.GRAD_DENSE and query:
                desc.grad = _QUERY_ADDRESS
                desc.grad_stride_k, desc.grad_stride_i = view.sk, view.si
            elif mode == nat.GRAD_DENSE:
                sk, si = view.sk, view.si
                if (sk, si) in ((N, 1), (1, K)):
                    grad = torch.empty_strided((K, N), (sk, si), dtype=torch.float32, device=device)
                else:
                    grad = torch.empty((K, N), dtype=torch.float32, device=device)
                desc.grad = grad.data_ptr()
                desc.grad_stride_k, desc.grad_stride_i = grad.stride()
            desc.grad_mode = mode
            desc.slot = op.slot if mode == nat.GRAD_PARTICLE else 0
            grads.append(grad)
        for index, (site, roles, mask) in enumerate(self.sites):
            desc = group.sites[index]
            desc.family = FAMILY_CODES[site.family]
            if site.family.startswith("bernoulli") or site.family == "poisson":
                roles = [roles[0], (-1, 0.0), roles[1]]   # one-parameter families
            for q in range(3):
                desc.operand[q] = roles[q][0]
                desc.constant[q] = roles[q][1]
            if mask is not None:
                if not query:
                    data.ensure_filled(mask.tensor)
                desc.mask = mask.tensor.data_ptr()
                desc.mask_stride_k, desc.mask_stride_i = mask.sk, mask.si
            desc.scale = site.scale
        if self.prior is not None:
            pr = group.prior
            pr.present, pr.family = 1, self.prior[1]
            pr.constant[0], pr.constant[1] = self.prior[2]
            pr.scale = self.prior[0].scale
        if self.pdraw is not None and not self.pdraw[0].done:
            rec, index = self.pdraw
            if rec.source is None and not query:
                # no fused exp for this scale: a deferred transform runs before the program reads
                # it (as for the operand draw above)
                guide.fill_exp(rec.scale)
            rec.describe(group.pdraw)
            group.pdraw.operand = index + 1
        return group, grads

    def source(self) -> str:
        """
        The specialised kernel source the library generates for this group (diagnostics).
        """
        group, _ = self.describe(True)
        needed = ctypes.c_size_t()
        lib = nat.lib()
        nat.check(lib.mi_group_source(ctypes.byref(group), None, 0, ctypes.byref(needed)),
                  "mi_group_source")
        buf = ctypes.create_string_buffer(needed.value)
        nat.check(lib.mi_group_source(ctypes.byref(group), buf, needed.value, None),
                  "mi_group_source")
        return buf.value.decode()

    def compile_check(self, compute_grads: bool = True) -> str:
        """
        Compile the specialised kernel with hiprtc (no device needed); raises with the log.
        """
        group, _ = self.describe(compute_grads)
        log = ctypes.create_string_buffer(1 << 16)
        code = nat.lib().mi_group_compile_check(ctypes.byref(group), log, len(log))
        if code != 0:
            raise nat.NativeError("site program failed to compile:\n" + log.value.decode())
        return log.value.decode()

    def run(self, compute_grads: bool, flags: Optional[torch.Tensor] = None,
            defer: bool = False):
        """
        Launch the group. ``flags``: an already-zeroed int32 slice (one word per site) to write the
        validation flags into, e.g. part of one buffer for every group of a step. ``defer``: leave
        the finalize reduction to the caller when the library allows (``self.reduce``, an
        ``mi_reduce``; None when the launch reduced itself).
        """
        device = self.device
        K, N = self.K, self.N
        self.exp_pending = None
        group, grads = self.describe(compute_grads, fuse_exp=True)
        if flags is None:
            flags = torch.empty(len(self.flag_sites), dtype=torch.int32, device=device)
        else:
            group.options |= nat.GROUP_FLAGS_ZEROED
        if self.prior is not None:   # its word after the group's own
            group.prior.flags = flags.data_ptr() + 4 * len(self.sites)
        size = ctypes.c_size_t()
        lib = nat.lib()
        nat.check(lib.mi_group_workspace_bytes(ctypes.byref(group), ctypes.byref(size)),
                  "mi_group_workspace_bytes")
        workspace = torch.empty(max(1, size.value), dtype=torch.uint8, device=device)
        self.side_out = None
        if self.side is not None:
            x, conc = self.side
            supported = ctypes.c_int(0)
            nat.check(lib.mi_group_side_supported(ctypes.byref(group), ctypes.byref(supported)),
                      "mi_group_side_supported")
            if supported.value:
                Ks, Ns = x.shape
                out = torch.empty((Ks, Ns, 2), dtype=torch.float64, device=device)
                sd = group.side
                sd.x, sd.c1, sd.c1_stride = x.data_ptr(), conc.data_ptr(), 2
                sd.c0, sd.c0_stride = conc.data_ptr() + 4, 2
                sd.K, sd.N, sd.out = Ks, Ns, out.data_ptr()
                nat.check(lib.mi_group_workspace_bytes(ctypes.byref(group), ctypes.byref(size)),
                          "mi_group_workspace_bytes")
                if workspace.numel() < size.value:
                    workspace = torch.empty(size.value, dtype=torch.uint8, device=device)
                self.side_out = out
        total = torch.empty(K, dtype=torch.float32, device=device)
        site_lp = torch.empty((len(self.sites), K), dtype=torch.float64, device=device) \
            if self.per_site else None
        slot_grad = torch.empty((max(1, group.num_slots), K), dtype=torch.float32, device=device)
        start = stop = None
        group.stamps = None   # (a cached descriptor must not keep an earlier timing slot)
        if KERNEL_TIMER is not None:
            start, stop = KERNEL_TIMER.pair(self)
            group.stamps = KERNEL_TIMER.stamps(self)
        reduce = nat.Reduce()

        def launch():
            return lib.mi_group_forward_deferred(
                ctypes.byref(group), workspace.data_ptr(), size.value, total.data_ptr(),
                nat.ptr(site_lp), slot_grad.data_ptr(), flags.data_ptr(),
                None if start is None else start.cuda_event,
                None if stop is None else stop.cuda_event,
                nat.stream_handle(device), ctypes.byref(reduce) if defer else None)
        code = launch()
        if group.pdraw.operand and code == nat.MI_EUNSUPPORTED:
            # this launch does not make the per-particle draw: the draw's own launch first
            rec = self.pdraw[0]
            rec.launch()
            guide.take_draw(rec)
            group.pdraw = nat.Draw()
            code = launch()
        nat.check(code, "mi_group_forward_deferred")
        self.made_pdraw = bool(group.pdraw.operand)
        if group.pdraw.operand:
            guide.take_draw(self.pdraw[0])
        if self.exp_pending is not None:
            self.exp_pending.filled = True
            self.exp_pending = None
        self.reduce = reduce if defer and reduce.part else None
        self.workspace = workspace
        self.partials = None
        if group.options & nat.GROUP_DRAW_PARTIALS:
            offset, rows = ctypes.c_size_t(), ctypes.c_int64()
            nat.check(lib.mi_group_draw_partials(ctypes.byref(group), ctypes.byref(offset),
                                                 ctypes.byref(rows)), "mi_group_draw_partials")
            self.partials = (workspace.data_ptr() + offset.value, rows.value)
        return total, site_lp, grads, slot_grad, flags


class _SiteGroupFn(torch.autograd.Function):
    """
    Autograd node of one site group: forward returns T_k (fp32 [K]); backward returns the
    speculative gradients (rescaled only if the upstream differs from g0).
    """
    @staticmethod
    def forward(ctx, launcher: _GroupLauncher, holder: dict, *inputs):  # type: ignore[override]
        need = any(op.mode != nat.GRAD_NONE for op in launcher.operands)
        total, site_lp, grads, slot_grad, flags = launcher.run(need)
        holder["flags"] = flags
        holder["site_lp"] = site_lp
        ctx.launcher = launcher
        ctx.grads = grads
        ctx.slot_grad = slot_grad
        return total

    @staticmethod
    def backward(ctx, g: torch.Tensor):  # type: ignore[override]
        launcher: _GroupLauncher = ctx.launcher
        grads, slot_grad = ctx.grads, ctx.slot_grad
        if grads is None:  # a second backward through the same graph: recompute
            _, _, grads, slot_grad, _ = launcher.run(True)
        ctx.grads = None
        g = g.contiguous()
        device = g.device
        out: List[Optional[torch.Tensor]] = []
        if launcher.num_slots:
            # slot gradients are speculative too (pre-multiplied by g0): slot_grad[j, k] is row k
            nat.check(nat.lib().mi_scale_rows(slot_grad.data_ptr(), 1, launcher.K, launcher.K,
                                              launcher.num_slots, g.data_ptr(), launcher.g0,
                                              nat.stream_handle(device)), "mi_scale_rows")
        for op, grad in zip(launcher.operands, grads):
            if op.mode == nat.GRAD_DENSE:
                sk, si = grad.stride()
                nat.check(nat.lib().mi_scale_rows(grad.data_ptr(), sk, si, launcher.K, launcher.N,
                                                  g.data_ptr(), launcher.g0,
                                                  nat.stream_handle(device)), "mi_scale_rows")
                out.append(grad)
            elif op.mode == nat.GRAD_PARTICLE:
                out.append(slot_grad[op.slot].reshape(launcher.K, 1))
            else:
                out.append(None)
        return (None, None, *out)


def _run_categorical(site: SiteRecord, g0: float, logits: torch.Tensor, value: torch.Tensor,
                     mask: Optional[torch.Tensor], need: bool,
                     flags: Optional[torch.Tensor] = None):
    """
    Launch ``mi_categorical_forward``: (total [K], speculative dlogits or None, flags [1]).
    """
    K, N, C = logits.shape
    device = logits.device
    dlogits = torch.empty_like(logits) if need else None   # every entry written
    size = ctypes.c_size_t()
    lib = nat.lib()
    nat.check(lib.mi_categorical_workspace_bytes(K, N, ctypes.byref(size)),
              "mi_categorical_workspace_bytes")
    workspace = torch.empty(max(1, size.value), dtype=torch.uint8, device=device)
    total = torch.empty(K, dtype=torch.float32, device=device)
    if flags is None:
        flags = torch.empty(1, dtype=torch.int32, device=device)
    nat.check(lib.mi_categorical_forward(
        logits.data_ptr(), logits.stride(0), logits.stride(1), logits.stride(2), K, N, C,
        value.data_ptr(), value.stride(0), value.stride(1),
        None if mask is None else mask.data_ptr(), 0 if mask is None else mask.stride(1),
        site.scale, g0, None if dlogits is None else dlogits.data_ptr(), workspace.data_ptr(),
        size.value, total.data_ptr(), flags.data_ptr(), nat.stream_handle(device)),
        "mi_categorical_forward")
    return total, dlogits, flags


class _CategoricalFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, site: SiteRecord, holder: dict, g0: float, logits: torch.Tensor,
                value: torch.Tensor, mask: Optional[torch.Tensor]):  # type: ignore[override]
        total, dlogits, flags = _run_categorical(site, g0, logits, value, mask,
                                                 logits.requires_grad)
        holder["flags"] = flags
        ctx.dlogits = dlogits
        ctx.g0 = g0
        return total

    @staticmethod
    def backward(ctx, g):  # type: ignore[override]
        dlogits = ctx.dlogits
        if dlogits is None:
            return None, None, None, None, None, None
        K, N, C = dlogits.shape
        g = g.contiguous()
        nat.check(nat.lib().mi_scale_rows(dlogits.data_ptr(), N * C, 1, K, N * C, g.data_ptr(),
                                          ctx.g0, nat.stream_handle(g.device)), "mi_scale_rows")
        return None, None, None, dlogits, None, None


# ------------------------------------------------------------------------------------------------
# Linear-predictor sites: Normal(X @ theta, sigma) / Bernoulli(logits = X @ theta), fused.
# ------------------------------------------------------------------------------------------------
class _LinearLauncher:
    """
    One ``mi_linear_forward`` site: the predictor ``X @ theta_k`` is evaluated inside the kernel
    (the model's matmul was deferred by :mod:`mininf_amd.linear`).
    """
    def __init__(self, site: SiteRecord, K: int, g0: float, device: torch.device,
                 theta: torch.Tensor, sigma: Optional[_View], value: _View,
                 mask: Optional[torch.Tensor]) -> None:
        self.site, self.K, self.g0, self.device = site, K, g0, device
        self.X = site.linear_X
        self.N, self.P = self.X.shape
        # device-resident minibatch read through its row index (mininf_amd.data): the dataset
        # columns of X and the value, and the batch's rows
        self.batch: Optional["data._Batch"] = None
        self.X_src, self.value_src = self.X, None
        self.theta = theta
        self.sigma = sigma
        self.sigma_input = None
        if sigma is not None and sigma.constant is None:
            self.sigma_input = sigma.tensor[:, :1]
        self.value = value
        self.mask = mask
        self.sites = [(site, None, mask)]   # flag layout: one word (+ the folded prior's)
        # a prior site over theta itself folded into this launch (mi_linear.prior,
        # fold_linear_priors): (site, family code, (constant, constant))
        self.prior: Optional[Tuple[SiteRecord, int, Tuple[float, float]]] = None
        # theta is a guide draw this launch makes itself (mi_linear.draw, guide.PendingDraw)
        self.draw: Optional[guide.PendingDraw] = None
        self.drew_theta = self.drew_rows = False   # what the last launch made itself
        # decided here, outside the autograd Function (whose forward runs with grad disabled)
        grad_on = torch.is_grad_enabled()
        self.theta_grad = grad_on and theta.requires_grad
        self.sigma_grad = grad_on and self.sigma_input is not None and \
            self.sigma_input.requires_grad

    @property
    def flag_sites(self) -> List[SiteRecord]:
        return [self.site] + ([self.prior[0]] if self.prior else [])

    def needs_grads(self) -> bool:
        return self.theta_grad or self.sigma_grad

    def inputs(self) -> List[Optional[torch.Tensor]]:
        return [self.theta, self.sigma_input]

    def describe(self, compute_grads: bool, draw_rows: bool = True,
                 query: bool = False, draw: bool = True) -> nat.Linear:
        """
        The ``mi_linear`` descriptor. ``query``: for a support query only -- a minibatch's rows
        are neither drawn nor taken (the descriptor reads the dataset's first rows).
        """
        L = nat.Linear()
        L.K, L.N, L.P = self.K, self.N, self.P
        L.family = FAMILY_CODES[self.site.family]
        L.x = self.X_src.data_ptr()
        L.x_stride_i, L.x_stride_j = self.X_src.stride()
        L.theta = self.theta.data_ptr()
        L.theta_stride_k, L.theta_stride_j = self.theta.stride()
        if self.batch is not None and query:
            L.value = self.value_src.data_ptr()
            L.value_stride_i = self.value_src.stride(0)
        elif self.batch is not None:
            # the batch's rows: drawn by this kernel when nothing has drawn them yet (one launch
            # less per step), else read through the row index
            R = self.batch.take_rows() if draw_rows else None
            if R is not None:
                L.rows = R
            else:
                L.row_index = self.batch.rows.data_ptr()
            L.value = self.value_src.data_ptr()
            L.value_stride_i = self.value_src.stride(0)
        else:
            data.ensure_filled(self.X)
            data.ensure_filled(self.value.tensor)
            L.value = self.value.tensor.data_ptr()
            L.value_stride_i = self.value.si
        if self.mask is not None:
            L.mask = self.mask.data_ptr()
            L.mask_stride_i = self.mask.stride(0) if self.N > 1 else 1
        if self.sigma is not None:
            if self.sigma.constant is not None:
                L.scale_constant = self.sigma.constant
            else:
                L.scale = self.sigma_input.data_ptr()
                L.scale_stride_k = self.sigma_input.stride(0)
        L.grad_scale = self.g0
        L.site_scale = self.site.scale
        L.compute_grads = int(compute_grads)
        if self.prior is not None:
            pr = L.prior
            pr.present, pr.family = 1, self.prior[1]
            pr.constant[0], pr.constant[1] = self.prior[2]
            pr.scale = self.prior[0].scale
        if draw and self.draw is not None and not self.draw.done:
            self.draw.describe(L.draw)
        return L

    def run(self, compute_grads: bool, flags: Optional[torch.Tensor] = None,
            defer: bool = False):
        device = self.device
        L = self.describe(compute_grads)
        if flags is None:
            flags = torch.empty(len(self.flag_sites), dtype=torch.int32, device=device)
        else:
            L.options |= nat.GROUP_FLAGS_ZEROED
        size = ctypes.c_size_t()
        lib = nat.lib()
        if self.prior is not None:   # its word after the site's
            L.prior.flags = flags.data_ptr() + 4
        nat.check(lib.mi_linear_workspace_bytes(ctypes.byref(L), ctypes.byref(size)),
                  "mi_linear_workspace_bytes")
        workspace = torch.empty(max(1, size.value), dtype=torch.uint8, device=device)
        total = torch.empty(self.K, dtype=torch.float32, device=device)
        nslots = self.P + (1 if L.scale else 0)
        dslots = torch.empty((nslots, self.K), dtype=torch.float32, device=device) \
            if compute_grads else None
        start = stop = None
        L.stamps = None
        if KERNEL_TIMER is not None:
            start, stop = KERNEL_TIMER.pair(self)
            L.stamps = KERNEL_TIMER.stamps(self)
        reduce = nat.Reduce()

        def launch(L):
            return lib.mi_linear_forward_deferred(
                ctypes.byref(L), workspace.data_ptr(), size.value, total.data_ptr(),
                nat.ptr(dslots), flags.data_ptr(), None if start is None else start.cuda_event,
                None if stop is None else stop.cuda_event, nat.stream_handle(device),
                ctypes.byref(reduce) if defer else None)
        code = launch(L)
        if L.draw.operand and code == nat.MI_EUNSUPPORTED:
            # this launch shape does not draw theta: the guide's own draw first
            self.draw.launch()
            guide.take_draw(self.draw)
            zeroed, prior_flags = L.options & nat.GROUP_FLAGS_ZEROED, L.prior.flags
            # the batch is still pending (take_rows changes nothing), so this descriptor draws
            # the rows in the launch again; reading batch.rows here would launch the rows kernel
            # AND leave them to this launch: the loader counter would advance twice
            L = self.describe(compute_grads, draw=False)
            L.options |= zeroed
            L.prior.flags = prior_flags
            code = launch(L)
        elif L.draw.operand and code == 0:
            guide.take_draw(self.draw)
            self.drew_theta = True
        if L.rows.counter:
            if code == nat.MI_EUNSUPPORTED:   # this launch shape does not draw rows: draw first
                zeroed, prior_flags = L.options & nat.GROUP_FLAGS_ZEROED, L.prior.flags
                L = self.describe(compute_grads, draw_rows=False)
                L.options |= zeroed
                L.prior.flags = prior_flags
                code = launch(L)
            elif code == 0:
                self.batch.rows_taken()
                self.drew_rows = True
        nat.check(code, "mi_linear_forward_deferred")
        self.reduce = reduce if defer and reduce.part else None
        self.workspace = workspace   # holds the deferred partials
        return total, dslots, flags

    def grads(self, dslots: Optional[torch.Tensor]) -> List[Optional[torch.Tensor]]:
        if dslots is None:
            return [None, None]
        dtheta = dslots[:self.P].t() if self.theta_grad else None
        dsigma = dslots[self.P].reshape(self.K, 1) if self.sigma_grad else None
        return [dtheta, dsigma]


class _LinearSiteFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, launcher: _LinearLauncher, holder: dict, theta, sigma):  # type: ignore
        total, dslots, flags = launcher.run(launcher.needs_grads())
        holder["flags"] = flags
        ctx.launcher, ctx.dslots = launcher, dslots
        return total

    @staticmethod
    def backward(ctx, g: torch.Tensor):  # type: ignore[override]
        launcher: _LinearLauncher = ctx.launcher
        dslots = ctx.dslots
        if dslots is None:
            return None, None, None, None
        ctx.dslots = None
        g = g.contiguous()
        # dslots[j, k] is row k of a [K, slots] view: rescale by g[k] / g0 unless equal
        nat.check(nat.lib().mi_scale_rows(dslots.data_ptr(), 1, launcher.K, launcher.K,
                                          dslots.shape[0], g.data_ptr(), launcher.g0,
                                          nat.stream_handle(g.device)), "mi_scale_rows")
        return (None, None, *launcher.grads(dslots))


def _storage(t: torch.Tensor) -> Optional[int]:
    return guide._storage_of(t)


def claim_linear_draws(trace: ParticleTrace) -> Dict[int, guide.PendingDraw]:
    """
    Deferred guide draws (:class:`guide.PendingDraw`) a linear site kernel makes itself
    (``mi_linear.draw``), by ``id`` of that site: the draw is the theta of exactly one linear site,
    and every other site tensor reading it is the [K, P] draw itself (e.g. the value of a prior
    over theta, which the linear launch evaluates too). Every other deferred draw is launched now,
    before planning reads anything.
    """
    if not guide._PENDING_DRAWS:
        return {}
    thetas: Dict[guide.PendingDraw, list] = collections.defaultdict(list)
    others: Dict[guide.PendingDraw, list] = collections.defaultdict(list)
    for site in trace.sites:
        if site.linear_X is not None and site.linear_theta is not None:
            rec = guide.pending_draw(site.linear_theta)
            if rec is not None:
                thetas[rec].append(site)
        for t in site.tensors:
            rec = guide.pending_draw(t)
            if rec is not None:
                others[rec].append(t)
    claims = {}
    # one-element draws (a global parameter's K draws, e.g. the missing-observations model's mu)
    # stay pending for claim_group_draws: a fused-draw site program may make them itself
    keep = {id(rec) for rec in guide._PENDING_DRAWS.values() if rec.z.shape[-1] == 1}
    for rec, sites in thetas.items():
        z = rec.z
        if len(sites) == 1 and all(
                isinstance(t, torch.Tensor) and t.data_ptr() == z.data_ptr() and
                tuple(t.shape) == tuple(z.shape) and tuple(t.stride()) == tuple(z.stride())
                for t in others.get(rec, [])):
            claims[id(sites[0])] = rec
            rec.claimed = True
    claimed = set(map(id, claims.values())) | keep
    for key, rec in list(guide._PENDING_DRAWS.items()):
        if id(rec) not in claimed:
            del guide._PENDING_DRAWS[key]
            rec.launch()
    return claims


def claim_group_draws(trace: ParticleTrace, launchers: List["_GroupLauncher"]) -> None:
    """
    Deferred one-element Normal guide draws (a global parameter's K draws: the missing-
    observations model's ``mu``, examples/missing-observations.md:33-45) that a fused-draw site
    program makes itself (``mi_group.pdraw``): the draw is read only by that program, as one
    per-particle operand (its sites, and a prior folded into it). The program computes the draws
    from the same counter as ``mi_normal_rsample`` into a table of its own and writes them out, so
    the draw has no launch of its own. Unclaimed draws are launched by the caller's flush.
    """
    pending = [rec for rec in guide._PENDING_DRAWS.values()
               if not rec.claimed and not rec.done and rec.z.shape[-1] == 1]
    if not pending:
        return
    lib = nat.lib()
    for rec in pending:
        key = _storage(rec.z)
        # every site reading the draw must belong to one launcher (or be its folded prior)
        readers = []
        for site in trace.sites:
            if any(isinstance(t, torch.Tensor) and guide.pending_draw(t) is rec for t in site.tensors):
                readers.append(site)
        hosts = [(l, i) for l in launchers for i, op in enumerate(l.operands)
                 if op.view.tensor is not None and _storage(op.view.tensor) == key]
        if len(hosts) != 1:
            continue
        host, index = hosts[0]
        own = {id(site) for site, _, _ in host.sites}
        if host.prior is not None:
            own.add(id(host.prior[0]))
        if host.draw is None or host.operands[index].view.si != 0 or \
                any(id(site) not in own for site in readers):
            continue
        host.pdraw = (rec, index)
        group, _ = host.describe(True, query=True)
        if host.prior is not None:
            group.prior.flags = _QUERY_ADDRESS
        supported = ctypes.c_int(0)
        nat.check(lib.mi_group_pdraw_supported(ctypes.byref(group), ctypes.byref(supported)),
                  "mi_group_pdraw_supported")
        if supported.value:
            rec.claimed = True
        else:
            host.pdraw = None


def release_unsafe_claims(linears: List["_LinearLauncher"], launchers: List["_GroupLauncher"],
                          categorical) -> None:
    """
    Launch the claimed draws that a group or categorical launch also reads (a prior over theta
    that was not folded into the linear launch): those run before the linear sites.
    """
    drawn = {_storage(l.draw.z): l for l in linears if l.draw is not None}
    if not drawn:
        return
    read = set()
    for launcher in launchers:
        for op in launcher.operands:
            if op.view.tensor is not None:
                read.add(_storage(op.view.tensor))
    for site, lg, val, _ in categorical:
        read.update(_storage(t) for t in (lg, val) if isinstance(t, torch.Tensor))
    for key in read & set(drawn):
        linear = drawn[key]
        linear.draw.launch()
        guide.take_draw(linear.draw)
        linear.draw = None


def plan_linear(trace: ParticleTrace, g0: float, device: torch.device,
                claims: Optional[Dict[int, guide.PendingDraw]] = None) -> List[_LinearLauncher]:
    """
    Launchers for the fused linear-predictor sites of a trace. A site whose operands the kernel
    cannot take (per-element sigma, particle-dependent values, non-float32) gets its predictor
    materialised here as ``theta @ X.T`` and is planned like any other site.
    """
    K = trace.K
    out: List[_LinearLauncher] = []
    for site in trace.sites:
        if site.linear_X is None:
            continue
        theta = site.linear_theta
        shape = site.site_shape
        launcher = None
        ok = theta is not None and theta.dtype == torch.float32 and theta.dim() == 2 and \
            theta.device == device and site.linear_X.device == device
        if ok:
            value_t, const = _to_device(_float(site.tensors[-1], site.name), K, device,
                                        f"site '{site.name}'", allow_constant=False)
            value = _collapse(value_t, K, shape)
            sigma = None
            if site.family == "normal":
                t, c = _to_device(_float(site.tensors[1], site.name), K, device,
                                  f"site '{site.name}'")
                sigma = _View(None, 0, 0, c) if c is not None else _collapse(t, K, shape)
                if sigma.constant is None and sigma.si != 0:
                    ok = False
            if value.sk != 0:
                ok = False
            mask = None
            if site.mask is not None:
                mask = site.mask.to(device).bool().expand(shape).reshape(-1)
            if ok:
                launcher = _LinearLauncher(site, K, g0, device, theta, sigma, value, mask)
                xb, vb = data.lookup(site.linear_X), data.lookup(value.tensor)
                if xb is not None and vb is not None and xb[0] is vb[0] and mask is None and \
                        value.si == 1:
                    batch = xb[0]
                    launcher.batch = batch
                    launcher.X_src = batch.loader.columns[xb[1]]
                    launcher.value_src = batch.loader.columns[vb[1]]
        if launcher is None:
            # materialise the predictor as the model would have: [K, N] = theta @ X^T
            guide.flush_draws(claimed=True)
            site.tensors[0] = theta @ site.linear_X.t()
            site.linear_X = None
            continue
        launcher.draw = (claims or {}).get(id(site))
        out.append(launcher)
    return out


@dataclasses.dataclass
class LogJoint:
    """
    Per-particle log joint of a trace plus the device-side validation results.
    """
    total: torch.Tensor                       # [K] fp32, differentiable
    pending: List[Tuple[str, dict, List[SiteRecord]]]
    checks: list
    flags: Optional[torch.Tensor] = None      # int32, one word per pending site, in order
    sticky: bool = False                      # flags are never zeroed by a replay (graph mode)
    mirror: Optional[torch.Tensor] = None     # host copy of `flags` the ELBO forward writes

    def flag_vector(self) -> Optional[torch.Tensor]:
        """
        All validation results of the step as one int64 device vector: one MI_FLAG_* word per
        kernel-evaluated site, then one 0/1 per deferred support / constraint check.
        """
        step = _PENDING
        if step is not None and (step.writes_flags or self.mirror is not None):
            # a held site launch finishing the ELBO writes the words, a held ELBO forward their
            # host mirror; a held ELBO forward with no mirror only reads them, and stays held for
            # the optimizer step (the validation read then waits for the site kernels alone)
            flush_pending_step()
        if self.flags is not None and not self.checks:
            return self.flags
        parts = []
        if self.flags is not None:
            parts.append(self.flags.to(torch.int64))
        else:
            for _, holder, _ in self.pending:
                parts.append(holder["flags"].reshape(-1).to(torch.int64))
        for _, ok in self.checks:
            parts.append((~ok.reshape(-1).bool()).any().reshape(1).to(torch.int64))
        if not parts:
            return None
        # host-evaluated checks (host values) join the device flags
        device = next((p.device for p in parts if p.device.type != "cpu"), parts[0].device)
        return torch.cat([p.to(device) for p in parts])

    def flag_count(self) -> int:
        return sum(len(sites) for _, _, sites in self.pending) + len(self.checks)

    def raise_from(self, values) -> None:
        """
        Raise the reference's errors (core.py:186-188 for values, torch validate_args for
        parameters) from host copies of :meth:`flag_vector`.
        """
        # every violation, then the first in model order (the reference raises at the first
        # sample statement that fails, core.py:142-189)
        found = []
        cursor = 0
        for kind, holder, sites in self.pending:
            for site in sites:
                bits = int(values[cursor])
                cursor += 1
                if bits & nat.FLAG_INTERNAL:
                    flush_pending_step()
                    raise RuntimeError(f"site '{site.name}': an in-kernel completion wait of its "
                                       "launch timed out (results of this step are invalid)")
                if bits & nat.FLAG_PARAM:
                    found.append((site.order, len(found), (
                        f"Expected parameters of distribution {site.description} for site "
                        f"'{site.name}' to satisfy their constraints, but found invalid values.")))
                elif bits & nat.FLAG_SUPPORT:
                    found.append((site.order, len(found),
                                  f"Parameter '{site.name}' is not in the support of "
                                  f"{site.description}."))
        for check, _ in self.checks:
            if int(values[cursor]):
                found.append((check.order, len(found), check.message))
            cursor += 1
        if found:
            flush_pending_step()   # the step's launches all run, as without a violation
            raise ValueError(min(found)[2])
        for check, _ in self.checks:
            if check.memo is not None:
                particles.memo_commit(check.memo)

    def raise_on_violation(self) -> None:
        """
        One host synchronisation for all validation flags of the step.
        """
        vector = self.flag_vector()
        if vector is not None:
            self.raise_from(vector.cpu().tolist())


def plan_groups(trace: ParticleTrace, g0: float, device: torch.device):
    """
    Prepare every recorded site for launch: categorical sites as (site, logits, value, mask) and
    the other families packed into site groups sharing their element space and a dense operand.
    """
    K = trace.K
    groups: List[Tuple[torch.Size, _GroupLauncher]] = []
    categorical = []
    for site in trace.sites:
        if site.linear_X is not None:
            continue   # planned by plan_linear
        if site.family == "categorical":
            logits, value = (_to_device(t, K, device, f"site '{site.name}'", False)[0]
                             for t in site.tensors)
            shape = site.site_shape
            C = logits.shape[-1]
            N = int(shape.numel())
            lg = _float(logits, site.name)
            lg = lg.reshape((K,) + (1,) * (len(shape) + 1 - (lg.dim() - 1)) + tuple(lg.shape[1:]))
            lg = lg.expand((K,) + tuple(shape) + (C,)).reshape(K, N, C).contiguous()
            if value.is_floating_point():
                # non-integer (or NaN) values are outside integer_interval(0, C - 1): -1 makes
                # the kernel flag them instead of the cast truncating them into the support
                value = torch.where(value == value.trunc(), value, torch.full_like(value, -1.0))
            val = _collapse(value.to(torch.int64), K, shape).tensor.expand(K, N)
            mask = None if site.mask is None else site.mask.to(device).bool().expand(shape) \
                .reshape(1, N).expand(K, N)
            categorical.append((site, lg, val, mask))
            continue
        shape = site.site_shape
        N = int(shape.numel())
        views = []
        for role, t in enumerate(site.tensors):
            is_value = role == len(site.tensors) - 1
            lazy = guide.lazy_of(t)
            if lazy is not None:   # exact-shape use, checked by _lazy_uses
                views.append(_View(None, N, 1, None, lazy))
                continue
            if is_value and site.family == "poisson" and not t.is_floating_point():
                t = t.to(torch.float32)   # integer counts (exact in fp32 below 2^24)
            moved, constant = _to_device(_float(t, site.name), K, device, f"site '{site.name}'",
                                         allow_constant=not is_value)
            views.append(_View(None, 0, 0, constant) if constant is not None
                         else _collapse(moved, K, shape))
        mask = None
        if site.mask is not None:
            flat_mask = site.mask.to(device).bool().expand(shape).reshape(N)
            mask = _View(flat_mask, 0, flat_mask.stride(0) if N > 1 else 1)
        placed = False
        for group_shape, launcher in groups:
            if group_shape == shape and launcher.shares_dense_operand(views) and \
                    launcher.try_add(site, views, mask):
                placed = True
                break
        if not placed:
            launcher = _GroupLauncher(K, N, g0, device)
            launcher.try_add(site, views, mask)
            groups.append((shape, launcher))
    return [launcher for _, launcher in groups], categorical


_PRIOR_FAMILIES = ("beta", "normal", "gamma")


# a non-null address for descriptors that are only queried (never dereferenced)
_QUERY_ADDRESS = 1 << 20


def fold_priors(launchers: List[_GroupLauncher]) -> List[_GroupLauncher]:
    """
    Fold one-element-per-particle prior sites into the launch of the site that reads the same
    per-particle tensor as its parameter (``mi_prior``; the README model's ``theta ~ Beta(2, 2)``
    under ``x ~ Bernoulli(theta)``, README.md:43-47): the prior's log density and its gradient are
    evaluated by that launch's particle-constant workgroups instead of a launch of their own.
    Only when the library's kernel for the host group carries it (``mi_group_prior_supported``)
    and both sites have the same scale; MININF_AMD_FOLD_PRIOR=0 disables it.
    """
    if os.environ.get("MININF_AMD_FOLD_PRIOR", "1") == "0":
        return launchers
    out = list(launchers)
    lib = nat.lib()
    for prior in launchers:
        if len(prior.sites) != 1 or prior.N != 1 or prior.draw is not None or prior.per_site:
            continue
        site, roles, mask = prior.sites[0]
        if mask is not None or site.family not in _PRIOR_FAMILIES or roles[0][0] != -1 or \
                roles[1][0] != -1 or roles[2][0] < 0:
            continue
        value = prior.operands[roles[2][0]]
        for host in out:
            # the host's site 0 reads the prior's value as its per-particle parameter: a one-site
            # BCAST launch (the README model) or a fused-draw site program (the missing-
            # observations model's mu ~ Normal(0, 1) under z ~ Normal(mu, 1)); the library decides
            if host is prior or host.prior is not None or host.per_site:
                continue
            hsite, hroles, _ = host.sites[0]
            if hroles[0][0] < 0 or hsite.scale != site.scale:
                continue
            param = host.operands[hroles[0][0]]
            if param.view.key != value.view.key or param.mode != value.mode:
                continue
            host.prior = (site, FAMILY_CODES[site.family], (roles[0][1], roles[1][1]))
            group, _ = host.describe(True, query=True)
            group.prior.flags = _QUERY_ADDRESS
            supported = ctypes.c_int(0)
            nat.check(lib.mi_group_prior_supported(ctypes.byref(group), ctypes.byref(supported)),
                      "mi_group_prior_supported")
            if not supported.value:
                host.prior = None
                continue
            out.remove(prior)
            break
    return out


def fold_linear_priors(launchers: List[_GroupLauncher],
                       linears: List["_LinearLauncher"]) -> List[_GroupLauncher]:
    """
    Fold a prior site over a linear site's theta itself (every element, constant parameters: the
    regression's ``theta ~ Normal(0, 1)``, examples/minibatch.md:45-50) into the linear launch
    (``mi_linear.prior``): the first row block's workgroups evaluate it from the theta fragment
    they already hold, so the prior has no launch of its own. MININF_AMD_FOLD_PRIOR=0 disables it.
    """
    if os.environ.get("MININF_AMD_FOLD_PRIOR", "1") == "0" or not linears:
        return launchers
    out = list(launchers)
    lib = nat.lib()
    for prior in launchers:
        if len(prior.sites) != 1 or prior.draw is not None or prior.per_site:
            continue
        site, roles, mask = prior.sites[0]
        if mask is not None or site.family not in _PRIOR_FAMILIES or roles[0][0] != -1 or \
                roles[1][0] != -1 or roles[2][0] < 0:
            continue
        value = prior.operands[roles[2][0]]
        t = value.view.tensor
        for linear in linears:
            theta = linear.theta
            if linear.prior is not None or prior.N != linear.P or t is None or \
                    t.data_ptr() != theta.data_ptr() or (value.view.sk, value.view.si) != \
                    tuple(theta.stride()) or (value.mode == nat.GRAD_DENSE) != linear.theta_grad:
                continue
            linear.prior = (site, FAMILY_CODES[site.family], (roles[0][1], roles[1][1]))
            L = linear.describe(True, query=True)
            L.prior.flags = 1 << 20   # (any non-null word: only the launch shape is queried)
            supported = ctypes.c_int(0)
            nat.check(lib.mi_linear_prior_supported(ctypes.byref(L), ctypes.byref(supported)),
                      "mi_linear_prior_supported")
            if not supported.value:
                linear.prior = None
                continue
            out.remove(prior)
            break
    return out


def log_joint(trace: ParticleTrace, g0: float, device: torch.device) -> LogJoint:
    """
    Launch the site kernels for every recorded site and return the per-particle log joint.
    """
    K = trace.K
    lazy, _ = _lazy_uses(trace)
    if lazy:   # per-particle upstream gradients need the draws themselves
        _materialize_draws(trace, lazy)
    linears = plan_linear(trace, g0, device)
    launchers, categorical = plan_groups(trace, g0, device)
    totals: List[torch.Tensor] = []
    pending: List[Tuple[str, dict, List[SiteRecord]]] = []
    for site, lg, val, mask in categorical:
        holder: dict = {}
        totals.append(_CategoricalFn.apply(site, holder, g0, lg, val, mask))
        pending.append(("categorical", holder, [site]))
    for linear in linears:
        holder = {}
        totals.append(_LinearSiteFn.apply(linear, holder, *linear.inputs()))
        pending.append(("linear", holder, linear.flag_sites))
    for launcher in launchers:
        holder = {}
        totals.append(_SiteGroupFn.apply(launcher, holder, *launcher.inputs()))
        pending.append(("group", holder, launcher.flag_sites))
    for _, value in trace.fallback:
        totals.append(value.to(device=device, dtype=torch.float32))
    if totals:
        total = totals[0]
        for extra in totals[1:]:
            total = total + extra
    else:
        total = torch.zeros(K, device=device)
    return LogJoint(total=total, pending=pending, checks=trace.checks)


# ------------------------------------------------------------------------------------------------
# Fused ELBO: site groups + entropy + the scalar reduction in one autograd node.
# ------------------------------------------------------------------------------------------------
@dataclasses.dataclass
class EntropyFactor:
    """
    A guide factor whose entropy the ELBO kernels evaluate (``mi_factor``): ``tensor`` is the
    autograd input -- Normal: the scale as [n] (stride 1, or any stride when n == 1); Beta: the
    interleaved [n, 2] concentration array; Gamma: the interleaved [n, 2] (concentration, rate). ``name`` / ``distribution`` identify the factor's
    draw in the samples (for absorbing the draw's backward).
    """
    family: int
    n: int
    tensor: torch.Tensor
    name: Optional[str] = None
    distribution: Optional[object] = None
    weight: float = 1.0   # mi_factor.weight: 1/W for a factor replicated on W data-sharded ranks


@dataclasses.dataclass(eq=False)
class _Absorbed:
    """
    A guide factor whose draw feeds only this ELBO's kernels: the ELBO backward computes the
    draw's backward, the entropy gradient and the guide transform's chain rule in one kernel and
    returns the gradients of the module's unconstrained parameters directly (``mi_factor`` with
    ``draw_kind``). ``uses``: (kind, launcher / linear index, operand index) with kind in
    "draw" (fused draw partials), "dense", "slot" (group gradients), "lin_theta", "lin_sigma".
    ``params``: per factor parameter (Normal loc, scale; Beta concentration1, concentration0) the
    unconstrained tensor and its MI_TRANSFORM, or None for a constant.
    """
    kind: int
    uses: List[Tuple[str, int, int]]
    params: List[Optional[Tuple[torch.Tensor, int]]]
    drawn: Optional[guide.Drawn] = None
    lazy: Optional[guide.LazyDraw] = None
    side_dgrad: Optional[torch.Tensor] = None   # Beta factors computed by a site launch (mi_side)
    saved: Optional[torch.Tensor] = None        # Beta: [n, 4] fp64 forward sums (mi_factor.saved)


_FACTOR_PARAMS = {nat.NORMAL: ("loc", "scale"), nat.BETA: ("concentration1", "concentration0")}


def _depends_on(tensors: Sequence[Optional[torch.Tensor]], target, limit: int = 20000) -> bool:
    """
    Whether autograd would route a gradient from any of ``tensors`` into the node ``target``.
    """
    if target is None:
        return False
    stack = [t.grad_fn for t in tensors if isinstance(t, torch.Tensor) and t.grad_fn is not None]
    seen = set()
    keep = []
    while stack:
        fn = stack.pop()
        if fn is None or id(fn) in seen:
            continue
        if fn is target:
            return True
        seen.add(id(fn))
        keep.append(fn)
        if len(seen) > limit:
            return True   # too large to prove independence
        stack.extend(next_fn for next_fn, _ in fn.next_functions)
    return False


def _absorb_factor(factor: EntropyFactor, samples: Dict[str, torch.Tensor], launchers, linears,
                   categorical, fallback) -> Optional[_Absorbed]:
    """
    The absorption plan of one guide factor, or None when its draw's backward has to stay with
    autograd (the draw reaches the loss other than through the kernels' own operands, a parameter
    does not come straight from a ParameterizedDistribution, ...).
    """
    dist = factor.distribution
    if dist is None or factor.name is None or factor.name not in samples or \
            factor.family not in _FACTOR_PARAMS:
        return None   # Gamma draws keep their own backward (mi_gamma_rsample_backward)
    sources = getattr(dist, "_mininf_amd_sources", None) or {}
    params: List[Optional[Tuple[torch.Tensor, int]]] = []
    for pname in _FACTOR_PARAMS[factor.family]:
        source = sources.get(pname)
        if source is None:
            value = getattr(dist, pname, None)
            if isinstance(value, torch.Tensor) and value.requires_grad:
                return None   # derived some other way: autograd keeps it
            params.append(None)
            continue
        u, kind = source
        if tuple(u.shape) != tuple(dist.batch_shape) or u.dtype != torch.float32 or \
                not u.is_cuda or (u.numel() > 1 and not u.is_contiguous()):
            return None
        transform = nat.TRANSFORM_EXP if kind == "exp" else nat.TRANSFORM_NONE
        params.append((u, transform) if u.requires_grad else None)
    if all(p is None for p in params):
        return None
    sample = samples[factor.name]
    uses: List[Tuple[str, int, int]] = []
    lazy = guide.lazy_of(sample)
    if lazy is not None:
        if lazy.real is not None or factor.family != nat.NORMAL:
            return None
        for li, launcher in enumerate(launchers):
            for oi, op in enumerate(launcher.operands):
                if op.view.draw is lazy:
                    if op.mode != nat.GRAD_DENSE:
                        return None
                    uses.append(("draw", li, oi))
        if len(uses) != 1:
            return None
        return _Absorbed(nat.DRAW_PARTIALS, uses, params, lazy=lazy)
    drawn = guide.drawn_of(sample)
    if drawn is None or drawn.base._version != 0:
        return None
    if (drawn.family == guide.BETA_FAMILY) != (factor.family == nat.BETA):
        return None
    z = drawn.base
    N = drawn.N
    storage = z.untyped_storage().data_ptr()

    def shares(t) -> bool:
        return isinstance(t, torch.Tensor) and t.untyped_storage().data_ptr() == storage

    others: List[Optional[torch.Tensor]] = []
    for li, launcher in enumerate(launchers):
        for oi, op in enumerate(launcher.operands):
            v = op.view
            if v.draw is not None:
                others.extend([v.draw.loc, v.draw.scale])
                continue
            if v.tensor is None:
                continue
            if not shares(v.tensor):
                others.append(v.tensor)
                continue
            if v.tensor.data_ptr() != z.data_ptr():
                return None
            if op.mode == nat.GRAD_PARTICLE and N == 1 and v.sk == z.stride(0):
                uses.append(("slot", li, oi))
            elif op.mode == nat.GRAD_DENSE and launcher.N == N and v.sk == z.stride(0) and \
                    (v.si == z.stride(1) or N == 1):
                uses.append(("dense", li, oi))
            else:
                return None
    for j, linear in enumerate(linears):
        theta, sigma = linear.inputs()
        for which, t in (("lin_theta", theta), ("lin_sigma", sigma)):
            if t is None:
                continue
            if not shares(t):
                others.append(t)
                continue
            if t.data_ptr() != z.data_ptr():
                return None
            if which == "lin_theta" and linear.theta_grad and N == linear.P and \
                    tuple(t.stride()) == tuple(z.stride()):
                uses.append((which, j, -1))
            elif which == "lin_sigma" and linear.sigma_grad and N == 1 and \
                    t.stride(0) == z.stride(0):
                uses.append((which, j, -1))
            else:
                return None
    for _, logits, _, _ in categorical:
        if shares(logits):
            return None
        others.append(logits)
    others.extend(fallback)
    if len(uses) > nat.MAX_SOURCES or _depends_on(others, z.grad_fn):
        return None
    return _Absorbed(nat.DRAW_SOURCES, uses, params, drawn=drawn)


def plan_absorption(factors: List[EntropyFactor], samples: Optional[Dict[str, torch.Tensor]],
                    launchers, linears, categorical, fallback) -> Dict[int, _Absorbed]:
    """
    Factor index -> absorption plan, for the factors whose draws' backward the ELBO kernels take
    over (``MININF_AMD_ABSORB=0`` disables it).
    """
    if not samples or not torch.is_grad_enabled() or \
            os.environ.get("MININF_AMD_ABSORB", "1") == "0":
        return {}
    out: Dict[int, _Absorbed] = {}
    for index, factor in enumerate(factors):
        plan = _absorb_factor(factor, samples, launchers, linears, categorical, fallback)
        if plan is not None:
            out[index] = plan
    return out


_ELBO_WORKSPACE: Dict[Tuple[str, int], torch.Tensor] = {}
# workspaces replaced by a larger one: a captured hipGraph may still hold their addresses, so they
# are never freed
_ELBO_RETIRED: List[torch.Tensor] = []


def _elbo_workspace(device: torch.device, nbytes: int) -> torch.Tensor:
    """
    Per-device workspace of ``mi_elbo_forward`` / ``mi_elbo_backward`` (its completion counters
    must start at zero and are left at zero by every launch, so the buffer is allocated and zeroed
    once and reused by every step, including captured graphs).
    """
    key = (device.type, device.index if device.index is not None else torch.cuda.current_device())
    ws = _ELBO_WORKSPACE.get(key)
    if ws is None or ws.numel() < nbytes:
        if ws is not None:
            _ELBO_RETIRED.append(ws)
        ws = torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8, device=device)
        nat.check(nat.lib().mi_elbo_workspace_init(ws.data_ptr(), ws.numel(),
                                                   nat.stream_handle(device)),
                  "mi_elbo_workspace_init")
        _ELBO_WORKSPACE[key] = ws
    return ws


class _ElboPlan:
    """
    Everything one ELBO evaluation launches, in the order of the autograd inputs:
    site groups (their operand tensors), categorical sites (logits, value, mask), linear sites
    (theta, sigma), torch-evaluated sites (their [K] log densities) and the entropy factors (their
    parameter tensor, or -- absorbed -- the unconstrained parameters of both parameters).
    """
    def __init__(self, K: int, g0: float, device: torch.device, launchers, categorical,
                 fallback: List[torch.Tensor], factors: List[EntropyFactor],
                 entropy_scale: float, linears: Optional[List[_LinearLauncher]] = None,
                 absorbed: Optional[Dict[int, _Absorbed]] = None,
                 zeroed_flags: Optional[torch.Tensor] = None,
                 step_words: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                 mirror: Optional[torch.Tensor] = None) -> None:
        self.K, self.g0, self.device = K, g0, device
        self.zeroed_flags = zeroed_flags
        # (counter, snapshot): the generator words the ELBO forward advances (mi_elbo.step_counter)
        self.step_words = step_words
        # host-mapped copy of the validation words written by the ELBO forward (mi_elbo.flags_mirror)
        self.mirror = mirror
        self.recompute = False
        self.launchers = launchers
        self.categorical = categorical
        self.linears = linears or []
        self.lin_holders = [dict() for _ in self.linears]
        self.fallback = [v.to(device=device, dtype=torch.float32).reshape(K) for v in fallback]
        self.factors = factors
        self.entropy_scale = entropy_scale
        self.holders = [dict() for _ in launchers]
        self.cat_holders = [dict() for _ in categorical]
        self.flags: Optional[torch.Tensor] = None
        self.state = None
        self.tensor_inputs: Optional[List[bool]] = None
        self.deferred_count = 0
        self.absorbed = absorbed or {}
        # operands / linear inputs whose gradient an absorbed factor consumes
        self.skip_ops: Dict[int, set] = collections.defaultdict(set)
        self.skip_lin: set = set()
        for plan in self.absorbed.values():
            for kind, index, operand in plan.uses:
                if kind in ("draw", "dense", "slot"):
                    self.skip_ops[index].add(operand)
                    if kind == "draw":
                        launchers[index].draw_partials = True
                else:
                    self.skip_lin.add((kind, index))

    def inputs(self) -> List[Optional[torch.Tensor]]:
        out: List[Optional[torch.Tensor]] = []
        for li, launcher in enumerate(self.launchers):
            out.extend(launcher.inputs(self.skip_ops.get(li, ())))
        for _, lg, val, mask in self.categorical:
            out.extend([lg, val, mask])
        for j, linear in enumerate(self.linears):
            theta, sigma = linear.inputs()
            out.append(None if ("lin_theta", j) in self.skip_lin else theta)
            out.append(None if ("lin_sigma", j) in self.skip_lin else sigma)
        out.extend(self.fallback)
        for index, f in enumerate(self.factors):
            plan = self.absorbed.get(index)
            if plan is None:
                out.append(f.tensor)
            else:
                out.extend(p[0] if p is not None else None for p in plan.params)
        return out

    def _describe(self, terms: List[torch.Tensor], buffers: List[torch.Tensor],
                  fill: bool = True) -> nat.Elbo:
        E = nat.Elbo()
        E.K = self.K
        E.g0 = self.g0
        E.entropy_scale = self.entropy_scale
        E.num_terms = len(terms)
        for j, t in enumerate(terms):
            E.terms[j] = t.data_ptr()
        E.num_factors = len(self.factors)
        for j, f in enumerate(self.factors):
            d = E.factors[j]
            d.family, d.n = f.family, f.n
            d.weight = f.weight
            # the entropy kernels read the parameters directly: a deferred exp transform no draw
            # kernel has written yet runs first (a no-op once a draw kernel wrote it; `fill`
            # False: the launch being described writes it)
            if fill:
                guide.fill_exp(f.tensor)
            base = f.tensor.data_ptr()
            if f.family in (nat.BETA, nat.GAMMA):
                d.param[0], d.param[1] = base, base + 4
                d.stride[0] = d.stride[1] = 2
            else:
                d.param[1] = base
                d.stride[1] = f.tensor.stride(0) if f.n > 1 else 0
        E.num_buffers = len(buffers)
        for j, b in enumerate(buffers):
            E.buffers[j] = b.data_ptr()
            E.buffer_len[j] = b.numel()
        return E

    def _describe_absorbed(self, E: nat.Elbo, results, lin_results) -> None:
        """Fill the absorbed draws' fields of the factor descriptors (after the site launches)."""
        for index, plan in self.absorbed.items():
            d = E.factors[index]
            f = self.factors[index]
            d.draw_kind = plan.kind
            for j, p in enumerate(plan.params):
                if p is not None:
                    d.transform[j] = p[1]
            if f.family == nat.NORMAL:
                loc = f.distribution.loc.reshape(f.n)
                if f.n > 1 and loc.stride(0) != 1:
                    loc = loc.contiguous()
                plan.loc = loc   # kept alive with the plan
                d.param[0] = loc.data_ptr()
                d.stride[0] = loc.stride(0) if f.n > 1 else 0
            if plan.kind == nat.DRAW_PARTIALS:
                _, li, _ = plan.uses[0]
                ptr, rows = self.launchers[li].partials
                d.partial[0], d.partial[1] = ptr, ptr + 4 * rows * f.n
                d.partial_rows = rows
                continue
            cfg = plan.drawn.cfg
            if f.family == nat.BETA:
                # the forward's per-element sums for this evaluation's backward, owned by the
                # plan so that interleaved evaluations never share them
                plan.saved = torch.empty(4 * f.n, dtype=torch.float64, device=self.device)
                d.saved = plan.saved.data_ptr()
                d.draws = plan.drawn.base.data_ptr()
                d.dgrad = nat.ptr(plan.side_dgrad if plan.side_dgrad is not None
                                  else plan.drawn.dgrad)
            else:
                d.eps = nat.ptr(cfg.noise)
                d.seed, d.step = guide._philox_key(cfg)
                d.step_device = nat.ptr(guide.backward_step(cfg))   # read by the ELBO backward
                d.stream_id = cfg.stream_id
                d.particle_offset = cfg.particle_offset
                d.element_offset = cfg.element_offset
            d.num_sources = len(plan.uses)
            for s, (kind, li, oi) in enumerate(plan.uses):
                src = d.source[s]
                if kind == "dense":
                    grad = results[li][0][oi]
                    src.ptr = grad.data_ptr()
                    src.stride_k, src.stride_i = grad.stride()
                elif kind == "slot":
                    slot_grad = results[li][1]
                    src.ptr = slot_grad[self.launchers[li].operands[oi].slot].data_ptr()
                    src.stride_k, src.stride_i = 1, 0
                elif kind == "lin_theta":
                    src.ptr = lin_results[li].data_ptr()
                    src.stride_k, src.stride_i = 1, self.K
                else:   # lin_sigma
                    src.ptr = lin_results[li][self.linears[li].P].data_ptr()
                    src.stride_k, src.stride_i = 1, 0

    def forward(self) -> torch.Tensor:
        terms: List[torch.Tensor] = []
        buffers: List[torch.Tensor] = []
        results = []
        deferred: List[Tuple[nat.Reduce, torch.Tensor]] = []   # finalize reductions left to us
        # one zeroed flag buffer for every site of the step, in `pending` order (categorical first)
        sizes = [1] * len(self.categorical) + [len(l.flag_sites) for l in self.linears] + \
            [len(l.flag_sites) for l in self.launchers]
        words = max(1, sum(sizes))
        zeroed, self.zeroed_flags = self.zeroed_flags, None   # zero only for the first forward
        if zeroed is not None and zeroed.numel() >= words:
            self.flags = zeroed[:words]
        else:
            self.flags = torch.zeros(words, dtype=torch.int32, device=self.device)
        cursor = len(self.categorical) + sum(len(l.flag_sites) for l in self.linears)
        # absorbed Beta draws whose implicit-gradient factors a site launch can carry (mi_side)
        side_jobs = [plan for plan in self.absorbed.values()
                     if plan.drawn is not None and plan.drawn.family == guide.BETA_FAMILY and
                     plan.drawn.dgrad is None and plan.drawn.conc is not None and
                     plan.drawn.base.numel() <= guide.BETA_DGRAD_MAX and
                     os.environ.get("MININF_AMD_BETA_SIDE", "1") != "0"]
        for plan in side_jobs:
            plan.side_dgrad = None
        for li, (launcher, holder) in enumerate(zip(self.launchers, self.holders)):
            need = any(op.mode != nat.GRAD_NONE for op in launcher.operands)
            job = side_jobs[0] if side_jobs else None
            launcher.side = None if job is None else (
                job.drawn.base.reshape(self.K, job.drawn.N), job.drawn.conc)
            part = self.flags[cursor:cursor + len(launcher.flag_sites)]
            cursor += len(launcher.flag_sites)
            total, site_lp, grads, slot_grad, flags = launcher.run(need, part, defer=True)
            if launcher.reduce is not None:
                deferred.append((launcher.reduce, total))
            if job is not None and launcher.side_out is not None:
                job.side_dgrad = launcher.side_out
                side_jobs.pop(0)
            launcher.side = None
            holder["flags"], holder["site_lp"] = flags, site_lp
            terms.append(total)
            skip = self.skip_ops.get(li, set())
            if need:
                # speculative buffers the backward rescales when the upstream is not 1 (those an
                # absorbed factor consumes are scaled inside its own reduction instead)
                for oi, g in enumerate(grads):
                    if oi in skip:
                        continue
                    if isinstance(g, tuple):
                        buffers.extend(g)
                    elif g is not None:
                        buffers.append(g)
                if launcher.num_slots:
                    absorbed_slots = {launcher.operands[oi].slot for oi in skip
                                      if launcher.operands[oi].mode == nat.GRAD_PARTICLE}
                    if absorbed_slots:
                        buffers.extend(slot_grad[j:j + 1] for j in range(launcher.num_slots)
                                       if j not in absorbed_slots)
                    else:
                        buffers.append(slot_grad[:launcher.num_slots])
            results.append((grads, slot_grad, launcher.workspace))
        cat_results = []
        for j, ((site, lg, val, mask), holder) in enumerate(zip(self.categorical,
                                                                 self.cat_holders)):
            total, dlogits, flags = _run_categorical(site, self.g0, lg, val, mask,
                                                     lg.requires_grad, self.flags[j:j + 1])
            holder["flags"] = flags
            terms.append(total)
            if dlogits is not None:
                buffers.append(dlogits)
            cat_results.append(dlogits)
        lin_results = []
        base = len(self.categorical)
        for j, (linear, holder) in enumerate(zip(self.linears, self.lin_holders)):
            words = len(linear.flag_sites)
            total, dslots, flags = linear.run(linear.needs_grads(),
                                              self.flags[base:base + words], defer=True)
            base += words
            if linear.reduce is not None:
                deferred.append((linear.reduce, total))
            holder["flags"] = flags
            terms.append(total)
            if dslots is not None:
                theta_out = ("lin_theta", j) in self.skip_lin
                sigma_out = ("lin_sigma", j) in self.skip_lin
                if not theta_out and not sigma_out:
                    buffers.append(dslots)
                else:
                    if not theta_out:
                        buffers.append(dslots[:linear.P])
                    if not sigma_out and dslots.shape[0] > linear.P:
                        buffers.append(dslots[linear.P:])
            lin_results.append(dslots)
        terms.extend(t.contiguous() for t in self.fallback)
        # The deferred reductions run inside the ELBO forward (their totals then leave `terms`)
        # unless there are too many, or a forward-absorbed Beta factor lacks its precomputed
        # implicit-gradient factors (mi_elbo.reduce); otherwise each runs as its own launch.
        fused = self._reduce_ok() and len(deferred) <= nat.MAX_REDUCE and \
            os.environ.get("MININF_AMD_FUSE_REDUCE", "1") != "0"
        lib = nat.lib()
        self.deferred_count = len(deferred) if fused else 0
        if fused:
            reduced = {id(t) for _, t in deferred}
            terms = [t for t in terms if id(t) not in reduced]
        else:
            stream = nat.stream_handle(self.device)
            for job, _ in deferred:
                nat.check(lib.mi_reduce_launch(ctypes.byref(job), stream), "mi_reduce_launch")
            deferred = []
        if len(terms) > nat.MAX_TERMS:
            head = nat.MAX_TERMS - 1
            terms = terms[:head] + [torch.stack(terms[head:]).sum(0)]
        extra = buffers[nat.MAX_BUFFERS:]
        buffers = buffers[:nat.MAX_BUFFERS]
        E = self._describe(terms, buffers)
        self._describe_absorbed(E, results, lin_results)
        E.num_reduce = len(deferred)
        for j, (job, _) in enumerate(deferred):
            E.reduce[j] = job
        if self.step_words is not None and not self.recompute:
            E.step_counter = self.step_words[0].data_ptr()
            E.step_snapshot = self.step_words[1].data_ptr()
        if self.mirror is not None:
            E.flags = self.flags.data_ptr()
            E.flags_mirror = self.mirror.data_ptr()
            E.nflags = min(self.flags.numel(), self.mirror.numel())
        # The guide gradients of an upstream of exactly 1 (loss.backward() through nn._Loss's unit
        # seed) written by the forward when that leaves the backward nothing to do: the backward
        # then returns them without a launch (MI_ELBO_FINAL_GRADS).
        self.final = None
        if not self.recompute and not self.fallback and not extra and \
                os.environ.get("MININF_AMD_FINAL_GRADS", "1") != "0":
            complete = ctypes.c_int(0)
            nat.check(lib.mi_elbo_final_grads(ctypes.byref(E), ctypes.byref(complete)),
                      "mi_elbo_final_grads")
            if complete.value:
                self.final = self._factor_grads(E)
                E.options |= nat.ELBO_FINAL_GRADS
        size = ctypes.c_size_t()
        nat.check(lib.mi_elbo_workspace_bytes(ctypes.byref(E), ctypes.byref(size)),
                  "mi_elbo_workspace_bytes")
        ws = _elbo_workspace(self.device, size.value)
        loss = torch.empty((), dtype=torch.float32, device=self.device)
        guide.join_side()   # Beta implicit-gradient factors (mi_beta_dgrad) from the side stream
        stream = nat.stream_handle(self.device)

        def launch(adam):
            if adam is None:
                return lib.mi_elbo_forward(ctypes.byref(E), ws.data_ptr(), ws.numel(),
                                           loss.data_ptr(), stream)
            return lib.mi_elbo_forward_adam(ctypes.byref(E), ws.data_ptr(), ws.numel(),
                                            loss.data_ptr(), adam, stream)
        self.state = (E, results, cat_results, lin_results, extra, terms)
        # with the final gradients written, the launch is held for the optimizer step, which
        # then runs in its last block (mi_elbo_forward_adam). Everything E points to stays alive
        # until it runs: the backward drops self.state, and the deferred reductions' outputs
        # (written by this launch) are referenced nowhere else -- freed early, their memory would
        # be handed to the allocations made before the launch (the optimizer's own descriptor).
        keep = (self, E, ws, loss, self.state, self.final, deferred, buffers)
        if self.final is None or not _defer_step(launch, "mi_elbo_forward", self.final, keep,
                                                 self._elbo_adam(E), stream=(self.device, stream)):
            nat.check(launch(None), "mi_elbo_forward")
        return loss

    def _elbo_adam(self, E):
        """The adapter of the held ELBO forward: an mi_adam descriptor whose every tensor's
        gradient is one of the final gradients this launch writes -> the device pointer of the
        matching mi_elbo_adam (None: declined)."""
        final = self.final
        device = self.device

        def adapt(adam):
            if adam.num > nat.ELBO_ADAM_SLOTS:
                return None
            where = {}
            for f, grads in enumerate(final):
                if f not in self.absorbed:
                    continue
                for j, g in enumerate(grads):
                    if g is not None:
                        where[g.data_ptr()] = (f, j, g.numel())
            desc = nat.ElboAdam()
            desc.num, desc.maximize = adam.num, adam.maximize
            desc.lr, desc.beta1, desc.beta2 = adam.lr, adam.beta1, adam.beta2
            desc.eps, desc.weight_decay = adam.eps, adam.weight_decay
            for t in range(adam.num):
                T = adam.tensors[t]
                hit = where.get(T.grad)
                if hit is None or hit[2] != T.numel:
                    return None
                slot = desc.slots[t]
                slot.factor, slot.param = hit[0], hit[1]
                slot.value, slot.exp_avg, slot.exp_avg_sq = T.param, T.exp_avg, T.exp_avg_sq
                slot.step, slot.numel = T.step, T.numel
            ok = ctypes.c_int(0)
            nat.check(nat.lib().mi_elbo_adam_supported(ctypes.byref(E), ctypes.byref(desc),
                                                       ctypes.byref(ok)), "mi_elbo_adam_supported")
            return _elbo_adam_device(desc, device) if ok.value else None
        return adapt

    def fusions(self) -> Dict[str, int]:
        """
        Which fast paths this evaluation took (structural patterns the planner recognised; a model
        slightly off a pattern takes the general path, and this says so):
        folded_priors: prior sites evaluated by the launch of the site that reads their value
        (mi_prior); linear_theta_draws / linear_rows: linear launches that drew the guide's theta
        (mi_linear.draw) / their minibatch rows (mi_rows) themselves; fused_draws: Normal guide
        factors drawn in registers by the site programs (mi_draw); program_draws: one-element
        Normal guide factors drawn per particle by the site program that reads them (mi_group.pdraw,
        no draw launch); deferred_reductions: site
        reductions finished by the ELBO forward; final_grads: the forward wrote the guide
        gradients (no backward launch for loss.backward()); optimizer_step: the Adam step ran in the held launch's last block (no launch of its own).
        """
        return {
            "folded_priors": sum(l.prior is not None for l in self.launchers) +
            sum(l.prior is not None for l in self.linears),
            "linear_theta_draws": sum(l.drew_theta for l in self.linears),
            "linear_rows": sum(l.drew_rows for l in self.linears),
            "fused_draws": sum(p.kind == nat.DRAW_PARTIALS for p in self.absorbed.values()),
            "program_draws": sum(l.made_pdraw for l in self.launchers),
            "deferred_reductions": self.deferred_count,
            "final_grads": int(getattr(self, "final", None) is not None),
            "optimizer_step": 0,   # set when the optimizer step joins the held launch
        }

    def _reduce_ok(self) -> bool:
        """
        Whether the deferred reductions can join the ELBO forward: every forward-absorbed Beta
        factor has its implicit-gradient factors precomputed (its particle sums then move to the
        ELBO backward).
        """
        for index, plan in self.absorbed.items():
            f = self.factors[index]
            if f.family != nat.BETA or plan.kind == nat.DRAW_PARTIALS:
                continue
            dgrad = plan.side_dgrad if plan.side_dgrad is not None else plan.drawn.dgrad
            if dgrad is None:
                return False
        return True

    def backward(self, u: torch.Tensor, hold: bool = False) -> List[Optional[torch.Tensor]]:
        if self.state is None:   # a second backward through the same graph: recompute
            # with this evaluation's generator step (the snapshot) and without advancing it again
            self.recompute = True
            for launcher in self.launchers:
                if launcher.draw is not None:
                    guide.use_snapshot(launcher.draw.cfg)
            self.forward()
        E, results, cat_results, lin_results, extra, _ = self.state
        self.state = None
        final, self.final = getattr(self, "final", None), None
        if final is not None and _is_unit_seed(u):
            # the forward wrote the gradients of exactly this upstream (MI_ELBO_FINAL_GRADS);
            # autograd reads them next (nn._accumulate_final_grads may hold them instead)
            if not hold:
                flush_pending_step()
            return self._outputs(results, cat_results, lin_results, None, final)
        device = self.device
        u = u.to(torch.float32).contiguous()
        dterm = torch.empty(1, dtype=torch.float32, device=device)
        fgrads = self._factor_grads(E)
        size = ctypes.c_size_t()
        lib = nat.lib()
        nat.check(lib.mi_elbo_workspace_bytes(ctypes.byref(E), ctypes.byref(size)),
                  "mi_elbo_workspace_bytes")
        ws = _elbo_workspace(device, size.value)
        nat.check(lib.mi_elbo_backward(ctypes.byref(E), u.data_ptr(), dterm.data_ptr(),
                                       ws.data_ptr(), ws.numel(), nat.stream_handle(device)),
                  "mi_elbo_backward")
        for buffer in extra:
            buffer.mul_(u)
        return self._outputs(results, cat_results, lin_results, dterm, fgrads)

    def _factor_grads(self, E) -> List[List[Optional[torch.Tensor]]]:
        """The guide factors' gradient outputs, their addresses written into E's factors."""
        device = self.device
        fgrads: List[List[Optional[torch.Tensor]]] = []
        for j, f in enumerate(self.factors):
            d = E.factors[j]
            plan = self.absorbed.get(j)
            if plan is not None:
                out_j: List[Optional[torch.Tensor]] = []
                for q, p in enumerate(plan.params):
                    if p is None:
                        d.grad[q] = None
                        out_j.append(None)
                        continue
                    grad = torch.empty(p[0].shape, dtype=torch.float32, device=device)
                    d.grad[q] = grad.data_ptr()
                    d.grad_stride[q] = 1
                    out_j.append(grad)
                fgrads.append(out_j)
                continue
            grad = torch.empty_like(f.tensor)
            base = grad.data_ptr()
            if f.family in (nat.BETA, nat.GAMMA):
                d.grad[0], d.grad[1] = base, base + 4
                d.grad_stride[0] = d.grad_stride[1] = 2
            else:
                d.grad[1] = base
                d.grad_stride[1] = grad.stride(0) if f.n > 1 else 1
            fgrads.append([grad])
        return fgrads

    def _outputs(self, results, cat_results, lin_results, dterm, fgrads
                 ) -> List[Optional[torch.Tensor]]:
        """The backward's gradients in the order of the autograd node's inputs."""
        out: List[Optional[torch.Tensor]] = []
        for li, (launcher, (grads, slot_grad, _)) in enumerate(zip(self.launchers, results)):
            skip = self.skip_ops.get(li, ())
            for oi, (op, grad) in enumerate(zip(launcher.operands, grads)):
                if op.view.draw is not None:
                    out.extend((None, None) if oi in skip or grad is None else grad)
                elif oi in skip:
                    out.append(None)
                elif op.mode == nat.GRAD_DENSE:
                    out.append(grad)
                elif op.mode == nat.GRAD_PARTICLE:
                    out.append(slot_grad[op.slot].reshape(launcher.K, 1))
                else:
                    out.append(None)
        for dlogits in cat_results:
            out.extend([dlogits, None, None])
        for j, (linear, dslots) in enumerate(zip(self.linears, lin_results)):
            dtheta, dsigma = linear.grads(dslots)
            out.append(None if ("lin_theta", j) in self.skip_lin else dtheta)
            out.append(None if ("lin_sigma", j) in self.skip_lin else dsigma)
        out.extend(dterm.expand(self.K) for _ in self.fallback)
        for grads_j in fgrads:
            out.extend(grads_j)
        return out


def _is_unit_seed(u: torch.Tensor) -> bool:
    """Whether the upstream gradient is nn._Loss's cached device 1.0 (never written)."""
    from .nn import _UNIT
    seed = _UNIT.get(u.device)
    return seed is not None and u.dtype == torch.float32 and u.numel() == 1 and \
        u.data_ptr() == seed.data_ptr()


# ---- the step-finishing launch held for the optimizer --------------------------------------------
# The ELBO forward that writes the final guide gradients of loss.backward() itself (mi_elbo_forward
# with MI_ELBO_FINAL_GRADS) is the step's last kernel before the optimizer's. The launch is therefore
# held (not enqueued) until its first consumer: when that is the Adam step over its gradients
# (mininf_amd.optim.Adam), the launch runs the update in its last block (mi_elbo_forward_adam) and
# the optimizer has no launch of its own. Any other consumer enqueues it first, as it would have been:
# every native launch (_native.stream_handle), every torch operation on the loss (nn._Loss) or on
# a held gradient (PendingGrad) other than metadata queries, the validation read, graph capture
# boundaries (graph.StepGraph) and the distributed gradient reductions. MININF_AMD_DEFER_STEP=0
# launches at once.

_PENDING: Optional["_PendingStep"] = None

# queries that read no tensor data (they run before the launch without flushing it)
_NO_FLUSH = frozenset({
    torch.Tensor.dim, torch.Tensor.size, torch.Tensor.numel, torch.Tensor.nelement,
    torch.Tensor.is_contiguous, torch.Tensor.stride,
    torch.Tensor.storage_offset, torch.Tensor.element_size, torch.Tensor.is_floating_point,
    torch.Tensor.is_complex, torch.Tensor.get_device, torch.Tensor.ndimension,
    torch.Tensor.requires_grad_})
# tensor-valued properties (everything else read through a property is metadata)
_DATA_PROPERTIES = frozenset({"data", "T", "mT", "H", "mH", "real", "imag", "grad", "_base"})
# properties that hand the device address to another library (CuPy, numba, ...), which then reads
# the data on its own: the launch that writes it must be enqueued first
_RAW_POINTER_PROPERTIES = tuple(p for p in (torch.Tensor.__dict__.get("__cuda_array_interface__"),)
                                if p is not None)


def _called_from_package() -> bool:
    """Whether the Python code asking (the first frame outside this module's flush machinery) is
    mininf_amd's own: the package reads gradient addresses to describe launches that the stream
    orders after the held one, so those reads need no flush."""
    frame = sys._getframe(1)
    while frame is not None and frame.f_globals.get("__name__") == __name__:
        frame = frame.f_back
    name = frame.f_globals.get("__name__", "") if frame is not None else ""
    return name == "mininf_amd" or name.startswith("mininf_amd.")


def _flushes(func) -> bool:
    if func is torch.Tensor.data_ptr:
        # a raw address read by user code (ctypes, a DDP-like hook, another kernel library) is a
        # data use the stream does not see; the package's own descriptor reads are not
        return not _called_from_package()
    if func in _NO_FLUSH:
        return False
    if getattr(func, "__name__", None) == "__get__":
        owner = getattr(func, "__self__", None)
        if any(owner is p for p in _RAW_POINTER_PROPERTIES):
            return True
        return getattr(owner, "__name__", None) in _DATA_PROPERTIES
    return True


def torch_function_flush(func, types, args, kwargs):
    """__torch_function__ of the tensors a held launch writes: flush, then the plain operation."""
    if _PENDING is not None and _flushes(func):
        flush_pending_step()
    return torch._C._disabled_torch_function_impl(func, types, args,
                                                 {} if kwargs is None else kwargs)


class PendingGrad(torch.Tensor):
    """
    A guide gradient (``param.grad``) that the held finishing launch writes: an ordinary tensor
    whose first data use enqueues the launch. Plain ``torch.Tensor`` again once it has run.
    """
    __torch_function__ = classmethod(lambda cls, func, types, args=(), kwargs=None:
                                     torch_function_flush(func, types, args, kwargs))


def grad_meta(g: torch.Tensor):
    """(address, dtype, device, contiguous) of a gradient: a PendingGrad's recorded values (no
    flush hook), any other tensor's own."""
    meta = g.__dict__.get("_mi_meta") if type(g) is PendingGrad else None
    return meta if meta is not None else (g.data_ptr(), g.dtype, g.device, g.is_contiguous())


def _current_stream(device: torch.device) -> int:
    index = getattr(device, "index", None)
    if index is None:
        return torch.cuda.current_stream(device).cuda_stream
    return torch._C._cuda_getCurrentRawStream(index)   # (no torch.cuda.Stream object)


class _PendingStep:
    def __init__(self, launch, what: str, grads: List[torch.Tensor], keep, adapter,
                 stream=None) -> None:
        self._launch = launch        # launch(optimizer argument or None) -> error code
        self.what = what
        # the site launches that finish the ELBO write the step's validation words themselves;
        # the ELBO forward (mi_elbo_forward) only mirrors them
        self.writes_flags = what != "mi_elbo_forward"
        self.grad_ptrs = {g.data_ptr() for g in grads if g is not None}
        self.held: List[Tuple[torch.Tensor, torch.Tensor]] = []   # (param, PendingGrad)
        self._keep = keep            # the launch's buffers, alive until it has run
        self.adapt = adapter         # adapter(mi_adam descriptor) -> launch argument, or None
        # (device, hipStream_t) the launch is enqueued on: the stream current at the forward
        self.stream = stream

    def other_stream(self) -> bool:
        """Whether the stream current now is not the one the launch goes to (a consumer inside
        ``torch.cuda.stream(side)``)."""
        return self.stream is not None and _current_stream(self.stream[0]) != self.stream[1]

    def hold(self, var: torch.Tensor, grad: torch.Tensor) -> torch.Tensor:
        """``grad`` as the PendingGrad to assign to ``var.grad``. Its address and layout ride along
        as plain attributes (``_mi_meta``: address, dtype, device, contiguous), so the package's
        own checks (the optimizer's plan, the launch descriptors) read them without a torch call
        -- each torch call on a PendingGrad goes through its flush hook."""
        held = grad.as_subclass(PendingGrad)
        held._mi_meta = (grad.data_ptr(), grad.dtype, grad.device, grad.is_contiguous())
        self.held.append((var, held))
        return held

    def run(self, adam=None) -> None:
        code = self._launch(adam)
        if code == 0 and self.other_stream():
            # the consumer's stream waits for the launch (a wait_stream recorded before this flush
            # could not have seen it)
            device, handle = self.stream
            done = torch.cuda.Event()
            done.record(torch.cuda.ExternalStream(handle, device=device))
            torch.cuda.current_stream(device).wait_event(done)
        self._keep = None
        for var, held in self.held:   # the gradients are ordinary tensors from here on
            if var.grad is held:
                var.grad = held.as_subclass(torch.Tensor)
        self.held = []
        nat.check(code, self.what)


def flush_pending_step() -> None:
    """Enqueue the held finishing launch, if any (without an optimizer step)."""
    global _PENDING
    step = _PENDING
    if step is not None:
        _PENDING = None
        step.run(None)


def discard_pending_step() -> None:
    """Drop the held finishing launch unlaunched (a capture that failed part-way)."""
    global _PENDING
    _PENDING = None


def pending_step() -> Optional[_PendingStep]:
    return _PENDING


def attach_optimizer(adam, grads: Sequence[torch.Tensor]) -> bool:
    """
    Run the held finishing launch with the optimizer step ``adam`` (an ``mi_adam`` descriptor over
    ``grads``) in its last block, when the launch writes at least one of those gradients and the
    step is small enough (<= 16384 elements, csrc/adam_math.hpp kFusedAdamMaxNumel); the other
    gradients are complete already (earlier launches on the stream). False: nothing done.
    """
    global _PENDING, LAST_FUSIONS
    step = _PENDING
    if step is None or adam.num < 1 or \
            not any(grad_meta(g)[0] in step.grad_ptrs for g in grads):
        return False
    if step.other_stream():
        # an optimizer stepping on another stream than the forward's: the launch runs first (the
        # current stream waits for it), the step on its own
        flush_pending_step()
        return False
    arg = step.adapt(adam)
    if arg is None:
        return False
    _PENDING = None
    step.run(arg)
    LAST_FUSIONS["optimizer_step"] = 1
    return True


_FUSED_ADAM_MAX_NUMEL = 16384


def _small_adam(adam):
    """The finishing launches take the mi_adam descriptor itself (csrc/adam_math.hpp's limit)."""
    numel = sum(adam.tensors[j].numel for j in range(adam.num))
    return adam if numel <= _FUSED_ADAM_MAX_NUMEL else None


def _defer_step(launch, what: str, grads, keep, adapter=_small_adam, stream=None) -> bool:
    """Hold ``launch`` for the optimizer (True), or False: the caller launches now. ``stream``:
    (device, hipStream_t) the launch goes to, for consumers on other streams."""
    global _PENDING
    if os.environ.get("MININF_AMD_DEFER_STEP", "1") == "0":
        return False
    flush_pending_step()
    _PENDING = _PendingStep(launch, what, [g for gs in grads for g in gs if g is not None], keep,
                            adapter, stream)
    return True


# device copies of mi_elbo_adam descriptors (a captured step reads its copy on every replay, so
# copies are never freed; a process has a handful -- one per optimizer and model structure)
_ELBO_ADAM_COPIES: Dict[Tuple[int, bytes], torch.Tensor] = {}
_ELBO_ADAM_MAX_COPIES = 256


def _elbo_adam_device(desc, device: torch.device) -> Optional[int]:
    raw = bytes(desc)
    key = (device.index if device.index is not None else torch.cuda.current_device(), raw)
    buf = _ELBO_ADAM_COPIES.get(key)
    if buf is None:
        if len(_ELBO_ADAM_COPIES) >= _ELBO_ADAM_MAX_COPIES or \
                torch.cuda.is_current_stream_capturing():
            return None   # (no host-to-device copy inside a capture)
        buf = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)
        _ELBO_ADAM_COPIES[key] = buf
    return buf.data_ptr()


nat.set_launch_hook(flush_pending_step)


class _ElboFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, plan: _ElboPlan, *inputs):  # type: ignore[override]
        ctx.plan = plan
        return plan.forward()

    @staticmethod
    def backward(ctx, u: torch.Tensor):  # type: ignore[override]
        return (None, *ctx.plan.backward(u))


def _materialize_draws(trace: ParticleTrace, draws) -> None:
    """
    Replace the placeholders of the given lazy draws in the trace's site tensors by the real
    draws (mi_normal_rsample), broadcast like the placeholders were.
    """
    for site in trace.sites:
        site.tensors = [t if guide.lazy_of(t) not in draws else
                        guide.lazy_of(t).materialize().expand(t.shape) for t in site.tensors]


def _lazy_uses(trace: ParticleTrace) -> Tuple[set, set]:
    """
    (all lazy draws in the trace's site tensors, those used where the kernels cannot compute
    them: linear / categorical sites, or broadcast beyond the draw's own shape).
    """
    seen, bad = set(), set()
    for site in trace.sites:
        for t in site.tensors:
            lazy = guide.lazy_of(t)
            if lazy is None:
                continue
            seen.add(lazy)
            if site.linear_X is not None or site.family == "categorical" or \
                    tuple(t.shape[1:]) != tuple(site.site_shape) or \
                    int(site.site_shape.numel()) != lazy.N:
                bad.add(lazy)
    return seen, bad


def entropy_factors(approximation) -> Tuple[List[EntropyFactor], list]:
    """
    Split a factorised guide into factors whose entropy the ELBO kernels evaluate (Normal, Beta,
    Gamma) and the rest (whose entropy torch.distributions evaluates).
    """
    from torch.distributions import Beta, Gamma, Normal

    from . import guide
    fused: List[EntropyFactor] = []
    rest = []
    for name, factor in approximation.items():
        cls = type(factor)
        n = max(1, int(factor.batch_shape.numel()))
        if len(fused) < nat.MAX_FACTORS and cls is Normal and factor.scale.dtype == torch.float32 \
                and factor.scale.is_cuda and factor.scale.numel() == n:
            scale = factor.scale.reshape(n)
            if n > 1 and scale.stride(0) != 1:
                scale = scale.contiguous()
            fused.append(EntropyFactor(nat.NORMAL, n, scale, name, factor))
        elif len(fused) < nat.MAX_FACTORS and cls is Gamma and factor.concentration.is_cuda and \
                factor.concentration.dtype == torch.float32:
            # interleaved [n, 2] (concentration, rate), the Beta layout (one stack kernel)
            pair = torch.stack(torch.broadcast_tensors(factor.concentration, factor.rate), -1)
            fused.append(EntropyFactor(nat.GAMMA, n, pair.reshape(n, 2).contiguous(), name, factor))
        elif len(fused) < nat.MAX_FACTORS and cls is Beta:
            conc = guide.beta_concentration(factor, n)
            if conc.is_cuda:
                fused.append(EntropyFactor(nat.BETA, n, conc, name, factor))
            else:
                rest.append(factor)
        else:
            rest.append(factor)
    return fused, rest


# _ElboPlan.fusions() of the last ELBO evaluation (EvidenceLowerBoundLoss.last_fusions)
LAST_FUSIONS: Dict[str, int] = {}


def elbo(trace: ParticleTrace, g0: float, device: torch.device, factors: List[EntropyFactor],
         entropy_scale: float, samples: Optional[Dict[str, torch.Tensor]] = None,
         flags: Optional[torch.Tensor] = None,
         step_words: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
         mirror: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, LogJoint]:
    """
    ``g0 * sum_k log p(x, z_k) - entropy_scale * H[factors]`` as one autograd node: the site
    kernels, the entropy and the reduction run in ``mi_group_forward`` / ``mi_elbo_forward``;
    backward is one ``mi_elbo_backward`` launch (plus the guide samplers' own backward).
    ``flags``: already-zeroed int32 validation words for the step, used when the plan's sites fit.
    ``step_words``: (counter, snapshot) generator words; the ELBO forward copies the counter to the
    snapshot and advances it. ``mirror``: host-mapped int32 words the ELBO forward copies the
    validation words into.
    """
    _, bad = _lazy_uses(trace)
    if bad:
        _materialize_draws(trace, bad)
    claims = claim_linear_draws(trace)
    linears = plan_linear(trace, g0, device, claims)
    while True:
        launchers, categorical = plan_groups(trace, g0, device)
        bad = {l.draw for l in launchers if l.draw is not None and not l.draw_supported()}
        if not bad:
            break
        _materialize_draws(trace, bad)
    launchers = fold_linear_priors(fold_priors(launchers), linears)
    release_unsafe_claims(linears, launchers, categorical)
    claim_group_draws(trace, launchers)
    guide.flush_draws()   # draws made while planning (materialised lazy draws)
    fallback = [value for _, value in trace.fallback]
    absorbed = plan_absorption(factors, samples, launchers, linears, categorical, fallback)
    plan = _ElboPlan(trace.K, g0, device, launchers, categorical, fallback, factors,
                     entropy_scale, linears, absorbed, flags, step_words, mirror)
    inputs = plan.inputs()
    # which autograd inputs are tensors (nn._Loss.backward maps the gradients to next_functions)
    plan.tensor_inputs = [isinstance(t, torch.Tensor) for t in inputs]
    loss = _ElboFn.apply(plan, *inputs)
    global LAST_FUSIONS
    LAST_FUSIONS = plan.fusions()
    pending: List[Tuple[str, dict, List[SiteRecord]]] = []
    for (site, _, _, _), holder in zip(categorical, plan.cat_holders):
        pending.append(("categorical", holder, [site]))
    for linear, holder in zip(linears, plan.lin_holders):
        pending.append(("linear", holder, linear.flag_sites))
    for launcher, holder in zip(launchers, plan.holders):
        pending.append(("group", holder, launcher.flag_sites))
    joint = LogJoint(total=loss, pending=pending, checks=trace.checks, flags=plan.flags)
    if mirror is not None and plan.flags is not None and plan.flags.numel() <= mirror.numel():
        joint.mirror = mirror[:plan.flags.numel()]
    return loss, joint
