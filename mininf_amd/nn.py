"""
Learnable guides and losses (mirror of the reference's ``mininf/nn.py``).

``ParameterizedDistribution`` / ``FactorizedDistribution`` / ``ParameterizedFactorizedDistribution``
keep the reference's semantics exactly (host-side PyTorch modules, reference ``nn.py:29-187``).

``EvidenceLowerBoundLoss`` (reference ``nn.py:190-228``) is the hot path. The reference draws ONE
guide sample per call and runs the model once under ``LogProbTracer``; here ``num_particles=K``
draws are taken at once by HIP samplers, the unchanged model is traced once over all particles
(:mod:`mininf_amd.particles`), and the per-site log densities, their gradients and the
Monte-Carlo reduction run in fused HIP kernels (:mod:`mininf_amd.engine`). With ``num_particles=1``
the estimator is the reference's; for K > 1 it is the mean of K independent single-particle
estimates. The returned loss is a 0-d float32 tensor with ``grad_fn``.
"""
from __future__ import annotations

import ctypes
import os
import struct
from typing import Callable, cast, Dict, Optional, Set, Type

import torch
from torch import distributions, nn

from . import _native, engine, graph, guide, linear, particles
from .core import condition, LogProbTracer
from .util import _normalize_shape, maybe_as_tensor, OptionalSize, TensorDict


DistributionDict = Dict[str, torch.distributions.Distribution]


def _is_identity_transform(transform: distributions.Transform) -> bool:
    """
    ``transform_to`` of an unconstrained support returns an empty ComposeTransform (reference
    ``nn.py:16-26``).
    """
    return isinstance(transform, torch.distributions.ComposeTransform) and not transform.parts


def _forward_transform(transform: distributions.Transform) -> distributions.Transform:
    """
    The transform to apply in ``forward``: ``transform_to(positive)`` is
    ``ComposeTransform([ExpTransform(), AffineTransform(0., 1)])`` and ``0 + 1 * exp(u)`` is
    ``exp(u)`` exactly (same values and gradients), so the affine no-op -- two kernels forward and
    one backward per parameter -- is dropped.
    """
    if isinstance(transform, distributions.ComposeTransform) and len(transform.parts) == 2:
        first, second = transform.parts
        if isinstance(first, distributions.ExpTransform) and \
                isinstance(second, distributions.AffineTransform) and \
                isinstance(second.loc, (int, float)) and second.loc == 0 and \
                isinstance(second.scale, (int, float)) and second.scale == 1:
            return first
    return transform


class ParameterizedDistribution(nn.Module):
    """
    Distribution whose (constrained) parameters are learnable; they are stored unconstrained via
    ``transform_to(constraint).inv`` and mapped back on every call (reference ``nn.py:29-97``).

    Args:
        cls: Distribution type.
        _const: Names of parameters held constant.
        _clone: Copy parameters that need no transform so training does not modify the inputs.
        **parameters: Initial parameter values.

    Example:

        >>> from mininf_amd.nn import ParameterizedDistribution
        >>> from torch.distributions import Normal
        >>> ParameterizedDistribution(Normal, loc=0.5, scale=1.2)()
        Normal(loc: 0.5, scale: 1.2000000476837158)
    """
    def __init__(self, cls: Type[distributions.Distribution], *, _const: Set[str] | None = None,
                 _clone: bool = True, **parameters: torch.Tensor) -> None:
        super().__init__()
        self.distribution_cls = cls
        constant_names = _const or set()
        constraints = cast(Dict, cls.arg_constraints)
        self.distribution_constants: TensorDict = {}
        learnable = {}
        for name, initial in parameters.items():
            if name in constant_names or name not in constraints:
                self.distribution_constants[name] = initial
                continue
            initial = cast(torch.Tensor, maybe_as_tensor(initial))
            transform = distributions.transform_to(constraints[name])
            if _is_identity_transform(transform) and _clone:
                unconstrained = 1 * initial
            else:
                unconstrained = transform.inv(initial)
            learnable[name] = nn.Parameter(unconstrained)
        self.distribution_parameters = nn.ParameterDict(learnable)

    def forward(self) -> distributions.Distribution:
        """"""
        fused = self._fused_beta()
        if fused is not None:
            return fused
        constraints = cast(Dict, self.distribution_cls.arg_constraints)
        validate = self.distribution_constants.get("validate_args")
        if validate is None:
            validate = distributions.Distribution._validate_args
        arguments = {}
        sources = {}
        for name, unconstrained in self.distribution_parameters.items():
            transform = distributions.transform_to(constraints[name])
            # The reference exposes `1 * value` so the distribution never holds the nn.Parameter
            # itself (nn.py:92-94); a view is likewise a distinct tensor and costs no kernel.
            if _is_identity_transform(transform):
                arguments[name] = unconstrained.view_as(unconstrained)
                sources[name] = (unconstrained, "identity")
            else:
                forward = _forward_transform(transform)
                if isinstance(forward, distributions.ExpTransform) and unconstrained.is_cuda and \
                        unconstrained.dtype == torch.float32:
                    # one mi_transform_params; left to the draw unless the argument check
                    # below reads it at once
                    arguments[name] = _ExpFn.apply(unconstrained, not validate)
                else:
                    arguments[name] = forward(unconstrained)
                if isinstance(forward, distributions.ExpTransform):
                    sources[name] = (unconstrained, "exp")
        distribution = _construct(self.distribution_cls, arguments, self.distribution_constants)
        # How each parameter derives from this module's nn.Parameters: the fused ELBO can then
        # write the guide's gradients directly (mi_factor transforms, engine.elbo).
        distribution._mininf_amd_sources = sources  # type: ignore[attr-defined]
        return distribution  # type: ignore


    def _fused_beta(self) -> Optional[distributions.Distribution]:
        """
        A Beta guide with both concentrations learnable on the device: the two ``exp`` transforms
        and the ``torch.stack`` of ``Beta.__init__`` (beta.py:36-40) as one launch
        (``mi_transform_params``) writing the interleaved ``[..., 2]`` array its Dirichlet keeps;
        the distribution is then assembled exactly as ``Beta.__init__`` does, argument
        validation included.
        """
        if self.distribution_cls is not distributions.Beta:
            return None
        params = self.distribution_parameters
        if set(params) != {"concentration1", "concentration0"} or \
                set(self.distribution_constants) - {"validate_args"}:
            return None
        u1, u0 = params["concentration1"], params["concentration0"]
        if not (u1.is_cuda and u1.dtype == torch.float32 and u0.dtype == torch.float32 and
                u1.device == u0.device and u1.shape == u0.shape):
            return None
        validate = self.distribution_constants.get("validate_args")
        if validate is None:
            validate = distributions.Distribution._validate_args
        # validated: the check below reads the array at once, so the transform is launched here
        # instead of being left to the draw
        conc = _ExpStackFn.apply(u1, u0, not validate)
        beta = distributions.Beta.__new__(distributions.Beta)
        beta._dirichlet = distributions.Dirichlet(conc, validate_args=False)
        distributions.Distribution.__init__(beta, beta._dirichlet._batch_shape,
                                            validate_args=False)
        if validate:
            # Dirichlet's and Beta's three argument checks are all `conc > 0` elementwise: one
            # host synchronisation instead of three; torch raises its own error on failure
            if not torch._is_all_true(conc > 0):   # (it reduces the mask itself)
                distributions.Beta(conc[..., 0], conc[..., 1], validate_args=True)
            beta._validate_args = beta._dirichlet._validate_args = True
        beta._mininf_amd_sources = {  # type: ignore[attr-defined]
            "concentration1": (u1, "exp"), "concentration0": (u0, "exp")}
        return beta


# Guide families whose constructor builds no inner distribution: their argument validation can
# be taken over by _construct.
_ONE_SYNC = (distributions.Normal, distributions.Gamma)


def _construct(cls, arguments: Dict, constants: Dict) -> distributions.Distribution:
    """
    ``cls(**arguments, **constants)`` with torch's argument validation (``Distribution.__init__``,
    torch distribution.py:68-80) evaluated with ONE host synchronisation for all parameters
    instead of one per parameter. When a check fails the distribution is constructed again with
    validation, so torch raises its own error for the first failing parameter.
    """
    validate = constants.get("validate_args")
    if validate is None:
        validate = distributions.Distribution._validate_args
    if cls not in _ONE_SYNC or not validate:
        return cls(**arguments, **constants)
    plain = {k: v for k, v in constants.items() if k != "validate_args"}
    distribution = cls(**arguments, **plain, validate_args=False)
    checks = []
    for param, constraint in distribution.arg_constraints.items():
        if distributions.constraints.is_dependent(constraint) or param not in distribution.__dict__:
            continue
        checks.append(constraint.check(getattr(distribution, param)).reshape(-1))
    if checks:
        # one reduction of every parameter's mask (torch._is_all_true reduces it itself)
        ok = checks[0] if len(checks) == 1 else torch.cat(checks)
        if not torch._is_all_true(ok):
            cls(**arguments, **plain, validate_args=True)   # raises torch's error
    distribution._validate_args = True
    return distribution


def _float32(value: float) -> float:
    """``value`` rounded to float32 (as ``float(torch.tensor(value, dtype=torch.float32))``,
    without creating a tensor)."""
    return struct.unpack("f", struct.pack("f", value))[0]


def _defer_exp() -> bool:
    """Whether guide exp transforms are left to the draws that read them (MININF_AMD_DEFER_EXP)."""
    return os.environ.get("MININF_AMD_DEFER_EXP", "1") != "0"


class _ExpFn(torch.autograd.Function):
    """``exp(u)`` of a positive-constrained guide parameter (``transform_to(positive)``,
    nn.py:91-96) as one ``mi_transform_params`` launch."""
    @staticmethod
    def forward(ctx, u: torch.Tensor, defer: bool = True):  # type: ignore[override]
        out = torch.empty(u.shape, dtype=torch.float32, device=u.device)
        ctx.save_for_backward(out)
        if u.numel() > 0:
            flat = u.reshape(-1)
            P = _native.Params()
            P.m, P.n = 1, flat.numel()
            P.u[0] = flat.data_ptr()
            P.stride[0] = flat.stride(0) if flat.numel() > 1 else 0
            P.transform[0] = _native.TRANSFORM_EXP
            if defer and _defer_exp() and u.is_contiguous():
                # the guide's draw computes and writes the scale (mi_normal_rsample_exp); any
                # earlier reader launches the transform itself (guide.PendingConcentration)
                return guide.defer_exp(out.as_subclass(guide.PendingConcentration), u, None, P)
            _native.check(_native.lib().mi_transform_params(ctypes.byref(P), out.data_ptr(),
                                                            _native.stream_handle(u.device)),
                          "mi_transform_params")
        return out

    @staticmethod
    def backward(ctx, grad: torch.Tensor):  # type: ignore[override]
        (out,) = ctx.saved_tensors
        return grad * out, None   # d exp(u) / du = exp(u)


class _ExpStackFn(torch.autograd.Function):
    """``torch.stack([exp(u1), exp(u0)], -1)`` in one launch (``mi_transform_params``)."""
    @staticmethod
    def forward(ctx, u1: torch.Tensor, u0: torch.Tensor,  # type: ignore[override]
                defer: bool = True):
        out = torch.empty(tuple(u1.shape) + (2,), dtype=torch.float32, device=u1.device)
        P = _native.Params()
        P.m, P.n = 2, max(1, u1.numel())
        for j, u in enumerate((u1, u0)):
            flat = u.reshape(-1)
            P.u[j] = flat.data_ptr()
            P.stride[j] = flat.stride(0) if u.numel() > 1 else 0
            P.transform[j] = _native.TRANSFORM_EXP
        ctx.save_for_backward(out)
        if defer and _defer_exp() and u1.is_contiguous() and u0.is_contiguous():
            # the guide's draw computes and writes the array (mi_beta_rsample_exp); any earlier
            # reader launches the transform itself (guide.PendingConcentration). Only for
            # contiguous parameters: P then points into their own storage, not into a reshape
            # copy that is freed when this call returns
            return guide.defer_exp(out.as_subclass(guide.PendingConcentration), u1, u0, P)
        _native.check(_native.lib().mi_transform_params(ctypes.byref(P), out.data_ptr(),
                                                        _native.stream_handle(u1.device)),
                      "mi_transform_params")
        return out

    @staticmethod
    def backward(ctx, grad: torch.Tensor):  # type: ignore[override]
        (out,) = ctx.saved_tensors
        d = grad * out   # d exp(u) / du = exp(u)
        return d[..., 0], d[..., 1], None


class FactorizedDistribution(DistributionDict):
    """
    Mean-field joint of independent named factors (reference ``nn.py:100-159``).
    """
    def entropy(self) -> torch.Tensor:
        """
        Total entropy, summed over factors and their elements.
        """
        return cast(torch.Tensor, sum(factor.entropy().sum() for factor in self.values()))

    def rsample(self, sample_shape: OptionalSize = None) -> TensorDict:
        """
        One reparameterised draw per factor.
        """
        shape = _normalize_shape(sample_shape)
        return {name: factor.rsample(shape) for name, factor in self.items()}

    def sample(self, sample_shape: OptionalSize = None) -> TensorDict:
        """
        One draw per factor (no gradient).
        """
        shape = _normalize_shape(sample_shape)
        return {name: factor.sample(shape) for name, factor in self.items()}


class ParameterizedFactorizedDistribution(nn.ModuleDict):
    """
    Module dictionary of :class:`ParameterizedDistribution` returning a
    :class:`FactorizedDistribution` (reference ``nn.py:162-187``).
    """
    def __init__(self, arg: Dict[str, ParameterizedDistribution] | None = None,
                 **kwargs: ParameterizedDistribution) -> None:
        modules = dict(arg or {})
        modules.update(kwargs)
        super().__init__(modules)

    def forward(self) -> FactorizedDistribution:
        return FactorizedDistribution({name: module() for name, module in self.items()})


_UNIT: Dict[torch.device, torch.Tensor] = {}


class _Loss(torch.Tensor):
    """
    The loss tensor the fused ELBO returns: an ordinary 0-d tensor (operations on it give plain
    tensors) whose ``backward()`` seeds autograd with a cached device 1.0 instead of
    ``torch.ones_like(loss)`` -- otherwise a fill launch in every (captured) training step. An
    operation on it first enqueues the step's held finishing launch (engine._PendingStep).
    """
    __torch_function__ = classmethod(lambda cls, func, types, args=(), kwargs=None:
                                     engine.torch_function_flush(func, types, args, kwargs))

    def __repr__(self, *, tensor_contents=None):
        return torch._tensor_str._str(self, tensor_contents=tensor_contents).replace(
            type(self).__name__ + "(", "tensor(", 1)

    def backward(self, gradient=None, retain_graph=None, create_graph=False, inputs=None):
        if gradient is None and self.dim() == 0 and self.is_cuda and not create_graph:
            gradient = _UNIT.get(self.device)
            if gradient is None and not torch.cuda.is_current_stream_capturing():
                gradient = _UNIT[self.device] = torch.ones((), dtype=self.dtype,
                                                           device=self.device)
            if gradient is not None and gradient.dtype != self.dtype:
                gradient = None
            if gradient is not None and inputs is None and not retain_graph and \
                    _accumulate_final_grads(self, gradient):
                return
        torch.Tensor.backward(self, gradient, retain_graph, create_graph, inputs)


def _accumulate_final_grads(loss: torch.Tensor, unit: torch.Tensor) -> bool:
    """
    ``loss.backward()`` of a fused ELBO whose forward already wrote the guide gradients for this
    upstream (engine MI_ELBO_FINAL_GRADS, the README training loop): when every gradient goes
    straight to a leaf parameter (no hooks, same layout), accumulate them as AccumulateGrad would
    -- ``p.grad = g``, or ``p.grad += g`` -- without starting the autograd engine (its device
    thread hand-off is most of an eager backward's host time). False (nothing done): let autograd
    run. MININF_AMD_DIRECT_GRADS=0 disables it.

    Autograd also runs when ``loss.retain_grad()`` was called (it sets ``loss.grad``), and while a
    ``torch.distributed`` process group is initialised: hooks on the AccumulateGrad nodes
    themselves (DDP's reducer, ``grad_acc.register_hook``) are not visible on the parameter, and
    only the engine runs them. A single-process user of node-level hooks sets
    MININF_AMD_DIRECT_GRADS=0.
    """
    fn = loss.grad_fn
    plan = getattr(fn, "plan", None)
    tensor_inputs = getattr(plan, "tensor_inputs", None)
    if plan is None or getattr(plan, "final", None) is None or plan.state is None or \
            tensor_inputs is None or loss._backward_hooks or loss.retains_grad or \
            os.environ.get("MININF_AMD_DIRECT_GRADS", "1") == "0":
        return False
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return False
    # next_functions: one entry per tensor input of _ElboFn.apply (None inputs have none)
    nexts = fn.next_functions
    if len(nexts) != sum(tensor_inputs):
        return False
    leaves = []
    cursor = 0
    for is_tensor in tensor_inputs:
        if not is_tensor:
            leaves.append(None)
            continue
        node = nexts[cursor][0]
        cursor += 1
        if node is None:   # an input that needs no gradient
            leaves.append(None)
            continue
        var = getattr(node, "variable", None)   # AccumulateGrad of a leaf
        if var is None or var._backward_hooks or \
                getattr(var, "_post_accumulate_grad_hooks", None) or not var.is_contiguous():
            return False
        leaves.append(var)
    grads = plan.backward(unit, hold=True)
    if len(grads) != len(leaves):
        raise RuntimeError("fused ELBO: gradient count does not match the autograd inputs")
    pending = engine.pending_step()
    for var, grad in zip(leaves, grads):
        if var is None or grad is None:
            continue
        if grad.shape != var.shape:
            grad = grad.reshape(var.shape)   # (contiguous: a view)
        if var.grad is None:
            # a gradient the held finishing launch writes stays held (the optimizer step may
            # join that launch): its first use enqueues it
            if pending is not None and grad.data_ptr() in pending.grad_ptrs:
                grad = pending.hold(var, grad)
            var.grad = grad
        else:
            engine.flush_pending_step()
            var.grad += grad
    return True


class EvidenceLowerBoundLoss(nn.Module):
    """
    Negative evidence lower bound, estimated with ``num_particles`` Monte-Carlo particles on the
    MI355X (reference ``nn.py:190-228``).

    Args:
        num_particles: Total number of particles K across all ranks (reference: 1).
        seed: Seed of the counter-based guide sampler (default: derived from ``torch.initial_seed``).
        validate: Check value supports and parameter constraints (one host sync per call), as the
            reference does on every call (``core.py:142-189``).
        process_group: ``torch.distributed`` group to shard the particles over (one rank per GPU);
            each rank returns its share of the loss and gradients, combine them with
            :func:`mininf_amd.distributed.all_reduce_gradients`.
        data_shard: Shard the data axis instead of the particles
            (:class:`mininf_amd.distributed.DataShard`): every rank evaluates all
            ``num_particles`` particles on its slice of the elements; the model and guide it is
            called with are the rank's slice. Shared factors and sites count 1/W per rank, the
            sharded factors draw their slice of the global draw.

    Example:

        >>> import torch
        >>> from mininf_amd import sample
        >>> from mininf_amd.nn import EvidenceLowerBoundLoss
        >>> from torch.distributions import Normal
        >>> def model():
        ...     sample("x", Normal(0, 1))
        >>> loss = EvidenceLowerBoundLoss(num_particles=256)
        >>> loss(model, {"x": Normal(torch.zeros((), device="cuda"), 1.0)})  # doctest: +SKIP
        tensor(..., device='cuda:0')
    """
    def __init__(self, num_particles: int = 1, *, seed: Optional[int] = None,
                 validate: bool = True, process_group=None, data_shard=None) -> None:
        super().__init__()
        if num_particles < 1:
            raise ValueError("num_particles must be positive")
        self.num_particles = int(num_particles)
        self.seed = int(seed if seed is not None else torch.initial_seed()) & ((1 << 64) - 1)
        self.validate = validate
        self.process_group = process_group
        self.data_shard = data_shard
        if data_shard is not None and process_group is None and data_shard.world is None:
            raise ValueError("data_shard needs the process_group it shards over (or its world)")
        self._counter: Optional[torch.Tensor] = None   # device step counter of the guide RNG
        # the fast paths the last evaluation took (engine._ElboPlan.fusions)
        self.last_fusions: Dict[str, int] = {}
        self._sticky_flags: Optional[torch.Tensor] = None   # graph-mode validation words
        # eager steps' validation words: rows of one zeroed block, a fresh block every
        # FLAG_POOL steps (one fill launch per block instead of one per step)
        self._flag_pool: Optional[torch.Tensor] = None
        self._flag_next = 0
        self._mirror: Optional[torch.Tensor] = None   # their pinned host copy

    # validation words zeroed with the step counter's advance; plans with more sites zero their own
    FLAG_WORDS = 64
    FLAG_POOL = 64

    def _zeroed_flags(self, device: torch.device) -> torch.Tensor:
        """Zeroed validation words for one eager step: a row no earlier step wrote (a used block
        is never zeroed again: it is dropped, and lives on only while a joint still reads it).
        Inside a graph capture the words come from the graph's own pool (a fill every replay): a
        row of a block allocated outside the capture would not be zeroed by replays, and the block
        could be freed while the graph still writes into it."""
        if device.type == "cuda" and torch.cuda.is_current_stream_capturing():
            return torch.zeros(self.FLAG_WORDS, dtype=torch.int32, device=device)
        pool = self._flag_pool
        if pool is None or pool.device != device or self._flag_next >= pool.shape[0]:
            pool = self._flag_pool = torch.zeros((self.FLAG_POOL, self.FLAG_WORDS),
                                                 dtype=torch.int32, device=device)
            self._flag_next = 0
        row = pool[self._flag_next]
        self._flag_next += 1
        return row

    def _shard(self):
        """
        (world size, rank, local K, particle offset) of this rank.
        """
        if self.data_shard is not None:   # every rank holds every particle
            import torch.distributed as dist
            world = self.data_shard.world or dist.get_world_size(self.process_group)
            rank = dist.get_rank(self.process_group) if self.process_group is not None else 0
            return world, rank, self.num_particles, 0
        if self.process_group is None:
            return 1, 0, self.num_particles, 0
        import torch.distributed as dist
        world = dist.get_world_size(self.process_group)
        rank = dist.get_rank(self.process_group)
        if self.num_particles % world:
            raise ValueError(f"num_particles={self.num_particles} is not divisible by the world "
                             f"size {world}")
        local = self.num_particles // world
        return world, rank, local, rank * local

    def _element_offsets(self, approximation) -> Optional[Dict[str, int]]:
        """Global element offsets of the data-sharded guide factors (None: no data sharding)."""
        if self.data_shard is None:
            return None
        return {name: self.data_shard.start for name in approximation
                if name not in self.data_shard.shared}

    def forward(self, model: Callable,
                approximation: torch.distributions.Distribution | DistributionDict,
                _noise: Optional[Dict[str, torch.Tensor]] = None) -> torch.Tensor:
        """"""
        if isinstance(approximation, Dict):
            approximation = FactorizedDistribution(approximation)
        if self.data_shard is not None and not isinstance(approximation, dict):
            raise TypeError("data sharding needs a factorised (dictionary) guide")
        world, _, K, offset = self._shard()
        if isinstance(approximation, dict):
            device = _guide_device(approximation)
            if self._counter is None or self._counter.device != device:
                self._counter = torch.zeros(1, dtype=torch.int64, device=device)
            # The forward's draws read the device counter; the ELBO forward copies it into this
            # call's snapshot (read by everything after it: the draws' backward) and advances it,
            # so replays of a captured step draw anew without a separate launch.
            sticky = False
            mirror = None
            step_words = None
            snapshot = None
            if device.type == "cuda":
                step = self._counter
                snapshot = torch.empty(1, dtype=torch.int64, device=device)
                step_words = (self._counter, snapshot)
                if graph.deferred() is not None:
                    # Graph mode: validation words that no replay zeroes. Violations accumulate
                    # until the host reads them (StepGraph), so a replay that the host never
                    # inspects cannot lose one; StepGraph clears them when it raises. The ELBO
                    # forward also copies them into pinned host memory (no separate copy).
                    if self._sticky_flags is None or self._sticky_flags.device != device:
                        self._sticky_flags = torch.zeros(self.FLAG_WORDS, dtype=torch.int32,
                                                         device=device)
                    if self._mirror is None and not torch.cuda.is_current_stream_capturing():
                        self._mirror = torch.zeros(self.FLAG_WORDS, dtype=torch.int32,
                                                   pin_memory=True)
                    flags, sticky = self._sticky_flags, True
                    mirror = self._mirror if graph.mirrors_flags() else None
                else:
                    flags = self._zeroed_flags(device)
            else:   # the samplers reject host guides with the engine's device error
                step, flags = self._counter.clone(), None
                self._counter.add_(1)
            # Large Normal factors are drawn lazily: the site kernels compute them in registers
            # (mi_draw). If the model uses a draw in any other operation, the trace is repeated
            # with real draws (same counter, same values).
            offsets = self._element_offsets(approximation)
            samples = guide.draw_all(approximation, K, self.seed, 0, offset, _noise,
                                     step_device=step, lazy=True, step_snapshot=snapshot,
                                     element_offsets=offsets)
            try:
                trace = particles.trace_particles(model, samples, K, validate=self.validate)
            except linear.NeedsDraws:
                guide.release_lazy()
                samples = guide.draw_all(approximation, K, self.seed, 0, offset, _noise,
                                         step_device=step, step_snapshot=snapshot,
                                         element_offsets=offsets)
                trace = particles.trace_particles(model, samples, K, validate=self.validate)
        else:
            samples = approximation.rsample(torch.Size([K]))
            if not isinstance(samples, Dict):
                raise TypeError("Expected a distribution which samples dictionaries of tensors "
                                f"but got a sample of type {type(samples)}")
            trace = particles.trace_particles(model, samples, K, validate=self.validate)
        # d loss / d T_k = -1 / K exactly (fp32), matching the `mul(-1/K)` below.
        g0 = _float32(-1.0 / self.num_particles)
        device = next((t.device for t in samples.values() if isinstance(t, torch.Tensor)),
                      torch.device("cuda", torch.cuda.current_device()))
        shared = set(self.data_shard.shared) if self.data_shard is not None else None
        if shared is not None:
            # data sharding: replicated sites count 1/W on every rank (the ranks' sum is the
            # full log joint); the sharded sites' slices add up by themselves
            for site in trace.sites:
                if site.name in shared:
                    site.scale /= world
            trace.fallback = [(name, value / world if name in shared else value)
                              for name, value in trace.fallback]
        if isinstance(approximation, dict):
            # Fused path: site kernels, guide entropy and the reduction in one autograd node.
            factors, rest = engine.entropy_factors(approximation)
            entropy_scale = 1.0 / world
            if shared is not None:
                entropy_scale = 1.0
                for f in factors:
                    f.weight = 1.0 / world if f.name in shared else 1.0
            try:
                loss, joint = engine.elbo(trace, g0, device, factors, entropy_scale, samples,
                                          flags=flags, step_words=step_words, mirror=mirror)
                # (the same dict: an optimizer step that joins the held launch marks it)
                self.last_fusions = engine.LAST_FUSIONS
                joint.sticky = sticky and joint.flags is not None and not joint.checks and \
                    joint.flags.data_ptr() == flags.data_ptr()
            finally:
                # The placeholder registry is only needed while tracing and planning; holding it
                # would keep this step's autograd graph (and its AccumulateGrad streams) alive.
                guide.release_lazy()
            if rest:
                names = {id(f): name for name, f in approximation.items()}
                extra = cast(torch.Tensor, sum(
                    f.entropy().sum() / (world if shared is None or names[id(f)] in shared else 1)
                    for f in rest))
                engine.flush_pending_step()
                loss = loss - extra
            if loss.is_cuda and loss.dim() == 0 and type(loss) is torch.Tensor:
                loss.__class__ = _Loss   # the same tensor object and autograd node
        else:
            joint = engine.log_joint(trace, g0, device)
            entropy = approximation.entropy()
            if world > 1:
                entropy = entropy / world
            loss = (joint.total * g0).sum() - entropy
        if self.validate:
            collector = graph.deferred()
            if collector is not None:
                collector.append(joint)
            else:
                joint.raise_on_violation()
        return loss


def _guide_device(approximation: Dict[str, torch.distributions.Distribution]) -> torch.device:
    for factor in approximation.values():
        for item in vars(factor).values():
            if isinstance(item, torch.Tensor):
                return item.device
    return torch.device("cuda", torch.cuda.current_device())


class LogLikelihoodLoss(nn.Module):
    """
    Negative log likelihood at fixed parameter values (reference ``nn.py:231-257``).

    When the parameters live on a ROCm device, the model is traced with the particle tracer at
    K = 1 and every kernel-family site is evaluated by the same HIP site kernels as the ELBO
    (``mi_group_forward``; speculative gradients for the upstream -1). Host (CPU) parameters keep
    the reference's torch-CPU evaluation through :class:`~mininf_amd.core.LogProbTracer`.

    Example:

        >>> from mininf_amd import sample
        >>> from mininf_amd.nn import LogLikelihoodLoss
        >>> from torch.distributions import Normal
        >>> def model() -> None:
        ...     sample("x", Normal(0, 1))
        >>> LogLikelihoodLoss()(model, {"x": 0.1})
        tensor(0.9239)
    """
    def forward(self, model: Callable, parameters: TensorDict) -> torch.Tensor:
        """"""
        device = next((v.device for v in parameters.values()
                       if isinstance(v, torch.Tensor) and v.is_cuda), None)
        if device is None:
            with LogProbTracer() as log_prob:
                condition(model, **parameters)()
            return - log_prob.total
        samples, observed = {}, {}
        for name, value in parameters.items():
            if isinstance(value, torch.masked.MaskedTensor):
                observed[name] = value   # masked observations: shared data, not a particle axis
                continue
            if not isinstance(value, torch.Tensor):
                value = torch.as_tensor(value, dtype=torch.get_default_dtype(), device=device)
            samples[name] = value.unsqueeze(0)
        if observed:
            model = condition(model, **observed)
        trace = particles.trace_particles(model, samples, 1)
        joint = engine.log_joint(trace, -1.0, device)
        collector = graph.deferred()
        if collector is not None:
            collector.append(joint)
        else:
            joint.raise_on_violation()
        return - joint.total[0]
