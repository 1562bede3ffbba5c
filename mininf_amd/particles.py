"""
Particle tracer: run an unchanged model once over all K Monte-Carlo particles and record its sites.

The reference evaluates the log joint for ONE guide draw per loss call (``mininf/nn.py:217-226``)
by running the model under ``LogProbTracer`` (``mininf/core.py:207-277``), which calls
``distribution.log_prob(value)`` site by site. Here the model runs under :func:`torch.func.vmap`
over the particle axis: user code still sees per-particle shapes (so ``sample`` shape validation,
``batch`` and ``no_log_prob`` behave exactly as in the reference), but every tensor it produces is
batched over K. :class:`ParticleTracer` is a :class:`~mininf_amd.core.TracerMixin` (the reference's
plugin point, ``core.py:128-140``) that, instead of evaluating log densities, records each site's
family, parameter tensors, value, mask and minibatch scale. The recorded [K, ...] tensors come back
out of ``vmap`` and are handed to the HIP site kernels (:mod:`mininf_amd.engine`).

Sites recorded as "torch" sites (MultivariateNormal, other families without a site kernel) are
evaluated inside the same ``vmap`` (on the GPU) and contribute one per-particle sum; a float32
MultivariateNormal is refactorised in float64 and its density runs on ``mi_mvn_tril_forward``
(:mod:`mininf_amd.mvn`), anything else through ``torch.distributions``.
"""
from __future__ import annotations

import collections
import contextlib
import copy
import dataclasses
import hashlib
import os
import weakref
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple, cast

import torch
from torch.distributions import Bernoulli, Beta, Categorical, Distribution, Gamma, \
    MultivariateNormal, Normal, Poisson, PowerTransform, TransformedDistribution
from torch.distributions.constraints import Constraint
from torch.distributions.utils import lazy_property
from torch.overrides import TorchFunctionMode
from torch.utils._pytree import tree_flatten, tree_map

from . import core, data, mvn, predictive
from .distributions import InverseGamma
from .core import batch, no_log_prob, State, TracerMixin, Value, validate_shape
from .util import _normalize_shape, check_constraint, OptionalSize


_functorch = torch._C._functorch
from torch._functorch import vmap as _vmap  # noqa: E402  (vmap_increment_nesting)


def is_batched(tensor: Any) -> bool:
    return isinstance(tensor, torch.Tensor) and _functorch.is_batchedtensor(tensor)


def broadcast_shapes(*shapes: Tuple[int, ...]) -> Tuple[int, ...]:
    """``torch.broadcast_shapes`` of plain shape tuples in a few Python operations (torch's version
    goes through its reference implementation: several microseconds per site and trace); a
    mismatch is handed to torch, which raises its own error."""
    ndim = max((len(s) for s in shapes), default=0)
    out = [1] * ndim
    for s in shapes:
        for i, d in enumerate(s, ndim - len(s)):
            if d != 1:
                if out[i] != 1 and out[i] != d:
                    return tuple(torch.broadcast_shapes(*shapes))
                out[i] = d
    return tuple(out)


def vmap_tensors(fn: Callable, args: Sequence[torch.Tensor]) -> Tuple[torch.Tensor, ...]:
    """
    ``torch.func.vmap(fn, randomness="different")(*args)`` for positional tensor arguments batched
    along dimension 0 and a tuple of tensors returned, on functorch's own primitives (one nesting
    level, ``_add_batch_dim`` per argument, ``_remove_batch_dim`` per output) without the pytree
    flattening and argument checks of the public wrapper -- about 90 us of host time per call on
    this image, the largest fixed cost of an eager trace. Anything else (a non-tensor argument,
    mismatched batch sizes) takes ``torch.func.vmap`` itself, which raises its own errors.
    """
    K = args[0].shape[0] if args and isinstance(args[0], torch.Tensor) and args[0].dim() else -1
    if K < 0 or any(not isinstance(a, torch.Tensor) or a.dim() == 0 or a.shape[0] != K
                    for a in args):
        return torch.func.vmap(fn, randomness="different")(*args)
    _vmap.lazy_load_decompositions()
    with _vmap.vmap_increment_nesting(K, "different") as level:
        outputs = fn(*[_functorch._add_batch_dim(a, 0, level) for a in args])
        if not isinstance(outputs, tuple) or \
                any(not isinstance(o, torch.Tensor) for o in outputs):
            raise ValueError(f"vmap({getattr(fn, '__name__', fn)}, ...): the traced function must "
                             f"return a tuple of Tensors, got {type(outputs)}")
        return tuple(_functorch._remove_batch_dim(o, level, K, 0) for o in outputs)


@dataclasses.dataclass
class SiteRecord:
    """
    One ``sample`` statement that contributes to the log joint.

    ``roles`` holds output indices into the vmapped function's outputs for the family's roles
    (Normal: loc, scale, value; Bernoulli: logits|probs, value; Beta: concentration1,
    concentration0, value; Categorical: logits, value). After :func:`trace_particles` returns,
    ``tensors`` holds the corresponding [K, ...] tensors.
    """
    name: str
    family: str
    roles: List[int]
    site_shape: torch.Size
    scale: float
    mask: Optional[torch.Tensor]
    description: str
    tensors: List[torch.Tensor] = dataclasses.field(default_factory=list)
    # Linear-predictor site (loc / logits = X @ theta deferred by mininf_amd.linear): the observed
    # design matrix, the output index of theta and, after tracing, theta as [K, P].
    linear_X: Optional[torch.Tensor] = None
    linear_theta_index: int = -1
    linear_theta: Optional[torch.Tensor] = None
    order: int = 0   # position of the sample statement in the model (errors raise in this order)


@dataclasses.dataclass
class CheckRecord:
    """
    A support / constraint check evaluated on the device and resolved with the step's single
    validation sync. ``output`` indexes a (per-particle) boolean output of the vmapped trace;
    ``memo`` is committed to the validation memo once the check has passed.
    """
    name: str
    output: int
    message: str
    memo: Optional[Tuple] = None
    order: int = 0


# Unbatched (conditioned) data is validated once per tensor version instead of on every step:
# key -> (weakref to tensor, version). The reference re-checks the full tensor on every call
# (core.py:186-188), which is 27-63 % of its step time; the result is identical.
_VALIDATED: Dict[Tuple, Tuple[weakref.ref, int]] = {}


def _memo_key(value: torch.Tensor, constraint: Constraint) -> Tuple:
    return (value.data_ptr(), tuple(value.shape), tuple(value.stride()), value.dtype,
            str(value.device), repr(constraint))


def _plain(value: torch.Tensor) -> torch.Tensor:
    # The private fields avoid MaskedTensor.get_data (an autograd.Function, not vmap-compatible);
    # the reference reads the same fields (mininf/util.py:85-89).
    return value._masked_data if isinstance(value, torch.masked.MaskedTensor) else value


def device_check(constraint: Constraint, value: torch.Tensor) -> torch.Tensor:
    """
    ``check_constraint(constraint, value).all()`` as a 0-d device tensor (no host sync), usable
    inside vmap; masked-out elements pass.
    """
    with torch.no_grad():
        passed = constraint.check(_plain(value))
        if isinstance(value, torch.masked.MaskedTensor):
            mask = value._masked_mask
            for _ in range(constraint.event_dim):
                mask = mask.all(-1)
            passed = passed | ~mask
        return passed.all()


def memo_lookup(value: torch.Tensor, constraint: Constraint) -> Optional[Tuple]:
    """
    None if this exact tensor version already passed this check, else the memo entry to commit
    once the (deferred) check has passed.
    """
    plain = _plain(value)
    key = _memo_key(plain, constraint)
    hit = _VALIDATED.get(key)
    if hit is not None and hit[0]() is plain and hit[1] == plain._version:
        return None
    return (key, weakref.ref(plain), plain._version)


def memo_commit(entry: Tuple) -> None:
    key, ref, version = entry
    if ref() is not None:
        _VALIDATED[key] = (ref, version)


# host tensors up to this size are also keyed by their contents (device_copy)
_CONTENT_KEY_BYTES = 1 << 20
_HOST_COPIES: "collections.OrderedDict[Tuple, Tuple[torch.Tensor, torch.Tensor]]" = \
    collections.OrderedDict()


# device copies read by the step being captured (StepGraph keeps them for the graph's lifetime:
# the LRU below may evict an entry while a graph still reads its copy)
_PINS: Optional[List[torch.Tensor]] = None


@contextlib.contextmanager
def pin_device_copies():
    """Collect every device copy ``device_copy`` hands out inside the block (a capture)."""
    global _PINS
    saved, _PINS = _PINS, []
    try:
        yield _PINS
    finally:
        _PINS = saved


def _content_digest(t: torch.Tensor) -> Optional[bytes]:
    """blake2b of a host tensor's values (None when numpy cannot view them)."""
    data = t.detach().resolve_conj().resolve_neg().contiguous()
    if data.dtype == torch.bfloat16:
        data = data.view(torch.int16)
    try:
        return hashlib.blake2b(data.numpy().tobytes(), digest_size=16).digest()
    except (TypeError, RuntimeError):
        return None


def device_copy(t: torch.Tensor, device: torch.device) -> torch.Tensor:
    """
    A cached device copy of an unbatched host tensor (keyed on storage, layout and version), so a
    constant such as the 2.0 of ``Gamma(2.0, 2.0)`` is copied once, not on every step (and not
    inside a captured graph).
    """
    out = _device_copy(t, device)
    if _PINS is not None:
        _PINS.append(out)
    return out


def _device_copy(t: torch.Tensor, device: torch.device) -> torch.Tensor:
    key = (t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.dtype, t._version, str(device))
    hit = _HOST_COPIES.get(key)
    digest = None
    if hit is None and t.numel() * t.element_size() <= _CONTENT_KEY_BYTES:
        digest = _content_digest(t)
    if digest is not None:
        # A small host intermediate the model computes afresh on every call (the GP example's
        # `x[:, None] - x`, examples/missing-observations.md:40) is a new tensor each time: key it
        # by its contents, so a captured step finds the copy its warm-up made instead of a
        # host-to-device copy, which a capturing stream refuses.
        content = ("content", tuple(t.shape), t.dtype, str(device), digest)
        hit = _HOST_COPIES.get(content)
        if hit is not None:
            _HOST_COPIES.move_to_end(content)
            return hit[1]
        key = content
        t = t.detach().resolve_conj().resolve_neg().contiguous()
    if hit is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError(
                f"a host tensor of shape {tuple(t.shape)} meets device particles for the first "
                "time inside a captured step; its host-to-device copy cannot be captured. Build it "
                "on the device, or run the step once before capturing it.")
        hit = (t, t.to(device))
        _HOST_COPIES[key] = hit
        while len(_HOST_COPIES) > 64:
            _HOST_COPIES.popitem(last=False)
    else:
        _HOST_COPIES.move_to_end(key)
    return hit[1]


def _on_device(obj: Any, device: torch.device) -> Any:
    """
    A shallow copy of a distribution (or transform) whose unbatched host tensors -- and those of
    nested distributions and transforms -- are replaced by device copies: torch-evaluated sites
    then compute on the device. (Under vmap, torch evaluates e.g. Gamma(2., 2.).log_prob of a
    device value on the HOST when the parameters are host tensors.)
    """
    from torch.distributions import Transform
    changes = {}
    for key, item in vars(obj).items():
        if isinstance(item, torch.Tensor):
            if item.device.type == "cpu" and not is_batched(item) and not item.requires_grad:
                changes[key] = device_copy(item, device)
        elif isinstance(item, (Distribution, Transform)):
            moved = _on_device(item, device)
            if moved is not item:
                changes[key] = moved
        elif isinstance(item, (list, tuple)) and any(isinstance(x, (Distribution, Transform))
                                                      for x in item):
            moved_items = [_on_device(x, device) if isinstance(x, (Distribution, Transform))
                           else x for x in item]
            if any(a is not b for a, b in zip(moved_items, item)):
                changes[key] = type(item)(moved_items)
    if not changes:
        return obj
    out = copy.copy(obj)
    for key, item in changes.items():
        setattr(out, key, item)
    return out


def classify(distribution: Distribution) -> Tuple[str, List[Any]]:
    """
    Map a distribution onto a HIP site family and its role tensors, or ``("torch", [])``.
    Exact type checks: subclasses may override ``log_prob``.
    """
    cls = type(distribution)
    if cls is Normal:
        return "normal", [distribution.loc, distribution.scale]
    if cls is Bernoulli:
        # torch evaluates via self.logits (bernoulli.py:121-125); use whichever parameter the
        # distribution was constructed with so no extra lazy tensor is materialised.
        if "logits" in distribution.__dict__:
            return "bernoulli_logits", [distribution.logits]
        return "bernoulli_probs", [distribution.probs]
    if cls is Beta:
        return "beta", [distribution.concentration1, distribution.concentration0]
    if cls is Categorical:
        return "categorical", [distribution.logits]
    if cls is Gamma:
        return "gamma", [distribution.concentration, distribution.rate]
    if cls is Poisson:
        return "poisson", [distribution.rate]
    if _is_inverse_gamma(distribution):
        base = cast(Gamma, cast(TransformedDistribution, distribution).base_dist)
        return "inverse_gamma", [base.concentration, base.rate]
    return "torch", []


def _is_inverse_gamma(distribution: Distribution) -> bool:
    """
    Gamma through a single PowerTransform(-1) (mininf/distributions.py:5-11, or the same
    construction spelled out) whose log_prob is TransformedDistribution's own.
    """
    if not isinstance(distribution, TransformedDistribution) or \
            type(distribution).log_prob is not TransformedDistribution.log_prob or \
            type(distribution.base_dist) is not Gamma or len(distribution.transforms) != 1:
        return False
    t = distribution.transforms[0]
    if type(t) is not PowerTransform or is_batched(t.exponent):
        return False
    if isinstance(distribution, InverseGamma):   # PowerTransform(-1) by construction
        return True
    exponent = t.exponent
    if not isinstance(exponent, torch.Tensor):
        return exponent == -1
    if exponent.device.type != "cpu" and torch.cuda.is_current_stream_capturing():
        return False   # unreadable while capturing: the generic torch site path (same density)
    return bool((exponent == -1).all())


class ParticleTracer(TracerMixin):
    """
    Records sites of a model executing under ``vmap`` over particles.
    """
    def __init__(self, validate: bool = True) -> None:
        super().__init__(_validate_parameters=validate)
        self.sites: List[SiteRecord] = []
        self.names: set = set()
        self.outputs: List[torch.Tensor] = []
        self.checks: List[CheckRecord] = []
        self.fallback_outputs: List[Tuple[str, int]] = []
        self.deferred = None   # the DeferredMatmul mode of the trace, if any
        self.order = 0         # sample statements seen so far

    def _emit(self, tensor: torch.Tensor) -> int:
        self.outputs.append(tensor)
        return len(self.outputs) - 1

    def _check_support(self, name: str, value: Any, distribution: Distribution,
                       constraint: Constraint) -> None:
        """
        Value-support check of sites the kernels do not read (values, no_log_prob sites, torch
        sites). Conditioned data that already passed (same storage and version) is skipped; the
        rest is evaluated on the device and raised with the step's single validation sync.
        """
        if not self._validate_parameters:
            return
        # A device-resident minibatch is a subset of its dataset column: the column is checked
        # (once per version) instead of every batch (mininf_amd.data).
        column = data.dataset_column(_plain(value))
        if column is not None:
            value = column
        memo = None
        if not (is_batched(value) or is_batched(_plain(value))):
            memo = memo_lookup(value, constraint)
            if memo is None:
                return
        try:
            described = str(distribution) if memo is not None else type(distribution).__name__
        except Exception:  # reprs of batched parameters
            described = type(distribution).__name__
        ok = device_check(constraint, value)
        self.checks.append(CheckRecord(name, self._emit(ok), str(core.support_error(
            name, described)), memo, self.order))

    def sample(self, state: State, name: str, distribution: Distribution,
               sample_shape: OptionalSize = None) -> torch.Tensor:
        self.order += 1
        if isinstance(distribution, Value):
            value = state.get(name, distribution.value)
            if self._validate_parameters:
                value = self._coerce(value, name)
                validate_shape(value, name, distribution, sample_shape)
                self._check_support(name, value, distribution, distribution.support)
            return value

        value = core._lookup_site_value(self.names, state, name)
        if self._validate_parameters:
            value = self._coerce(value, name)
            validate_shape(value, name, distribution, sample_shape)
        self.names.add(name)
        if no_log_prob.get_instance():
            if self._validate_parameters:
                self._check_support(name, value, distribution, cast(Constraint,
                                                                     distribution.support))
            return value

        masked = isinstance(value, torch.masked.MaskedTensor)
        mask = None
        data = value
        if masked:
            data, mask = value._masked_data, value._masked_mask
            if is_batched(data) or is_batched(mask):
                raise NotImplementedError(f"Masked values that depend on the particle axis are not "
                                          f"supported (site '{name}').")

        declared = batch.get_shape()
        family, params = classify(distribution)
        if family == "categorical" and self._validate_parameters and \
                torch.is_floating_point(data):
            # The kernel reads int64 values and checks only the range; fractional or NaN values
            # (integer_interval's `value % 1 == 0`, constraints.py) are checked here (memoised).
            self._check_support(name, value, distribution, cast(Constraint, distribution.support))
        if family == "categorical":
            shape = broadcast_shapes(tuple(data.shape), tuple(distribution.batch_shape))
        elif family != "torch":
            shape = broadcast_shapes(tuple(data.shape), *[tuple(p.shape) for p in params])
        else:
            shape = torch.Size(tuple(data.shape)[:data.dim() - len(distribution.event_shape)])
        shape = torch.Size(shape)
        if declared:
            if masked:
                raise ValueError("Batch dimensions are not supported for masked data.")
            observed = shape[:len(declared)].numel()
            scale = float(declared.numel()) / float(observed) if observed else 0.0
        else:
            scale = 1.0

        if family == "torch":
            self._record_torch_site(name, distribution, value, data, mask, scale)
            return value

        # A deferred `X @ theta` as the location / logits of a Normal / Bernoulli-logits site over
        # shared data becomes a fused linear site; every other deferred parameter is materialised.
        linear = None
        mode = self.deferred
        if mode is not None:
            info = mode.lookup(params[0]) if params else None
            if info is not None and family in ("normal", "bernoulli_logits") and \
                    not is_batched(data) and tuple(shape) == (info.X.shape[0],) and \
                    tuple(data.shape) == tuple(shape) and \
                    all(mode.lookup(p) is None for p in params[1:]):
                linear = info.root or info
            params = [p if (linear is not None and j == 0) else mode.materialize(p)
                      for j, p in enumerate(params)]

        # Value support is checked by the site kernels (fused flag); constraint checks on the
        # parameters as well (MI_FLAG_PARAM), replacing torch's validate_args at construction.
        roles = [self._emit(p) for p in params] + [self._emit(data)]
        record = SiteRecord(name=name, family=family, roles=roles, site_shape=shape, scale=scale,
                            mask=mask, description=type(distribution).__name__, order=self.order)
        if linear is not None:
            record.linear_X = linear.X
            record.linear_theta_index = self._emit(linear.theta)
        self.sites.append(record)
        return value

    def _check_parameters(self, name: str, distribution: Distribution) -> None:
        """
        Device checks of the distribution's ``arg_constraints`` (what ``Distribution.__init__``
        validates on the host in the reference, torch distribution.py:68-80), raised after the
        vmap with torch's message.
        """
        for param, constraint in distribution.arg_constraints.items():
            # as Distribution.__init__'s validation: parameters the distribution was not
            # constructed with (lazy properties, e.g. MultivariateNormal.precision_matrix)
            # are not checked
            if param not in distribution.__dict__ and (
                    not hasattr(type(distribution), param) or
                    isinstance(getattr(type(distribution), param), lazy_property)):
                continue
            try:
                tensor = getattr(distribution, param)
            except Exception:  # lazily defined, unused parametrisations
                continue
            if isinstance(tensor, torch.Tensor):
                ok = check_constraint(constraint, tensor).all()
                self.checks.append(CheckRecord(name, self._emit(ok), (
                    f"Expected parameter {param} of distribution "
                    f"{type(distribution).__name__} for site '{name}' to satisfy the "
                    f"constraint {constraint}, but found invalid values"), order=self.order))

    def _record_torch_site(self, name: str, distribution: Distribution, value: Any,
                           data: torch.Tensor, mask: Optional[torch.Tensor], scale: float) -> None:
        if isinstance(data, torch.Tensor) and data.device.type != "cpu":
            distribution = _on_device(distribution, data.device)
        if self._validate_parameters:
            self._check_support(name, value, distribution, cast(Constraint, distribution.support))
            self._check_parameters(name, distribution)
        if type(distribution) is MultivariateNormal and data.dtype == torch.float32 and \
                data.device.type != "cpu":
            # dense factorisations of float32 covariances are ill-conditioned in practice (the
            # missing-observations example's GP prior): refactorise in float64 on the device;
            # the density itself runs on mi_mvn_tril_forward. This departs from the reference's
            # float32 density on purpose ("MultivariateNormal precision").
            distribution = _mvn_float64(distribution)
            if mvn.enabled(distribution):
                log_prob = mvn.log_prob(distribution, data).float()
            else:
                log_prob = distribution.log_prob(data.double()).float()
        else:
            log_prob = distribution.log_prob(data)
        if mask is not None:
            log_prob = torch.where(mask, log_prob, torch.zeros((), dtype=log_prob.dtype,
                                                               device=log_prob.device))
        total = log_prob.sum() * scale if scale != 1.0 else log_prob.sum()
        self.fallback_outputs.append((name, self._emit(total)))


class TraceCompat(TorchFunctionMode):
    """
    Lets model code written for one draw on the host trace over device particles under vmap:

    * host tensors: the reference's examples keep globals such as ``x = torch.linspace(0, 1, n)``
      and build ``torch.eye(n)`` inside the model. Factory calls default to the particles' device
      (a ``torch.device`` context entered beside this mode), and host tensors (other than 0-d
      ones, which torch already mixes with device tensors) that meet a device tensor in an
      operation are replaced by cached device copies;
    * ``torch.linalg.cholesky`` (MultivariateNormal(loc, covariance_matrix)) checks its input on
      the host, which vmap cannot do per particle: it runs as ``cholesky_ex`` and the
      factorisation status becomes a deferred check with torch's message.

    Used only when a plain trace failed on one of these.
    """
    def __init__(self, device: Optional[torch.device], tracer: "ParticleTracer") -> None:
        super().__init__()
        self.device = device
        self.tracer = tracer

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if self.device is not None:
            leaves = [x for x in tree_flatten((args, kwargs))[0] if isinstance(x, torch.Tensor)]
            if any(x.device.type != "cpu" for x in leaves) and \
                    any(x.device.type == "cpu" and x.dim() > 0 for x in leaves):
                def lift(x):
                    if not isinstance(x, torch.Tensor) or x.device.type != "cpu" or x.dim() == 0:
                        return x
                    return x.to(self.device) if is_batched(x) or x.requires_grad else \
                        device_copy(x, self.device)
                args, kwargs = tree_map(lift, (args, kwargs))
        if func is torch.linalg.cholesky and not kwargs.get("upper", False) and "out" not in kwargs:
            A = args[0] if args else kwargs["input"]
            if mvn.cholesky_supported(A):
                # mi_cholesky: no host synchronisation, capturable (rocSOLVER's potrf is not)
                L, info = mvn.cholesky_ex(A)
            else:
                L, info = torch.linalg.cholesky_ex(*args, **kwargs)
            ok = (info == 0).all()
            self.tracer.checks.append(CheckRecord("cholesky", self.tracer._emit(ok), (
                "linalg.cholesky: The factorization could not be completed because the input is "
                "not positive-definite."), order=self.tracer.order))
            return L
        return func(*args, **kwargs)


def _needs_compat(error: RuntimeError) -> bool:
    text = str(error)
    return "same device" in text or ("device type" in text and "cpu" in text) or \
        "data-dependent control flow" in text


def _mvn_float64(distribution: MultivariateNormal) -> MultivariateNormal:
    """The same MultivariateNormal, constructed in float64 from the parameter it was given."""
    given = next(name for name in ("covariance_matrix", "precision_matrix", "scale_tril")
                 if name in distribution.__dict__)
    return MultivariateNormal(distribution.loc.double(),
                              **{given: getattr(distribution, given).double()},
                              validate_args=False)


@dataclasses.dataclass
class ParticleTrace:
    sites: List[SiteRecord]
    checks: List[Tuple[CheckRecord, torch.Tensor]]
    fallback: List[Tuple[str, torch.Tensor]]
    K: int


_NO_VALIDATE = object()


def trace_particles(model: Callable, samples: Dict[str, torch.Tensor], K: int,
                    validate: bool = True, defer_matmul: Optional[bool] = None,
                    lift_host: bool = False) -> ParticleTrace:
    """
    Run ``condition(model, **samples)`` once under ``vmap`` over the leading (particle) dimension of
    every sample and return the recorded sites with [K, ...] tensors. With ``defer_matmul``,
    ``X @ theta`` predictors of Normal / Bernoulli-logits sites are evaluated inside the site
    kernels instead of by the model (:mod:`mininf_amd.linear`). A model that mixes its own host
    tensors with the device particles, or factorises a matrix, is traced again under
    :class:`TraceCompat`.
    """
    device = next((t.device for t in samples.values() if isinstance(t, torch.Tensor)), None)
    lift = device if device is not None and device.type != "cpu" else None
    if not lift_host:
        try:
            return _trace(model, samples, K, validate, defer_matmul, False, None)
        except RuntimeError as error:
            if not _needs_compat(error):
                raise
    return _trace(model, samples, K, validate, defer_matmul, True, lift)


def _trace(model: Callable, samples: Dict[str, torch.Tensor], K: int, validate: bool,
           defer_matmul: Optional[bool], compat: bool,
           lift: Optional[torch.device]) -> ParticleTrace:
    from .linear import DeferredMatmul

    if defer_matmul is None:
        defer_matmul = os.environ.get("MININF_AMD_DEFER_MATMUL", "1") != "0"
    names = list(samples)
    tracer = ParticleTracer(validate=validate)

    from .guide import _LAZY, flush_draws
    use_mode = defer_matmul or bool(_LAZY)
    if not use_mode:
        flush_draws()   # no mode watches the model's reads of deferred guide draws

    def per_particle(*values):
        mode = DeferredMatmul(K, defer_matmul) if use_mode else None
        tracer.deferred = mode
        with tracer, contextlib.ExitStack() as stack:
            if lift is not None:
                stack.enter_context(torch.device(lift))
            if compat:
                stack.enter_context(TraceCompat(lift, tracer))
            if mode is not None:
                with mode:
                    core.condition(model, **dict(zip(names, values)))()
            else:
                core.condition(model, **dict(zip(names, values)))()
        tracer.deferred = None
        return tuple(tracer.outputs)

    previous = Distribution._validate_args
    Distribution.set_default_validate_args(False)
    try:
        if names:
            outputs = vmap_tensors(per_particle, [samples[name] for name in names])
        else:
            outputs = per_particle()
            outputs = tuple(torch.as_tensor(o).expand(K, *torch.as_tensor(o).shape)
                            for o in outputs)
    finally:
        Distribution.set_default_validate_args(previous)

    for site in tracer.sites:
        site.tensors = [outputs[index] for index in site.roles]
        if site.linear_theta_index >= 0:
            site.linear_theta = outputs[site.linear_theta_index]
    checks = [(check, outputs[check.output]) for check in tracer.checks]
    fallback = [(name, outputs[index]) for name, index in tracer.fallback_outputs]
    return ParticleTrace(sites=tracer.sites, checks=checks, fallback=fallback, K=K)


# ------------------------------------------------------------------------------------------------
# Posterior predictive on the particle machinery (reference core.py:495-584 broadcast_samples,
# SampleTracer core.py:192-204).
# ------------------------------------------------------------------------------------------------
class BroadcastTracer(ParticleTracer):
    """
    The reference's SampleTracer for a model running once under ``vmap`` over the samples' leading
    dimension: a site missing from the state is drawn with the distribution's own ``sample``
    (``vmap(randomness="different")``: independent per sample) and recorded; shapes are checked as
    the reference does; support checks become device outputs raised after the vmap.
    """
    def __init__(self, *args, **kwargs) -> None:
        super().__init__(*args, **kwargs)
        self.index: Optional[torch.Tensor] = None   # the sample number (batched under vmap)
        self.seed = 0
        self.draws = 0

    def sample(self, state: State, name: str, distribution: Distribution,
               sample_shape: OptionalSize = None) -> torch.Tensor:
        sample_shape = _normalize_shape(sample_shape)
        value = state.get(name)
        if value is None:
            if self.index is not None:
                # constants such as Beta(2.0, 5.0)'s are host tensors: draw on the device
                distribution = _on_device(distribution, self.index.device)
            if self.index is not None and predictive.supported(distribution):
                # the HIP samplers, keyed by (seed, this draw's index, sample, element)
                value = predictive.draw(distribution, sample_shape, self.index, self.seed,
                                        self.draws)
            else:
                value = distribution.sample(sample_shape)
            self.draws += 1
            state[name] = value
        if self._validate_parameters:
            value = self._coerce(value, name)
            validate_shape(value, name, distribution, sample_shape)
            # the reference constructs every distribution with validation on, so an invalid
            # parameter raises there (torch distribution.py:68-80) before the draw is used
            self._check_parameters(name, distribution)
            self._check_support(name, value, distribution,
                                cast(Constraint, distribution.support))
        return value


def broadcast_particles(model: Callable, states: Dict[str, torch.Tensor]) -> State:
    """
    ``broadcast_samples`` (reference core.py:548-584) as ONE traced run of ``model`` under
    ``torch.func.vmap`` over the samples' leading dimension instead of a Python loop over samples:
    deterministic values are computed batched, missing sites are drawn batched. Every value of the
    result lives on the samples' device. Returns a :class:`State` of [S, ...] tensors (Python
    numbers as [S] tensors, as the reference's transpose_states makes them).
    """
    names = list(states)
    device = next((v.device for v in states.values() if isinstance(v, torch.Tensor)),
                  torch.device("cpu"))

    lift = device if device.type != "cpu" else None

    S = core._assert_same_batch_size(cast(State, states))
    index = torch.arange(S, device=device)
    # one seed per call from torch's generator: reproducible under torch.manual_seed
    seed = int(torch.randint(0, 2 ** 62, ()).item())

    def run(compat: bool):
        tracer = BroadcastTracer()
        tracer.seed = seed
        keys: List[str] = []

        def per_sample(sample_index, *values):
            tracer.index = sample_index if lift is not None else None
            tracer.draws = 0
            inner = State(dict(zip(names, values)))
            with tracer, inner, contextlib.ExitStack() as stack:
                if compat:
                    if lift is not None:
                        stack.enter_context(torch.device(lift))
                    stack.enter_context(TraceCompat(lift, tracer))
                model()
            keys[:] = list(inner)
            out = [torch.as_tensor(inner[k]) for k in keys]
            return tuple(out) + tuple(tracer.outputs)

        previous = Distribution._validate_args
        Distribution.set_default_validate_args(False)
        try:
            outputs = vmap_tensors(per_sample, [index, *[states[name] for name in names]])
        finally:
            Distribution.set_default_validate_args(previous)
            tracer.index = None
        return tracer, keys, outputs

    try:
        tracer, keys, outputs = run(False)
    except RuntimeError as error:
        if not _needs_compat(error):
            raise
        tracer, keys, outputs = run(True)
    values = outputs[:len(keys)]
    failed = [check for check in tracer.checks
              if not bool(outputs[len(keys) + check.output].all())]
    if failed:
        raise ValueError(failed[0].message)
    for check in tracer.checks:
        if check.memo is not None:
            memo_commit(check.memo)
    return State({k: v.to(device) for k, v in zip(keys, values)})
