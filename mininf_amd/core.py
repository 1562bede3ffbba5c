"""
Probabilistic-program core: singleton contexts, the parameter tape (:class:`State`), tracers and the
``sample`` / ``condition`` / ``value`` / ``batch`` / ``no_log_prob`` primitives.

This is the host-side mirror of the reference's ``mininf/core.py``. The tracer plugin point
(:class:`TracerMixin`, reference ``core.py:128-140``) is what the MI355X ELBO engine plugs into: the
:class:`mininf_amd.particles.ParticleTracer` records the model's sites for the HIP site kernels
instead of evaluating ``Distribution.log_prob`` one site at a time.

The :class:`LogProbTracer` here keeps the reference's per-site dictionary semantics
(``log_prob[name] == (log_prob_tensor, batch_shape)``, reference ``core.py:207-277``) and evaluates
``torch.distributions`` on whatever device the values live on; it is the reference API, not the
hot path (see ``mininf_amd.nn.EvidenceLowerBoundLoss`` for that).
"""
from __future__ import annotations

import functools as ft
import logging
from typing import Any, Callable, cast, Dict, List, Literal, overload, Tuple, Type, TypeVar

import torch
from torch.distributions import Distribution
from torch.distributions.constraints import Constraint
from typing_extensions import Self

from .util import _format_dict_compact, _normalize_shape, check_constraint, \
    get_masked_data_with_dense_grad, maybe_as_tensor, OptionalSize, TensorDict


S = TypeVar("S", bound="SingletonContextMixin")
# the reference's logger name (mininf/core.py:16), so existing logging configuration applies
LOGGER = logging.getLogger("mininf.core")


class SingletonContextMixin:
    """
    Context manager base class of which at most one instance per :attr:`SINGLETON_KEY` can be active
    at any time (reference ``core.py:19-83``). Contexts are process-global and not re-entrant.
    """
    INSTANCES: Dict[str, "SingletonContextMixin"] = {}
    SINGLETON_KEY: str | None = None

    @classmethod
    def _assert_singleton_key(cls) -> str:
        key = cls.SINGLETON_KEY
        if not key:
            raise RuntimeError("Your class must define a singleton key.")
        return key

    def __enter__(self) -> Self:
        key = self._assert_singleton_key()
        current = self.INSTANCES.get(key)
        if current is self:
            raise RuntimeError(f"Cannot reactivate {self} because it is already active.")
        if current is not None:
            raise RuntimeError(f"Cannot activate {self} with singleton key '{key}'; {current} is "
                               "already active.")
        self.INSTANCES[key] = self
        LOGGER.info("Activated %s as context for singleton key '%s'.", self, key)
        return self

    def __exit__(self, *_) -> None:
        key = self._assert_singleton_key()
        current = self.INSTANCES.get(key)
        if current is None:
            raise RuntimeError(f"Cannot deactivate {self} with singleton key '{key}'; no context "
                               "is active.")
        if current is not self:
            raise RuntimeError(f"Cannot deactivate {self} with singleton key '{key}'; {current} is "
                               "active.")
        del self.INSTANCES[key]
        LOGGER.info("Deactivated %s as context for singleton key '%s'.", self, key)

    @overload
    @classmethod
    def get_instance(cls: Type[S], strict: Literal[True] = True) -> S: ...

    @overload
    @classmethod
    def get_instance(cls: Type[S], strict: Literal[False] = False) -> S | None: ...

    @classmethod
    def get_instance(cls: Type[S], strict: bool = False) -> S | None:
        """
        Return the active context of this class's singleton group (or :code:`None`).

        Args:
            strict: Raise a :class:`KeyError` if no context is active.
        """
        key = cls._assert_singleton_key()
        current = cls.INSTANCES.get(key)
        if current is None:
            if strict:
                raise KeyError(f"No '{key}' context is active.")
            return None
        if not isinstance(current, cls):
            raise TypeError(f"Active context {current} is not an instance of {cls}.")
        return current


class State(Dict[str, Any], SingletonContextMixin):
    """
    Tape of named parameters recorded by ``sample`` / ``condition`` (reference ``core.py:86-125``).

    Example:

        >>> from mininf_amd import sample, State
        >>> from torch.distributions import Normal
        >>> with State() as state:
        ...     x1 = sample("x", Normal(0, 1))
        >>> with state:
        ...     x2 = sample("x", Normal(0, 1))
        >>> x1 is x2
        True
    """
    SINGLETON_KEY = "state"

    def __repr__(self) -> str:
        return _format_dict_compact(self)

    def subset(self, *names: str) -> "State":
        """
        New :class:`State` holding only the given parameters (same tensor objects).
        """
        return State({name: self[name] for name in names})


def _expected_shape_message(name: str, batch_shape: torch.Size, shape: torch.Size,
                            actual: Tuple[int, ...]) -> str:
    parts = [f"{size}*" for size in batch_shape] + [str(size) for size in shape[len(batch_shape):]]
    text = ", ".join(parts) + ("," if len(parts) == 1 else "")
    return f"Expected shape ({text}) for parameter '{name}' but got {actual}."


def validate_shape(value: torch.Tensor, name: str, distribution: Distribution,
                   sample_shape: OptionalSize) -> None:
    """
    Shape half of the reference's parameter validation (``core.py:152-183``): the declared batch
    rank may not exceed the actual batch rank, and ``value.shape`` must equal
    ``sample_shape + batch_shape + event_shape`` except along batched (minibatch) dimensions, where a
    larger-than-declared size only logs a warning.
    """
    declared = batch.get_shape()
    sample_shape = _normalize_shape(sample_shape)
    actual_batch_shape = sample_shape + distribution.batch_shape
    if len(declared) > len(actual_batch_shape):
        raise ValueError(f"Declared batch shape {declared} for parameter '{name}' has more "
                         f"dimensions than the actual batch shape {actual_batch_shape}.")

    expected = sample_shape + distribution.batch_shape + distribution.event_shape
    actual = value.shape
    if len(expected) != len(actual):
        raise ValueError(_expected_shape_message(name, declared, expected, tuple(actual)))
    for dim, (size, actual_size) in enumerate(zip(expected, actual)):
        batched = dim < len(declared)
        if actual_size != size and not batched:
            raise ValueError(_expected_shape_message(name, declared, expected, tuple(actual)))
        if actual_size > size:
            LOGGER.warning("Actual batch shape %s for parameter '%s' exceeds expected batch shape "
                           "%s along dimension %d.", actual_batch_shape, name, declared, dim)


def support_error(name: str, distribution: Any) -> ValueError:
    return ValueError(f"Parameter '{name}' is not in the support of {distribution}.")


class TracerMixin(SingletonContextMixin):
    """
    Plugin point for everything that executes a model (reference ``core.py:128-189``). A tracer
    receives every ``sample`` statement through :meth:`sample`.
    """
    SINGLETON_KEY = "tracer"

    def __init__(self, *args, _validate_parameters: bool = True, **kwargs) -> None:
        super().__init__(*args, **kwargs)
        self._validate_parameters = _validate_parameters

    def sample(self, state: State, name: str, distribution: Distribution,
               sample_shape: OptionalSize = None) -> torch.Tensor:
        raise NotImplementedError

    def _coerce(self, value: Any, name: str) -> torch.Tensor:
        value = maybe_as_tensor(value)
        if not isinstance(value, torch.Tensor):
            raise TypeError(f"Expected a tensor for parameter '{name}' but got {type(value)}.")
        return value

    def _assert_valid_parameter(self, value: torch.Tensor | None, name: str,
                                distribution: Distribution, sample_shape: OptionalSize) \
            -> torch.Tensor | None:
        """
        Validate type, shape and support of a parameter (reference ``core.py:142-189``).
        """
        if not self._validate_parameters:
            return value
        value = self._coerce(value, name)
        validate_shape(value, name, distribution, sample_shape)
        support = cast(Constraint, distribution.support)
        if not check_constraint(support, value).all():
            raise support_error(name, distribution)
        return value


class SampleTracer(TracerMixin):
    """
    Default tracer: draw missing parameters from their distributions and record them in the state
    (reference ``core.py:192-204``).
    """
    def sample(self, state: State, name: str, distribution: Distribution,
               sample_shape: OptionalSize = None) -> torch.Tensor:
        sample_shape = _normalize_shape(sample_shape)
        value = state.get(name)
        if value is None:
            value = distribution.sample(sample_shape)
            state[name] = value
        self._assert_valid_parameter(value, name, distribution, sample_shape)
        return value


def _lookup_site_value(seen: Any, state: State, name: str) -> Any:
    """
    Shared bookkeeping of log-probability tracers: duplicate sites and missing values raise the
    reference's errors (``core.py:217-223``).
    """
    if name in seen:
        raise RuntimeError(f"Log probability has already been evaluated for '{name}'. Did you "
                           "call `sample` twice with the same variable name?")
    value = state.get(name)
    if value is None:
        raise ValueError(f"Cannot evaluate log probability; variable '{name}' is missing. Did "
                         "you forget to condition on observed data?")
    return value


class LogProbTracer(TracerMixin, Dict[str, Tuple[torch.Tensor, torch.Size]]):
    """
    Evaluate per-site log probabilities of a state under the model with ``torch.distributions``
    (reference ``core.py:207-277``). ``tracer[name]`` is ``(elementwise log_prob, batch_shape)``.
    """
    def sample(self, state: State, name: str, distribution: Distribution,
               sample_shape: OptionalSize = None) -> torch.Tensor:
        if isinstance(distribution, Value):
            value = state.get(name, distribution.value)
            self._assert_valid_parameter(value, name, distribution, sample_shape)
            return value
        value = _lookup_site_value(self, state, name)
        self._assert_valid_parameter(value, name, distribution, sample_shape)
        if no_log_prob.get_instance():
            return value

        if isinstance(value, torch.masked.MaskedTensor):
            support = cast(Constraint, distribution.support)
            if distribution._validate_args and not check_constraint(support, value).all():
                raise ValueError(f"Sample {value} is not in the support {distribution.support} of "
                                 f"distribution {distribution}.")
            validate_args = distribution._validate_args
            distribution._validate_args = False
            try:
                dense = distribution.log_prob(get_masked_data_with_dense_grad(value))
            finally:
                distribution._validate_args = validate_args
            log_prob = torch.masked.as_masked_tensor(dense, value.get_mask())
        else:
            log_prob = distribution.log_prob(value)

        self[name] = (log_prob, batch.get_shape())
        return value

    @property
    def total(self) -> torch.Tensor:
        """
        Sum of all site contributions in insertion order (``0`` if there are no sites).
        """
        return cast(torch.Tensor, sum(self.contribution(name) for name in self))

    def contribution(self, name: str) -> torch.Tensor:
        """
        Contribution of one site: the sum of its log probabilities, scaled by
        ``declared batch size / observed batch size`` for minibatched sites and restricted to the
        mask for masked values (reference ``core.py:251-273``).
        """
        log_prob, batch_shape = self[name]
        if isinstance(log_prob, torch.masked.MaskedTensor):
            if batch_shape:
                raise ValueError("Batch dimensions are not supported for masked data.")
            return get_masked_data_with_dense_grad(log_prob)[log_prob.get_mask()].sum()
        if not batch_shape:
            return log_prob.sum()
        observed = log_prob.shape[:len(batch_shape)].numel()
        return log_prob.sum() * batch_shape.numel() / observed

    def __repr__(self) -> str:
        return _format_dict_compact({key: item[0] for key, item in self.items()}, id(self),
                                    self.__class__.__name__)


def with_active_state(func: Callable) -> Callable:
    """
    Decorator passing the active :class:`State` (created on the fly if none is active) as the first
    argument (reference ``core.py:280-297``).
    """
    @ft.wraps(func)
    def _wrapper(*args, **kwargs) -> Any:
        state = State.get_instance()
        if state is not None:
            return func(state, *args, **kwargs)
        with State() as state:
            return func(state, *args, **kwargs)

    return _wrapper


@with_active_state
def sample(state: State, name: str, distribution: Distribution, sample_shape: OptionalSize = None) \
        -> torch.Tensor:
    """
    Draw (or look up) the random variable ``name`` with the given distribution.

    Args:
        name: Name of the random variable.
        distribution: Its distribution.
        sample_shape: Shape of iid draws; the result has shape
            ``sample_shape + distribution.batch_shape + distribution.event_shape``.

    Example:

        >>> from mininf_amd import sample
        >>> from torch.distributions import Normal
        >>> sample("x", Normal(0, 1), 3).shape
        torch.Size([3])
    """
    tracer = TracerMixin.get_instance()
    if tracer is None:
        tracer = SampleTracer()
    return tracer.sample(state, name, distribution, sample_shape)


def condition(model: Callable, values: TensorDict | None = None, *, _strict: bool = True,
              **kwargs: torch.Tensor) -> Callable:
    """
    Condition a model on values (reference ``core.py:331-387``). Keyword arguments take precedence
    over the ``values`` dictionary; with ``_strict`` a parameter may be conditioned at most once,
    otherwise the outermost ``condition`` wins.

    Example:

        >>> from mininf_amd import condition, sample
        >>> from torch.distributions import Normal
        >>> condition(lambda: sample("x", Normal(0, 1)), x=0.3)()
        tensor(0.3000)
    """
    merged = dict(values or {})
    merged.update(kwargs)
    merged ={key: cast(torch.Tensor, maybe_as_tensor(item)) for key, item in merged.items()}

    @with_active_state
    @ft.wraps(model)
    def _wrapper(state: State, *args, **inner_kwargs) -> Any:
        if _strict:
            conflict = set(state) & set(merged)
            if conflict:
                raise ValueError(f"Cannot update state {state} because it already has parameters "
                                 f"{conflict}.")
        state.update(merged)
        return model(*args, **inner_kwargs)

    return _wrapper


class Value(Distribution):
    """
    Pseudo-distribution of a constant or deterministic quantity (reference ``core.py:390-448``).
    ``sample`` returns the default value; ``log_prob`` is deliberately not implemented, so value
    sites never contribute to the log joint.

    Args:
        value: Default value.
        support: Support of the value (real line by default).
        validate_args: Passed to :class:`torch.distributions.Distribution`.
    """
    arg_constraints: Dict[str, Constraint] = {}

    def __init__(self, value: torch.Tensor | None = None, support: Constraint | None = None,
                 validate_args: bool | None = None):
        value = maybe_as_tensor(value)
        super().__init__(torch.Size(), torch.Size(), validate_args)
        self.value = value
        self._support = support or torch.distributions.constraints.real
        # A default computed from particles inside the vmapped trace (e.g. `X @ theta`) cannot be
        # checked eagerly; the particle tracers check it with the site's support instead.
        if value is not None and not torch._C._functorch.is_batchedtensor(value) and \
                not check_constraint(self._support, value).all():
            raise ValueError(f"Default value is not in the specified support {self._support}.")

    @property
    def support(self) -> Constraint:
        return self._support

    def sample(self, sample_shape=torch.Size()):
        if self.value is None:
            raise ValueError("No default value given. Did you mean to specify one value by "
                             "conditioning?")
        return self.value

    def log_prob(self, value):
        raise NotImplementedError("Values do not implement `log_prob` by design.")

    def __repr__(self) -> str:
        fields = [f"{key}={item}" for key, item in
                  (("value", self.value), ("support", self.support)) if item is not None]
        return f"Value({', '.join(fields)})"


def value(name: str, value: torch.Tensor | None = None, shape: torch.Size | None = None,
          support: Constraint | None = None, validate_args: bool | None = None) -> torch.Tensor:
    """
    Declare a deterministic variable or constant (reference ``core.py:451-492``). Without a default
    value, ``shape`` declares the expected shape and the value must be supplied by ``condition``.

    Example:

        >>> from mininf_amd import condition, value
        >>> condition(lambda: value("n", 3), n=5)()
        tensor(5)
    """
    if shape is None and value is not None:
        value = torch.as_tensor(value)
        shape = value.shape
    return sample(name, Value(value, support, validate_args), shape)


def _assert_same_batch_size(state: State) -> int:
    """
    Leading-dimension size shared by all entries of ``state`` (reference ``core.py:495-510``).
    """
    if not state:
        raise ValueError("Cannot check batch sizes because the state is empty.")
    groups: Dict[int, List[str]] = {}
    for key, item in state.items():
        groups.setdefault(item.shape[0], []).append(key)
    if len(groups) != 1:
        raise ValueError(f"Inconsistent batch sizes: {groups}")
    return next(iter(groups))


@overload
def transpose_states(states: State) -> List[State]: ...


@overload
def transpose_states(states: List[State]) -> State: ...


def transpose_states(states: State | List[State]) -> State | List[State]:
    """
    Convert a state of batched tensors into a list of unbatched states or vice versa (reference
    ``core.py:513-545``).
    """
    if isinstance(states, dict):
        size = _assert_same_batch_size(cast(State, states))
        return [State({key: item[index] for key, item in states.items()}) for index in range(size)]
    columns: Dict[str, List[torch.Tensor]] = {}
    for state in states:
        for key, item in state.items():
            columns.setdefault(key, []).append(cast(torch.Tensor, maybe_as_tensor(item))[None])
    return State({key: torch.concatenate(parts) for key, parts in columns.items()})


def broadcast_samples(model: Callable, states: State | None = None, **params: torch.Tensor) \
        -> State:
    """
    Run ``model`` once per leading-dimension entry of the given samples and stack the resulting
    states (reference ``core.py:548-584``). Samples on a ROCm device are broadcast in ONE run of the
    model under ``torch.func.vmap`` (:func:`mininf_amd.particles.broadcast_particles`); host
    samples take the reference's per-sample loop.

    Example:

        >>> import torch
        >>> from mininf_amd import broadcast_samples, sample
        >>> def model():
        ...     sample("x", torch.distributions.Normal(0, 1), [5])
        >>> broadcast_samples(model, x=torch.randn(7, 5))["x"].shape
        torch.Size([7, 5])
    """
    states = states if states is not None else State()
    states.update(params)
    if states and all(isinstance(v, torch.Tensor) and v.device.type != "cpu"
                      for v in states.values()):
        # device samples: one vmapped run of the model over the samples (particle machinery)
        from .particles import broadcast_particles
        return broadcast_particles(model, states)
    finished = []
    for state in transpose_states(states):
        with state:
            model()
        finished.append(state)
    return transpose_states(finished)


class batch(SingletonContextMixin):
    """
    Declare the full size of leading (minibatch) dimensions: site contributions are scaled by
    ``declared size / observed size`` (reference ``core.py:587-622``).
    """
    SINGLETON_KEY = "batch"

    def __init__(self, shape: torch.Size | int) -> None:
        self.shape = _normalize_shape(shape)

    @classmethod
    def get_shape(cls) -> torch.Size:
        """
        Declared batch shape of the active context (empty if none is active).
        """
        active = cls.get_instance()
        return torch.Size() if active is None else active.shape


class no_log_prob(SingletonContextMixin):
    """
    Skip log-probability evaluation of the enclosed sample statements (reference
    ``core.py:625-642``). Parameters are still validated.
    """
    SINGLETON_KEY = "no_log_prob"
