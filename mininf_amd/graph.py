"""
HIP-graph capture of a whole ELBO training step.

Every kernel of a step -- guide sampling, the site kernels, the finalize reductions, torch's own
elementwise ops for the guide transforms and entropy, autograd's backward and the optimizer update
-- is recorded once into a ``torch.cuda.CUDAGraph`` (a hipGraph on ROCm) and replayed, so a step
costs one graph launch instead of ~100 Python-dispatched kernel launches. This is the MI355X
substitute for a tracing compiler: the model is still traced by running its unchanged Python code
(during warm-up and capture); replays re-execute the recorded device work on the same buffers.

What makes the ELBO capturable:

* the guide generator reads its step counter from device memory (``mi_*_rsample`` ``step_device``),
  and the loss increments that word on the device, so every replay draws fresh particles;
* inside :func:`graph_safe` the engine does not synchronise to raise validation errors: the
  per-site flag words are accumulated on the device (never cleared by a replay, so a violation in
  any replay persists), copied to pinned host memory by each replay (the ELBO forward writes them
  there itself when it can, else one D2H copy follows the replay), and checked once that
  replay has finished (:meth:`StepGraph.check`, or non-blockingly before the next replay) --
  errors are raised with the reference's messages, a few steps late at most, and never lost;
* ``torch.distributions`` argument validation (a host sync per check) is off inside the captured
  region; the site kernels' MI_FLAG_PARAM checks cover the model's parameters;
* while capturing, ``torch.distributions``' ``broadcast_all`` turns Python numbers into device
  tensors with a fill kernel instead of a host-to-device copy (which a capturing stream forbids).

Conditioned data must keep its storage across replays (the graph records addresses), and the
optimizer must be created with ``capturable=True`` when its step is part of the graph.
"""
from __future__ import annotations

import contextlib
import sys
import threading
from numbers import Number
from typing import Callable, List, Optional

import torch
from torch.distributions import Distribution
from torch.distributions import utils as distribution_utils
from torch.overrides import is_tensor_like

_STATE = threading.local()
_ORIGINAL_BROADCAST_ALL = distribution_utils.broadcast_all


# Device scalars for the Python numbers of distributions built inside warm-up / captured steps,
# created once by a warm-up step (a real fill) and reused by the capture, so the captured step has
# no fill node per number; CONSTANT_VALUES maps their addresses to the numbers, so the site kernels
# take them as compile-time constants (mininf_amd.engine._to_device).
_CONSTANTS: dict = {}
CONSTANT_VALUES: dict = {}


def _device_constant(value: Number, options: dict) -> torch.Tensor:
    device = options.get("device")
    if device is None or torch.device(device).type == "cpu":
        return torch.full((), value, **options)
    key = (float(value), options["dtype"], str(device))
    hit = _CONSTANTS.get(key)
    if hit is not None:
        return hit
    out = torch.full((), value, **options)
    if not torch.cuda.is_current_stream_capturing():   # a recorded fill has not run yet
        _CONSTANTS[key] = out
        CONSTANT_VALUES[out.data_ptr()] = float(value)
    return out


def _capture_safe_broadcast_all(*values):
    """
    torch.distributions.utils.broadcast_all with Python numbers materialised by a device fill
    (``torch.full``, cached across steps) instead of a host-to-device copy
    (``torch.tensor(v, device=...)``), which a capturing stream does not permit -- e.g. the ``1``
    of ``Normal(X @ theta, 1)``.
    """
    if not all(is_tensor_like(v) or isinstance(v, Number) for v in values):
        return _ORIGINAL_BROADCAST_ALL(*values)
    if all(is_tensor_like(v) for v in values):
        return torch.broadcast_tensors(*values)
    options = dict(dtype=torch.get_default_dtype())
    for value in values:
        if isinstance(value, torch.Tensor):
            options = dict(dtype=value.dtype, device=value.device)
            break
    return torch.broadcast_tensors(*[v if is_tensor_like(v) else _device_constant(v, options)
                                     for v in values])


@contextlib.contextmanager
def _capture_safe_distributions():
    patched = []
    for name, module in list(sys.modules.items()):
        if name.startswith("torch.distributions") and \
                getattr(module, "broadcast_all", None) is _ORIGINAL_BROADCAST_ALL:
            module.broadcast_all = _capture_safe_broadcast_all
            patched.append(module)
    try:
        yield
    finally:
        for module in patched:
            module.broadcast_all = _ORIGINAL_BROADCAST_ALL


def deferred() -> Optional[list]:
    """
    The collector of deferred validations while a step is being warmed up or captured.
    """
    return getattr(_STATE, "collector", None)


@contextlib.contextmanager
def graph_safe(collector: list):
    """
    Run model code without host synchronisation: validation results are appended to `collector`
    instead of being checked, and torch.distributions argument validation is disabled.
    """
    previous = Distribution._validate_args
    Distribution.set_default_validate_args(False)
    _STATE.collector = collector
    try:
        yield
    finally:
        _STATE.collector = None
        Distribution.set_default_validate_args(previous)


class StepGraph:
    """
    Capture ``step()`` (any callable running one training step on the current device) and replay
    it. ``__call__`` returns the captured step's output tensors (updated in place by each replay).

    Args:
        step: The training step. It should call ``optimizer.zero_grad(set_to_none=True)`` first so
            that gradient buffers are allocated inside the graph's memory pool.
        warmup: Eager warm-up iterations on a side stream before capture (compiles the specialised
            site programs, fills caches, initialises library handles).
        repeat: Consecutive steps captured into the one graph (each replay runs ``repeat`` full
            steps). Every graph launch costs the device ~13 us of idle time between the last
            kernel of one replay and the first of the next on MI355X; a launch-bound step (a few
            dozen microseconds of kernels) amortises it over ``repeat`` steps. The step must keep
            its per-step state on the device (generator counter, minibatch counter, optimizer
            step counts), as the engine's own steps do.
    """
    def __init__(self, step: Callable[[], object], warmup: int = 3, repeat: int = 1) -> None:
        if repeat < 1:
            raise ValueError("repeat must be a positive integer")
        self.step = step
        self.repeat = repeat
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        count = 0
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                collector: List = []
                with graph_safe(collector), _capture_safe_distributions():
                    step()
                for joint in collector:
                    joint.raise_on_violation()
                count = sum(joint.flag_count() for joint in collector)
        torch.cuda.current_stream().wait_stream(side)
        # Validation results must survive replays the host does not inspect: the step's words are
        # OR-ed into this accumulator by the graph itself (allocated and zeroed outside the capture)
        # unless the step's only flags already are never-zeroed words (EvidenceLowerBoundLoss in
        # graph mode), which then serve as the accumulator without an extra node.
        self._accumulator = torch.zeros(max(1, count), dtype=torch.int64,
                                        device=torch.cuda.current_device())
        torch.cuda.synchronize()

        self.graph = torch.cuda.CUDAGraph()
        self._joints: List = []
        with graph_safe(self._joints), _capture_safe_distributions(), \
                torch.cuda.graph(self.graph):
            for _ in range(repeat):
                self.output = step()
            if len(self._joints) % repeat:
                raise RuntimeError("the captured steps recorded different validations")
            per_step = len(self._joints) // repeat
            # one step's validations: what the host checks (every captured step ORs into the
            # same words)
            steps = [self._joints[r * per_step:(r + 1) * per_step] for r in range(repeat)]
            mirror = None
            sticky = [j[0] for j in steps] if per_step == 1 else []
            if sticky and all(j.sticky and j.flag_vector() is not None and
                              j.flag_vector() is j.flags and
                              j.flags.data_ptr() == sticky[0].flags.data_ptr() for j in sticky):
                self._flags_device = sticky[0].flags
                self._accumulator = None
                mirror = sticky[0].mirror
            else:
                any_flags = False
                for joints in steps:
                    flags = [joint.flag_vector() for joint in joints]
                    flags = [f for f in flags if f is not None]
                    if not flags:
                        continue
                    any_flags = True
                    vector = torch.cat([f.to(torch.int64) for f in flags]) if len(flags) > 1 \
                        else flags[0]
                    if vector.numel() != count:
                        raise RuntimeError(f"the captured step has {vector.numel()} validation "
                                           f"words, its warm-up steps {count}")
                    self._accumulator.bitwise_or_(vector)
                if any_flags:
                    self._flags_device = self._accumulator
                else:
                    self._flags_device = None
                    self._accumulator = None
            self._joints = steps[0]
        # The ELBO forward of a sticky step writes its words to pinned host memory itself (the
        # mirror); otherwise the copy is enqueued after each replay (one small asynchronous D2H
        # copy: pinned host memory cannot be allocated while capturing).
        self._flags_host = None
        self._mirrored = mirror is not None and self._flags_device is not None and \
            mirror.numel() == self._flags_device.numel()
        if self._mirrored:
            self._flags_host = mirror
        elif self._flags_device is not None:
            self._flags_host = torch.empty(self._flags_device.shape, dtype=self._flags_device.dtype,
                                           pin_memory=True)
        self._done = torch.cuda.Event()
        self._pending = False

    def __call__(self):
        self._check(block=False)
        self.graph.replay()
        if self._flags_host is not None and not self._mirrored:
            self._flags_host.copy_(self._flags_device, non_blocking=True)
        self._done.record()
        self._pending = self._flags_device is not None
        return self.output

    def check(self) -> None:
        """
        Wait for the last replay and raise if it found a validation error.
        """
        self._check(block=True)

    def _check(self, block: bool) -> None:
        if not self._pending:
            return
        if block:
            self._done.synchronize()
        elif not self._done.query():
            return
        self._pending = False
        values = self._flags_host.tolist()
        if any(values):   # raising: clear the accumulated words for a caller that carries on
            self._done.synchronize()
            self._flags_device.zero_()
            self._flags_host.zero_()
        cursor = 0
        for joint in self._joints:
            count = joint.flag_count()
            joint.raise_from(values[cursor:cursor + count])
            cursor += count
