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
import gc
import ctypes
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


def register_host_check(check: Callable[[], None]) -> None:
    """
    Called by an operation being captured into a :class:`StepGraph` whose failures surface in
    host-visible memory (the peer all-reduce's error word): the graph calls ``check()`` before
    each replay and in :meth:`StepGraph.check`, so the error is raised at the next host read.
    Outside a capture, a no-op.
    """
    checks = getattr(_STATE, "host_checks", None)
    if checks is not None and check not in checks:
        checks.append(check)


def deferred() -> Optional[list]:
    """
    The collector of deferred validations while a step is being warmed up or captured.
    """
    return getattr(_STATE, "collector", None)


def mirrors_flags() -> bool:
    """
    Whether the step being run copies its sticky validation words to the host: every step except
    the first R - 1 of the R steps one StepGraph replay holds (their words are sticky, so the last
    step's copy carries them; the others skip a host-mapped write at the end of their ELBO
    forward).
    """
    position = getattr(_STATE, "capture_position", None)
    return position is None or position[0] == position[1] - 1


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


def _release_graph_refs(joints: list) -> None:
    """
    After a capture only the validation words (and the sites' names and order, for the messages)
    are read from the joints: drop their loss and the sites' particle tensors, which reach the
    captured step's autograd graph (the guide draws' nodes and the parameters' AccumulateGrad
    nodes, created on the capture stream -- kept alive, a later capture's warm-up on another
    stream warns about them).
    """
    for joint in joints:
        if hasattr(joint, "total"):
            joint.total = None
        for _, _, sites in getattr(joint, "pending", ()):
            for site in sites:
                site.tensors = []
                site.linear_theta = None
                site.linear_X = None


def _check_warmup(collector: list) -> int:
    """Raise a warm-up step's validation errors; the number of its validation words. (A function
    of its own: no loop variable outlives it holding a joint, and with it the step's graph.)"""
    for joint in collector:
        joint.raise_on_violation()
    return sum(joint.flag_count() for joint in collector)


def _detached(out):
    if isinstance(out, torch.Tensor):
        return out.detach()
    if isinstance(out, (tuple, list)):
        return type(out)(_detached(o) for o in out)
    if isinstance(out, dict):
        return {k: _detached(v) for k, v in out.items()}
    return out


class CaptureError(RuntimeError):
    """A training step could not be captured into a hipGraph (see :class:`StepGraph`)."""


def _flush_held_launch() -> None:
    """Enqueue a held step-finishing launch (engine._PendingStep) on the current stream."""
    from . import engine
    engine.flush_pending_step()


def _abandon_capture(cuda_graph: "torch.cuda.CUDAGraph", stream: "torch.cuda.Stream") -> None:
    """
    End a capture that failed part-way: torch's ``capture_end`` (which also hands the graph's
    memory pool back to the caching allocator) when the capture is still valid, then
    ``mi_capture_abandon`` for a capture torch could not end (an invalidated one), so the stream
    is no longer capturing; finally wait for the work queued before the capture.
    """
    from . import _native as nat
    from . import engine
    engine.discard_pending_step()   # a launch held inside the failed capture never runs
    try:
        cuda_graph.capture_end()
    except Exception:   # invalidated: torch raised before ending the capture
        pass
    was = ctypes.c_int(0)
    code = nat.lib().mi_capture_abandon(stream.cuda_stream, ctypes.byref(was))
    if code != 0:   # reported beside the original error, which the caller raises
        import warnings
        warnings.warn(f"mi_capture_abandon could not end the failed capture (hipError_t {code}); "
                      "later GPU work in this process may fail", RuntimeWarning)
        return
    torch.cuda.synchronize()


def _failing_op(error: BaseException) -> str:
    """``file:line (function)`` of the innermost frame of ``error`` outside torch and this package:
    the model code whose operation failed."""
    import os
    import traceback
    skip = (os.path.dirname(torch.__file__), os.path.dirname(os.path.abspath(__file__)))
    frames = [f for f in traceback.extract_tb(error.__traceback__)
              if not f.filename.startswith(skip)]
    if not frames:
        frames = traceback.extract_tb(error.__traceback__)
    if not frames:
        return "at an unknown operation"
    f = frames[-1]
    return f"at {f.filename}:{f.lineno} ({f.name}: {(f.line or '').strip()})"


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
        warmup_step: What the warm-up iterations run (default: ``step``) -- e.g. a whole training
            step when ``step`` is the part of it before a host-issued collective, so the warm-up
            advances the training state exactly as the replays will. ``warmup=0`` skips the
            warm-up (the caller has run the step on this process already).
        capture_error_mode: ``torch.cuda.CUDAGraph.capture_begin``'s mode. ``"thread_local"`` when
            the step holds a collective (RCCL): the process group's watchdog thread polls events
            while the capture runs, which the default ``"global"`` mode refuses.

    Raises:
        CaptureError: the step ran an operation a capturing stream does not permit (for example
            a synchronous host-to-device copy). The capture is abandoned, its partial graph freed
            and the stream left usable; the error names the model line that failed.
    """
    def __init__(self, step: Callable[[], object], warmup: int = 3, repeat: int = 1,
                 capture_error_mode: str = "global",
                 warmup_step: Optional[Callable[[], object]] = None) -> None:
        if repeat < 1:
            raise ValueError("repeat must be a positive integer")
        self.step = step
        self.repeat = repeat
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        if warmup < 0:
            raise ValueError("warmup must be non-negative")
        count = None
        with torch.cuda.stream(side):
            for _ in range(warmup):
                collector: List = []
                with graph_safe(collector), _capture_safe_distributions():
                    (warmup_step or step)()
                _flush_held_launch()
                count = _check_warmup(collector)
                # the joints hold the step's loss: drop them, or the warm-up's autograd graph
                # (its AccumulateGrad nodes on this side stream) stays alive into the capture --
                # a loop variable bound to the last joint did exactly that (the AccumulateGrad
                # stream warning of the first captured backward)
                del collector
        torch.cuda.current_stream().wait_stream(side)
        # Validation results must survive replays the host does not inspect: the step's words are
        # OR-ed into this accumulator by the graph itself (allocated and zeroed outside the capture)
        # unless the step's only flags already are never-zeroed words (EvidenceLowerBoundLoss in
        # graph mode), which then serve as the accumulator without an extra node.
        self._accumulator = torch.zeros(max(1, count or 0), dtype=torch.int64,
                                        device=torch.cuda.current_device())
        torch.cuda.synchronize()

        self.graph = torch.cuda.CUDAGraph()
        self._joints: List = []
        self._flags_device: Optional[torch.Tensor] = None
        mirror = None
        capture_stream = torch.cuda.Stream()
        capture_stream.wait_stream(torch.cuda.current_stream())
        # Garbage from earlier steps or graphs (pinned buffers, events, graph executables held in
        # reference cycles) is freed now: a collection during the capture would run their
        # finalizers on a capturing stream, which aborts the process. The collector stays off until
        # the capture ends (torch.cuda.graph collects before its capture too).
        gc.collect()
        gc_was_enabled = gc.isenabled()
        gc.disable()
        from . import particles
        self._host_checks: List[Callable[[], None]] = []
        with torch.cuda.stream(capture_stream):
            self.graph.capture_begin(capture_error_mode=capture_error_mode)
            _STATE.host_checks = self._host_checks
            try:
                # the cached device copies of host constants the captured step reads live as long
                # as the graph (particles.device_copy's cache may evict them)
                with graph_safe(self._joints), _capture_safe_distributions(), \
                        particles.pin_device_copies() as self._pinned:
                    try:
                        for r in range(repeat):
                            _STATE.capture_position = (r, repeat)
                            # detached: holding the captured step's autograd graph would keep its
                            # AccumulateGrad nodes (and their capture stream) alive past the
                            # capture
                            self.output = _detached(step())
                    finally:
                        _STATE.capture_position = None
                    _flush_held_launch()   # (a step without an optimizer leaves it held)
                    mirror = self._record_validation(count)
                self.graph.capture_end()
            except BaseException as error:
                self._joints = []
                _abandon_capture(self.graph, capture_stream)
                self.graph = None
                raise CaptureError("the step cannot be captured into a hipGraph, "
                                   f"{_failing_op(error)}: {type(error).__name__}: {error}") \
                    from error
            finally:
                _STATE.host_checks = None
                if gc_was_enabled:
                    gc.enable()
        torch.cuda.current_stream().wait_stream(capture_stream)
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

    def _record_validation(self, count: int) -> Optional[torch.Tensor]:
        """
        Inside the capture: route the captured steps' validation words into words no replay zeroes
        (``self._flags_device``); returns the pinned mirror the ELBO forward writes, if any.
        """
        repeat = self.repeat
        if len(self._joints) % repeat:
            raise RuntimeError("the captured steps recorded different validations")
        per_step = len(self._joints) // repeat
        # one step's validations: what the host checks (every captured step ORs into the same
        # words)
        steps = [self._joints[r * per_step:(r + 1) * per_step] for r in range(repeat)]
        mirror = None
        sticky = [j[0] for j in steps] if per_step == 1 else []
        if sticky and all(j.sticky and j.flag_vector() is not None and
                          j.flag_vector() is j.flags and
                          j.flags.data_ptr() == sticky[0].flags.data_ptr() for j in sticky):
            self._flags_device = sticky[0].flags
            self._accumulator = None
            mirror = sticky[-1].mirror   # (only the last step writes it: mirrors_flags)
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
                if count is None:   # the accumulator must exist (zeroed) before the capture
                    raise RuntimeError("a step with non-sticky validation words needs at least "
                                       "one warm-up iteration")
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
        _release_graph_refs(self._joints)
        return mirror

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
        if block:
            self._done.synchronize()
        for check in self._host_checks:   # (host-visible words: read without a wait)
            check()
        if not self._pending:
            return
        if not block and not self._done.query():
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
