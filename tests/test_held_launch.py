"""
The held step-finishing launch (engine._PendingStep, host logic only -- no GPU): a fused ELBO's
finishing launch is enqueued at its first consumer, or joined by the Adam step over its
gradients. Pinned here with a stand-in launch that writes host tensors:

* metadata queries on the loss / a held gradient do not enqueue it, data uses do (once);
* a held ``param.grad`` is a plain tensor again after the launch;
* ``attach_optimizer`` hands the descriptor to the launch only for gradients it writes and steps
  within the fused limit; every native launch (``_native.stream_handle``'s hook) flushes first;
* MININF_AMD_DEFER_STEP=0 disables holding.
"""
import ctypes

import pytest
import torch

from mininf_amd import _native as nat
from mininf_amd import engine, nn


class _Launch:
    def __init__(self, out):
        self.out = out
        self.calls = []

    def __call__(self, adam):
        self.calls.append(adam)
        for t in self.out:
            t.fill_(7.0)
        return 0


@pytest.fixture(autouse=True)
def _clean():
    engine.discard_pending_step()
    yield
    engine.discard_pending_step()


def _hold(out, grads=()):
    launch = _Launch(out)
    assert engine._defer_step(launch, "stand-in", [list(grads)], tuple(out))
    return launch


def test_metadata_does_not_flush_data_does():
    g = torch.zeros(4)
    launch = _hold([g], [g])
    held = engine.pending_step().hold(torch.zeros(4, requires_grad=True), g)
    assert isinstance(held, engine.PendingGrad)
    _ = (held.shape, held.dtype, held.device, held.is_sparse, held.dim(), held.numel(),
         held.is_contiguous(), held.stride(), held.requires_grad)
    assert nat.ptr(held) == g.data_ptr()   # the package's own descriptor reads: no flush
    assert launch.calls == []
    assert torch.equal(held.clone(), torch.full((4,), 7.0))
    assert launch.calls == [None]
    held.sum()
    assert launch.calls == [None]   # once


def test_raw_address_read_by_user_code_flushes():
    """data_ptr() outside the package (ctypes, a DDP-like hook, CuPy) is a data use the stream
    cannot see: the held launch is enqueued first."""
    g = torch.zeros(4)
    launch = _hold([g], [g])
    held = engine.pending_step().hold(torch.zeros(4, requires_grad=True), g)
    assert held.data_ptr() == g.data_ptr()
    assert launch.calls == [None]


def test_cuda_array_interface_flushes():
    g = torch.zeros(4)
    launch = _hold([g], [g])
    held = engine.pending_step().hold(torch.zeros(4, requires_grad=True), g)
    with pytest.raises((TypeError, AttributeError, RuntimeError)):
        held.__cuda_array_interface__   # (a CPU tensor here: torch refuses after the flush)
    assert launch.calls == [None]


def test_loss_class_flushes_on_float():
    loss = torch.zeros(())
    launch = _hold([loss])
    loss.__class__ = nn._Loss
    assert loss.dim() == 0 and launch.calls == []
    assert float(loss) == 7.0 and launch.calls == [None]
    assert "tensor(" in repr(loss)


def test_held_grad_is_plain_after_the_launch():
    p = torch.zeros(3, requires_grad=True)
    g = torch.zeros(3)
    launch = _hold([g], [g])
    p.grad = engine.pending_step().hold(p, g)
    assert type(p.grad) is engine.PendingGrad
    engine.flush_pending_step()
    assert launch.calls == [None]
    assert type(p.grad) is torch.Tensor and torch.equal(p.grad, torch.full((3,), 7.0))


def _adam(numel, grad):
    desc = nat.Adam()
    desc.num = 1
    desc.tensors[0].numel = numel
    desc.tensors[0].grad = grad.data_ptr()
    return desc


def test_attach_optimizer_joins_the_launch():
    g = torch.zeros(8)
    launch = _hold([g], [g])
    desc = _adam(8, g)
    assert engine.attach_optimizer(desc, [g])
    assert len(launch.calls) == 1 and launch.calls[0] is desc
    assert engine.pending_step() is None
    assert not engine.attach_optimizer(desc, [g])   # nothing held any more


def test_attach_optimizer_declines_foreign_or_large_steps():
    g, other = torch.zeros(8), torch.zeros(8)
    launch = _hold([g], [g])
    assert not engine.attach_optimizer(_adam(8, other), [other])   # not this launch's gradients
    assert not engine.attach_optimizer(_adam(engine._FUSED_ADAM_MAX_NUMEL + 1, g), [g])
    assert launch.calls == [] and engine.pending_step() is not None


def test_native_launches_flush_first():
    g = torch.zeros(2)
    launch = _hold([g], [g])
    assert nat._LAUNCH_HOOK is engine.flush_pending_step
    nat._LAUNCH_HOOK()
    assert launch.calls == [None]


def test_a_new_hold_flushes_the_previous_one():
    a, b = torch.zeros(1), torch.zeros(1)
    first = _hold([a], [a])
    second = _hold([b], [b])
    assert first.calls == [None] and second.calls == []


def test_failed_launch_raises_at_the_consumer():
    g = torch.zeros(1)
    assert engine._defer_step(lambda adam: -3, "mi_elbo_forward", [[g]], ())
    with pytest.raises(nat.NativeError, match="mi_elbo_forward failed: unsupported"):
        engine.flush_pending_step()


def test_defer_disabled(monkeypatch):
    monkeypatch.setenv("MININF_AMD_DEFER_STEP", "0")
    assert not engine._defer_step(_Launch([]), "stand-in", [[]], ())
    assert engine.pending_step() is None


def test_validation_read_flushes():
    flags = torch.zeros(2, dtype=torch.int32)
    launch = _hold([flags.view(torch.float32)])
    joint = engine.LogJoint(total=torch.zeros(()), pending=[], checks=[], flags=flags)
    joint.flag_vector()
    assert launch.calls == [None]


def test_adam_descriptor_pointer_argument():
    # the ctypes prototypes take the descriptor by pointer (NULL: no optimizer step)
    argtypes = nat._SIGNATURES["mi_elbo_adam_supported"][1]
    assert argtypes[1] is ctypes.POINTER(nat.ElboAdam)
