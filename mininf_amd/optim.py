"""
MI355X optimizer step: :class:`Adam`, a drop-in ``torch.optim.Adam`` whose ``step()`` is one HIP
launch (``mi_adam_step``, ``csrc/adam.hip``) for up to eight parameters, step-count increment
included -- torch's capturable fused Adam needs a ``_foreach_add_`` launch for the step counts
plus the fused update. After a fused ELBO whose finishing launch is held (engine._PendingStep) the
step joins that launch instead: no launch of its own. Same arithmetic as ``torch.optim.Adam(fused=True)`` (bit-identical
updates), same ``state`` layout (``step``, ``exp_avg``, ``exp_avg_sq``), so ``state_dict`` moves
between the two.

The reference trains with ``torch.optim.Adam`` (``README.md:66-69``); this class is the same call
with the same arguments.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Iterable, Tuple

import torch

from . import _native as nat
from . import engine


class Adam(torch.optim.Optimizer):
    """
    Adam (Kingma & Ba) on fp32 device parameters. ``amsgrad`` and differentiable steps are not
    supported (use ``torch.optim.Adam``).
    """
    def __init__(self, params: Iterable, lr: float = 1e-3, betas: Tuple[float, float] = (0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, *, maximize: bool = False,
                 amsgrad: bool = False) -> None:
        if amsgrad:
            raise NotImplementedError("mininf_amd.optim.Adam does not implement amsgrad")
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 0: {betas[0]}")
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 1: {betas[1]}")
        if not 0.0 <= weight_decay:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        # capturable=True: Optimizer.load_state_dict then moves a loaded `step` (torch.optim.Adam's
        # default keeps it as a host tensor) to the parameter's device as float32
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      maximize=maximize, amsgrad=False, capturable=True,
                                      foreach=None, fused=None, differentiable=False))
        self._counters: Dict[torch.device, torch.Tensor] = {}
        # per parameter group: the launch descriptors of the last step, reused while the group's
        # parameters, state tensors and hyper-parameters are unchanged (only the gradients'
        # addresses are rewritten): a step costs microseconds of Python, not a rebuild
        self._plans: Dict[int, "_Plan"] = {}
        # torch wraps Optimizer.step in a profiling / hook dispatcher (tens of microseconds of
        # Python per call); with no hooks registered this instance calls the step directly
        self.step = self._dispatch_step  # type: ignore[method-assign]

    def _dispatch_step(self, closure=None):
        from torch.optim import optimizer as torch_optimizer
        if self._optimizer_step_pre_hooks or self._optimizer_step_post_hooks or \
                torch_optimizer._global_optimizer_pre_hooks or \
                torch_optimizer._global_optimizer_post_hooks:
            return type(self).step(self, closure)   # torch's hooked path
        with torch.no_grad():
            return type(self).step.__wrapped__(self, closure) \
                if hasattr(type(self).step, "__wrapped__") else type(self).step(self, closure)

    def zero_grad(self, set_to_none: bool = True) -> None:
        """``Optimizer.zero_grad``: with ``set_to_none`` (the default) every gradient is dropped
        here directly -- torch's version runs behind a dynamo-disable wrapper and a profiler range,
        tens of microseconds of Python per eager step for the same effect."""
        if not set_to_none:
            return super().zero_grad(set_to_none=False)
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is not None:
                    p.grad = None

    def _counter_words(self, device: torch.device) -> torch.Tensor:
        words = self._counters.get(device)
        if words is None:
            words = torch.zeros(nat.ADAM_COUNTER_WORDS, dtype=torch.int32, device=device)
            self._counters[device] = words
        return words

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = nat.lib()
        for gi, group in enumerate(self.param_groups):
            active = [p for p in group["params"] if p.grad is not None]
            plan = self._plans.get(gi)
            if plan is not None and plan.matches(group, active, self.state):
                plan.launch(active, lib, self._counter_words)
                continue
            beta1, beta2 = group["betas"]
            batch = []
            for p in active:
                if p.grad.is_sparse:
                    raise RuntimeError("Adam does not support sparse gradients")
                nat.require_device(p, "Adam parameter")
                if p.dtype != torch.float32 or not p.is_contiguous() or \
                        not p.grad.is_contiguous() or p.grad.dtype != torch.float32:
                    raise nat.NativeError("mininf_amd.optim.Adam takes contiguous float32 "
                                          "parameters and gradients")
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state["exp_avg_sq"] = torch.zeros_like(p,
                                                           memory_format=torch.preserve_format)
                # the kernel reads and writes every state tensor on the device: a state assigned
                # or loaded from elsewhere (a host `step`, a checkpoint mapped to the CPU) is moved
                # here first, never handed over as a host pointer
                step = state["step"]
                if not isinstance(step, torch.Tensor):
                    state["step"] = step = torch.tensor(float(step), dtype=torch.float32,
                                                        device=p.device)
                if step.device != p.device or step.dtype != torch.float32 or step.dim() != 0:
                    state["step"] = step.to(device=p.device, dtype=torch.float32).reshape(())
                for key in ("exp_avg", "exp_avg_sq"):
                    moment = state[key]
                    if moment.device != p.device or moment.dtype != torch.float32 or \
                            moment.shape != p.shape or not moment.is_contiguous():
                        state[key] = moment.to(device=p.device, dtype=torch.float32) \
                            .reshape(p.shape).contiguous()
                batch.append((p, state))
            descs = []
            for start in range(0, len(batch), nat.ADAM_MAX_TENSORS):
                chunk = batch[start:start + nat.ADAM_MAX_TENSORS]
                desc = nat.Adam()
                desc.num = len(chunk)
                desc.maximize = int(group["maximize"])
                desc.lr, desc.beta1, desc.beta2 = float(group["lr"]), float(beta1), float(beta2)
                desc.eps, desc.weight_decay = float(group["eps"]), float(group["weight_decay"])
                for j, (p, state) in enumerate(chunk):
                    t = desc.tensors[j]
                    t.param, t.grad = p.data_ptr(), p.grad.data_ptr()
                    t.exp_avg, t.exp_avg_sq = (state["exp_avg"].data_ptr(),
                                               state["exp_avg_sq"].data_ptr())
                    t.step, t.numel = state["step"].data_ptr(), p.numel()
                descs.append((desc, chunk[0][0].device))
            plan = _Plan(group, batch, descs)
            self._plans[gi] = plan
            plan.launch(active, lib, self._counter_words, fresh=True)
        return loss


class _Plan:
    """The ``mi_adam`` descriptors of one parameter group, reusable across steps."""
    def __init__(self, group: dict, batch, descs) -> None:
        self.params = [p for p, _ in batch]
        self.states = [(s, s["step"], s["exp_avg"], s["exp_avg_sq"]) for _, s in batch]
        self.hyper = self._hyper(group)
        self.descs = descs
        self.ptrs = [p.data_ptr() for p in self.params]

    @staticmethod
    def _hyper(group: dict):
        return (group["lr"], tuple(group["betas"]), group["eps"], group["weight_decay"],
                group["maximize"])

    def matches(self, group: dict, active, state) -> bool:
        if len(active) != len(self.params) or self._hyper(group) != self.hyper:
            return False
        for p, q, ptr, (s, step, m, v) in zip(active, self.params, self.ptrs, self.states):
            g = p.grad
            if p is not q or p.data_ptr() != ptr or state.get(p) is not s or \
                    s.get("step") is not step or s.get("exp_avg") is not m or \
                    s.get("exp_avg_sq") is not v:
                return False
            # (a held gradient's recorded layout: no torch call through its flush hook)
            _, dtype, device, contiguous = engine.grad_meta(g)
            if type(g) is not engine.PendingGrad and g.is_sparse or dtype != torch.float32 or \
                    not contiguous or device != p.device:
                return False
        return True

    def launch(self, active, lib, counter_words, fresh: bool = False) -> None:
        cursor = 0
        for desc, device in self.descs:
            if not fresh:
                for j in range(desc.num):
                    desc.tensors[j].grad = engine.grad_meta(active[cursor + j].grad)[0]
            grads = [p.grad for p in active[cursor:cursor + desc.num]]
            cursor += desc.num
            # the step's held finishing launch writes these gradients: the update runs in its
            # last block (one kernel for the whole training step, engine._PendingStep)
            if engine.attach_optimizer(desc, grads):
                continue
            nat.check(lib.mi_adam_step(ctypes.byref(desc), counter_words(device).data_ptr(),
                                       nat.stream_handle(device)), "mi_adam_step")
