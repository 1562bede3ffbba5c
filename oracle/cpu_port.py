"""
The reference's ELBO step on the CPU (test / baseline infrastructure only).

Restates, on torch-CPU with one guide draw per loss call exactly as the reference does
(mininf/nn.py:212-228), the log-probability tracer of mininf/core.py:207-273 -- full parameter
validation on every call (core.py:142-189), masked branch (core.py:231-239), minibatch scaling
(core.py:267-271) -- through the same plugin point (TracerMixin) the reference uses. K particles are
``mean(loss_k for k in range(K))`` followed by backward and the optimizer step.
It is what bench.py times as ``cpu_baseline`` (kind "port").
"""
from __future__ import annotations

from typing import Callable, Dict

import torch
from torch.distributions.constraints import Constraint

from mininf_amd import core
from mininf_amd.core import batch, no_log_prob, TracerMixin, Value
from mininf_amd.util import check_constraint, get_masked_data_with_dense_grad


class PortTracer(TracerMixin):
    """
    Single-draw log joint with the reference's validation and accumulation semantics.
    """
    def __init__(self) -> None:
        super().__init__()
        self.contributions: Dict[str, torch.Tensor] = {}

    def sample(self, state, name, distribution, sample_shape=None):
        if isinstance(distribution, Value):
            value = state.get(name, distribution.value)
            self._assert_valid_parameter(value, name, distribution, sample_shape)
            return value
        if name in self.contributions:
            raise RuntimeError(f"Log probability has already been evaluated for '{name}'.")
        value = state.get(name)
        if value is None:
            raise ValueError(f"Cannot evaluate log probability; variable '{name}' is missing.")
        self._assert_valid_parameter(value, name, distribution, sample_shape)
        if no_log_prob.get_instance():
            return value
        declared = batch.get_shape()
        if isinstance(value, torch.masked.MaskedTensor):
            support = distribution.support
            if distribution._validate_args and not check_constraint(support, value).all():
                raise ValueError(f"Sample {value} is not in the support {support}.")
            flag = distribution._validate_args
            distribution._validate_args = False
            try:
                lp = distribution.log_prob(get_masked_data_with_dense_grad(value))
            finally:
                distribution._validate_args = flag
            if declared:
                raise ValueError("Batch dimensions are not supported for masked data.")
            self.contributions[name] = lp[value.get_mask()].sum()
        else:
            lp = distribution.log_prob(value)
            total = lp.sum()
            if declared:
                total = total * declared.numel() / lp.shape[:len(declared)].numel()
            self.contributions[name] = total
        return value

    def total(self):
        return sum(self.contributions.values())


def single_draw_loss(model: Callable, guide: Dict[str, torch.distributions.Distribution]):
    """
    -(log joint + entropy) for one reparameterised draw of every guide factor (nn.py:212-228).
    """
    draws = {name: factor.rsample() for name, factor in guide.items()}
    with PortTracer() as tracer:
        core.condition(model, **draws)()
    entropy = sum(factor.entropy().sum() for factor in guide.values())
    return -(tracer.total() + entropy)


def k_particle_step(model: Callable, guide_module: Callable, optimizer, K: int) -> float:
    """
    One optimisation step with K single-draw losses (the reference has no particle axis).
    """
    optimizer.zero_grad()
    guide = guide_module()
    if not isinstance(guide, dict):
        guide = dict(guide)
    loss = sum(single_draw_loss(model, guide) for _ in range(K)) / K
    loss.backward()
    optimizer.step()
    return float(loss.detach())
