"""
mininf_amd -- MI355X-native black-box variational inference with the public API of mininf.

The probabilistic-program layer (``sample``, ``condition``, ``value``, ``batch``, ``no_log_prob``,
``State``, ``broadcast_samples``) mirrors the reference's ``mininf/__init__.py:1-14``. The ELBO hot
path behind :class:`mininf_amd.nn.EvidenceLowerBoundLoss` runs on hand-written HIP kernels for gfx950
(``mininf_amd/csrc``) through the C ABI declared in ``include/mininf_amd.h``.
"""
from .core import batch, broadcast_samples, condition, no_log_prob, value, sample, State
from . import data, nn, optim
from .data import DeviceDataLoader


__all__ = [
    "batch",
    "broadcast_samples",
    "condition",
    "data",
    "DeviceDataLoader",
    "nn",
    "no_log_prob",
    "value",
    "sample",
    "State",
]
