"""
ctypes binding of ``libmininf_amd.so`` -- the C ABI declared in ``include/mininf_amd.h``.

The shared library is built in-tree by ``__graft_entry__.build()`` (``hipcc --offload-arch=gfx950``)
and loaded from this package directory. There is deliberately no fallback: if the library is missing
or a launch fails, :func:`lib` / :func:`check` raise, so a GPU run can never silently fall back to
PyTorch or CPU arithmetic.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch


LIB_NAME = "libmininf_amd.so"
# MININF_AMD_LIB: another build of the library (A/B measurements of kernel variants)
LIB_PATH = os.environ.get("MININF_AMD_LIB") or \
    os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

MAX_SITES = 4
MAX_OPERANDS = 6
MAX_SLOTS = 4
MAX_TERMS = 8
MAX_FACTORS = 8
MAX_BUFFERS = 16
LINEAR_MAX_P = 64
LINEAR_VALU = 2

NORMAL, BERNOULLI_LOGITS, BERNOULLI_PROBS, BETA, GAMMA, POISSON, INVERSE_GAMMA = 0, 1, 2, 3, 4, 5, 6
GRAD_NONE, GRAD_DENSE, GRAD_PARTICLE = 0, 1, 2
GROUP_FLAGS_ZEROED = 1
GROUP_DRAW_PARTIALS = 2
TRANSFORM_NONE, TRANSFORM_EXP = 0, 1
DRAW_NONE, DRAW_SOURCES, DRAW_PARTIALS = 0, 1, 2
MAX_SOURCES = 4
MAX_REDUCE = 4
REDUCE_MAX_SEG = 1024
ELBO_COUNTER_BYTES = 16640
ELBO_FINAL_GRADS = 1   # MI_ELBO_FINAL_GRADS
ABI_VERSION = 18   # MI_ABI_VERSION of include/mininf_amd.h
FLAG_SUPPORT, FLAG_PARAM, FLAG_INTERNAL = 1, 2, 0x40000000
MI_EINVAL, MI_EWORKSPACE, MI_EUNSUPPORTED = -1, -2, -3

c_i64 = ctypes.c_int64
c_f32p = ctypes.POINTER(ctypes.c_float)
c_vp = ctypes.c_void_p


class Operand(ctypes.Structure):
    _fields_ = [
        ("data", c_vp), ("stride_k", c_i64), ("stride_i", c_i64),
        ("grad_mode", ctypes.c_int32), ("slot", ctypes.c_int32),
        ("grad", c_vp), ("grad_stride_k", c_i64), ("grad_stride_i", c_i64),
    ]


class Site(ctypes.Structure):
    _fields_ = [
        ("family", ctypes.c_int32), ("operand", ctypes.c_int32 * 3),
        ("constant", ctypes.c_float * 3), ("pad0", ctypes.c_int32),
        ("mask", c_vp), ("mask_stride_k", c_i64), ("mask_stride_i", c_i64),
        ("scale", ctypes.c_double),
    ]


class Draw(ctypes.Structure):
    _fields_ = [
        ("operand", ctypes.c_int32), ("stream_id", ctypes.c_uint32),
        ("loc", c_vp), ("loc_stride", c_i64), ("scale", c_vp), ("scale_stride", c_i64),
        ("seed", ctypes.c_uint64), ("step", ctypes.c_uint64), ("step_device", c_vp),
        ("particle_offset", c_i64), ("dloc", c_vp), ("dscale", c_vp),
        ("scale_exp", c_vp), ("element_offset", c_i64),
    ]


class Side(ctypes.Structure):
    _fields_ = [("x", c_vp), ("c1", c_vp), ("c1_stride", c_i64), ("c0", c_vp),
                ("c0_stride", c_i64), ("K", c_i64), ("N", c_i64), ("out", c_vp)]


class Prior(ctypes.Structure):
    _fields_ = [("present", ctypes.c_int32), ("family", ctypes.c_int32),
                ("constant", ctypes.c_float * 2), ("scale", ctypes.c_double), ("flags", c_vp)]


class Group(ctypes.Structure):
    _fields_ = [
        ("K", c_i64), ("N", c_i64),
        ("num_sites", ctypes.c_int32), ("num_operands", ctypes.c_int32),
        ("num_slots", ctypes.c_int32), ("compute_grads", ctypes.c_int32),
        ("grad_scale", ctypes.c_float), ("options", ctypes.c_int32),
        ("sites", Site * MAX_SITES), ("operands", Operand * MAX_OPERANDS),
        ("draw", Draw), ("side", Side), ("prior", Prior), ("pdraw", Draw), ("stamps", c_vp),
    ]


class Rows(ctypes.Structure):
    _fields_ = [("counter", c_vp), ("n", c_i64), ("batch", c_i64), ("batches", c_i64),
                ("seed", ctypes.c_uint64), ("shuffle", ctypes.c_int32), ("pad0", ctypes.c_int32),
                ("out", c_vp)]


class Linear(ctypes.Structure):
    _fields_ = [
        ("K", c_i64), ("N", c_i64), ("P", c_i64),
        ("family", ctypes.c_int32), ("options", ctypes.c_int32),
        ("x", c_vp), ("x_stride_i", c_i64), ("x_stride_j", c_i64),
        ("theta", c_vp), ("theta_stride_k", c_i64), ("theta_stride_j", c_i64),
        ("value", c_vp), ("value_stride_i", c_i64),
        ("mask", c_vp), ("mask_stride_i", c_i64),
        ("scale", c_vp), ("scale_stride_k", c_i64),
        ("scale_constant", ctypes.c_float), ("grad_scale", ctypes.c_float),
        ("site_scale", ctypes.c_double),
        ("compute_grads", ctypes.c_int32), ("pad0", ctypes.c_int32),
        ("row_index", c_vp), ("rows", Rows), ("prior", Prior), ("draw", Draw),
        ("stamps", c_vp),
    ]


class Source(ctypes.Structure):
    _fields_ = [("ptr", c_vp), ("stride_k", c_i64), ("stride_i", c_i64)]


class Factor(ctypes.Structure):
    _fields_ = [
        ("family", ctypes.c_int32), ("draw_kind", ctypes.c_int32), ("n", c_i64),
        ("param", c_vp * 2), ("stride", c_i64 * 2), ("grad", c_vp * 2),
        ("grad_stride", c_i64 * 2), ("transform", ctypes.c_int32 * 2),
        ("num_sources", ctypes.c_int32), ("stream_id", ctypes.c_uint32),
        ("source", Source * MAX_SOURCES), ("draws", c_vp), ("eps", c_vp),
        ("seed", ctypes.c_uint64), ("step", ctypes.c_uint64), ("step_device", c_vp),
        ("particle_offset", c_i64), ("partial", c_vp * 2), ("partial_rows", c_i64),
        ("dgrad", c_vp), ("saved", c_vp), ("element_offset", c_i64), ("weight", ctypes.c_double),
    ]


MAX_PARAMS = 4


class Params(ctypes.Structure):
    _fields_ = [("m", ctypes.c_int32), ("pad0", ctypes.c_int32), ("n", c_i64),
                ("u", c_vp * MAX_PARAMS), ("stride", c_i64 * MAX_PARAMS),
                ("transform", ctypes.c_int32 * MAX_PARAMS)]


class Reduce(ctypes.Structure):
    _fields_ = [
        ("part", c_vp), ("nseg", c_i64), ("K", c_i64),
        ("num_sites", ctypes.c_int32), ("num_slots", ctypes.c_int32),
        ("rank1", ctypes.c_int32), ("pad0", ctypes.c_int32),
        ("scale", ctypes.c_double * MAX_SITES), ("slot_scale", ctypes.c_double),
        ("total", c_vp), ("site_lp", c_vp), ("slot_grad", c_vp),
    ]


class Elbo(ctypes.Structure):
    _fields_ = [
        ("K", c_i64), ("num_terms", ctypes.c_int32), ("num_factors", ctypes.c_int32),
        ("num_buffers", ctypes.c_int32), ("num_reduce", ctypes.c_int32),
        ("g0", ctypes.c_float), ("options", ctypes.c_int32), ("entropy_scale", ctypes.c_double),
        ("terms", c_vp * MAX_TERMS), ("factors", Factor * MAX_FACTORS),
        ("buffers", c_vp * MAX_BUFFERS), ("buffer_len", c_i64 * MAX_BUFFERS),
        ("reduce", Reduce * MAX_REDUCE),
        ("step_counter", c_vp), ("step_snapshot", c_vp),
        ("flags", c_vp), ("flags_mirror", c_vp), ("nflags", c_i64),
    ]


ADAM_MAX_TENSORS = 8
ADAM_COUNTER_WORDS = ADAM_MAX_TENSORS * 33 + ADAM_MAX_TENSORS * 16


class AdamTensor(ctypes.Structure):
    _fields_ = [("param", c_vp), ("grad", c_vp), ("exp_avg", c_vp), ("exp_avg_sq", c_vp),
                ("step", c_vp), ("numel", c_i64)]


PEER_MAX_RANKS = 8
PEER_MAX_FLOATS = 4096
PEER_HANDLE_BYTES = 64


class Peer(ctypes.Structure):
    """mi_peer (include/mininf_amd.h)."""
    _fields_ = [("rank", ctypes.c_int32), ("world", ctypes.c_int32), ("max_floats", c_i64),
                ("regions", c_vp * PEER_MAX_RANKS)]


class Adam(ctypes.Structure):
    _fields_ = [("num", ctypes.c_int32), ("maximize", ctypes.c_int32), ("lr", ctypes.c_double),
                ("beta1", ctypes.c_double), ("beta2", ctypes.c_double), ("eps", ctypes.c_double),
                ("weight_decay", ctypes.c_double), ("tensors", AdamTensor * ADAM_MAX_TENSORS)]


ELBO_ADAM_SLOTS = 4   # MI_ELBO_ADAM_SLOTS


class ElboAdamSlot(ctypes.Structure):
    _fields_ = [("factor", ctypes.c_int32), ("param", ctypes.c_int32), ("value", c_vp),
                ("exp_avg", c_vp), ("exp_avg_sq", c_vp), ("step", c_vp), ("numel", c_i64)]


class ElboAdam(ctypes.Structure):
    _fields_ = [("num", ctypes.c_int32), ("maximize", ctypes.c_int32), ("lr", ctypes.c_double),
                ("beta1", ctypes.c_double), ("beta2", ctypes.c_double), ("eps", ctypes.c_double),
                ("weight_decay", ctypes.c_double), ("slots", ElboAdamSlot * ELBO_ADAM_SLOTS)]


# name -> (restype, argtypes). Mirrors include/mininf_amd.h one to one.
_SIGNATURES = {
    "mi_abi_version": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t]),
    "mi_wall_clock_khz": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "mi_struct_sizes": (ctypes.c_int, [ctypes.POINTER(ctypes.c_size_t)] * 3),
    "mi_group_pdraw_supported": (ctypes.c_int, [ctypes.POINTER(Group),
                                                ctypes.POINTER(ctypes.c_int)]),
    "mi_group_workspace_bytes": (ctypes.c_int, [ctypes.POINTER(Group),
                                                ctypes.POINTER(ctypes.c_size_t)]),
    "mi_group_forward": (ctypes.c_int, [ctypes.POINTER(Group), c_vp, ctypes.c_size_t, c_vp, c_vp,
                                        c_vp, c_vp, c_vp]),
    "mi_group_forward_deferred": (ctypes.c_int, [ctypes.POINTER(Group), c_vp, ctypes.c_size_t,
                                                 c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                                 ctypes.POINTER(Reduce)]),
    "mi_reduce_launch": (ctypes.c_int, [ctypes.POINTER(Reduce), c_vp]),
    "mi_group_draw_partials": (ctypes.c_int, [ctypes.POINTER(Group),
                                              ctypes.POINTER(ctypes.c_size_t),
                                              ctypes.POINTER(c_i64)]),
    "mi_group_source": (ctypes.c_int, [ctypes.POINTER(Group), ctypes.c_char_p, ctypes.c_size_t,
                                       ctypes.POINTER(ctypes.c_size_t)]),
    "mi_group_compile_check": (ctypes.c_int, [ctypes.POINTER(Group), ctypes.c_char_p,
                                              ctypes.c_size_t]),
    "mi_scale_rows": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, ctypes.c_float,
                                     c_vp]),
    "mi_categorical_workspace_bytes": (ctypes.c_int, [c_i64, c_i64,
                                                      ctypes.POINTER(ctypes.c_size_t)]),
    "mi_categorical_forward": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64,
                                              c_vp, c_i64, c_i64, c_vp, c_i64, ctypes.c_double,
                                              ctypes.c_float, c_vp, c_vp, ctypes.c_size_t, c_vp,
                                              c_vp, c_vp]),
    "mi_cholesky": (ctypes.c_int, [c_vp, ctypes.c_int32, c_i64, c_i64, c_vp, ctypes.c_int32,
                                   c_vp, c_vp]),
    "mi_mvn_tril_forward": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp,
                                           c_vp]),
    "mi_normal_rsample": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, ctypes.c_uint64,
                                         ctypes.c_uint64, c_vp, ctypes.c_uint32, c_i64, c_i64, c_vp,
                                         c_vp, c_vp]),
    "mi_normal_rsample_backward_workspace_bytes": (ctypes.c_int, [
        c_i64, c_i64, ctypes.POINTER(ctypes.c_size_t)]),
    "mi_normal_rsample_backward": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, c_i64,
                                                  ctypes.c_uint64, ctypes.c_uint64, c_vp,
                                                  ctypes.c_uint32, c_i64, c_i64, c_vp, c_vp,
                                                  ctypes.c_size_t, c_vp, c_vp, c_vp]),
    "mi_beta_rsample": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, ctypes.c_uint64,
                                       ctypes.c_uint64, c_vp, ctypes.c_uint32, c_i64, c_vp, c_vp,
                                       c_vp]),
    "mi_normal_rsample_exp": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64,
                                             ctypes.c_uint64, ctypes.c_uint64, c_vp,
                                             ctypes.c_uint32, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "mi_beta_rsample_exp": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64,
                                           ctypes.c_uint64, ctypes.c_uint64, c_vp, ctypes.c_uint32,
                                           c_i64, c_vp, c_vp, c_vp]),
    "mi_beta_dgrad": (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "mi_capture_abandon": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_int)]),
    "mi_step_begin": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_vp]),
    "mi_group_side_supported": (ctypes.c_int, [ctypes.POINTER(Group),
                                               ctypes.POINTER(ctypes.c_int)]),
    "mi_group_prior_supported": (ctypes.c_int, [ctypes.POINTER(Group),
                                                ctypes.POINTER(ctypes.c_int)]),
    "mi_linear_prior_supported": (ctypes.c_int, [ctypes.POINTER(Linear),
                                                 ctypes.POINTER(ctypes.c_int)]),
    "mi_transform_params": (ctypes.c_int, [ctypes.POINTER(Params), c_vp, c_vp]),
    "mi_beta_rsample_backward_workspace_bytes": (ctypes.c_int, [
        c_i64, c_i64, ctypes.POINTER(ctypes.c_size_t)]),
    "mi_beta_rsample_backward": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64,
                                                c_i64, c_i64, c_vp, ctypes.c_size_t, c_vp, c_i64,
                                                c_vp, c_i64, c_vp]),
    "mi_gamma_rsample": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, ctypes.c_uint64,
                                        ctypes.c_uint64, c_vp, ctypes.c_uint32, c_i64, c_vp, c_vp,
                                        c_vp, c_vp]),
    "mi_gamma_rsample_backward_workspace_bytes": (ctypes.c_int, [c_i64, c_i64,
                                                                 ctypes.POINTER(ctypes.c_size_t)]),
    "mi_gamma_rsample_backward": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp,
                                                 c_i64, c_i64, c_i64, c_vp, ctypes.c_size_t, c_vp,
                                                 c_i64, c_vp, c_i64, c_vp]),
    "mi_philox_normal": (ctypes.c_int, [c_i64, c_i64, ctypes.c_uint64, ctypes.c_uint64,
                                        ctypes.c_uint32, c_i64, c_vp, c_vp]),
    "mi_philox4x32": (ctypes.c_int, [c_vp, c_i64, ctypes.c_uint32, ctypes.c_uint32, c_vp, c_vp]),
    "mi_elbo_struct_sizes": (ctypes.c_int, [ctypes.POINTER(ctypes.c_size_t)] * 2),
    "mi_linear_struct_size": (ctypes.c_int, [ctypes.POINTER(ctypes.c_size_t)]),
    "mi_linear_workspace_bytes": (ctypes.c_int, [ctypes.POINTER(Linear),
                                                 ctypes.POINTER(ctypes.c_size_t)]),
    "mi_linear_forward": (ctypes.c_int, [ctypes.POINTER(Linear), c_vp, ctypes.c_size_t, c_vp, c_vp,
                                         c_vp, c_vp]),
    "mi_linear_forward_deferred": (ctypes.c_int, [ctypes.POINTER(Linear), c_vp, ctypes.c_size_t,
                                                  c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                                  ctypes.POINTER(Reduce)]),
    "mi_minibatch_rows": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, ctypes.c_int32,
                                         ctypes.c_uint64, c_vp, c_i64, c_vp]),
    "mi_gather_rows": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "mi_adam_step": (ctypes.c_int, [ctypes.POINTER(Adam), c_vp, c_vp]),
    "mi_peer_region_bytes": (ctypes.c_int, [c_i64, ctypes.POINTER(ctypes.c_size_t)]),
    "mi_peer_alloc": (ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(c_vp), c_vp]),
    "mi_peer_open": (ctypes.c_int, [c_vp, ctypes.POINTER(c_vp)]),
    "mi_peer_close": (ctypes.c_int, [c_vp]),
    "mi_peer_free": (ctypes.c_int, [c_vp]),
    "mi_peer_allreduce": (ctypes.c_int, [ctypes.POINTER(Peer), c_vp, c_vp, c_i64, c_vp, c_vp]),
    "mi_peer_call_count": (ctypes.c_int, [ctypes.POINTER(Peer), ctypes.POINTER(ctypes.c_uint64)]),
    "mi_elbo_workspace_bytes": (ctypes.c_int, [ctypes.POINTER(Elbo),
                                               ctypes.POINTER(ctypes.c_size_t)]),
    "mi_elbo_workspace_init": (ctypes.c_int, [c_vp, ctypes.c_size_t, c_vp]),
    "mi_elbo_forward": (ctypes.c_int, [ctypes.POINTER(Elbo), c_vp, ctypes.c_size_t, c_vp, c_vp]),
    "mi_elbo_adam_supported": (ctypes.c_int, [ctypes.POINTER(Elbo), ctypes.POINTER(ElboAdam),
                                              ctypes.POINTER(ctypes.c_int)]),
    "mi_elbo_forward_adam": (ctypes.c_int, [ctypes.POINTER(Elbo), c_vp, ctypes.c_size_t, c_vp,
                                            c_vp, c_vp]),
    "mi_elbo_final_grads": (ctypes.c_int, [ctypes.POINTER(Elbo), ctypes.POINTER(ctypes.c_int)]),
    "mi_elbo_backward": (ctypes.c_int, [ctypes.POINTER(Elbo), c_vp, c_vp, c_vp, ctypes.c_size_t,
                                        c_vp]),
}

EXPORTED_SYMBOLS = tuple(_SIGNATURES)

_LIB: Optional[ctypes.CDLL] = None


class NativeError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """
    Load (once) and return the HIP library. Raises if it has not been built.
    """
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"{LIB_PATH} is missing; build it with `python -c 'import "
                              "__graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950).")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (restype, argtypes) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = restype
            fn.argtypes = argtypes
        target = ctypes.create_string_buffer(16)
        version = handle.mi_abi_version(target, 16)
        if version != ABI_VERSION:   # the struct mirrors below would be misread
            raise NativeError(f"{LIB_PATH} has ABI version {version}, this binding expects "
                              f"{ABI_VERSION}; rebuild it (mininf_amd/build.py --force).")
        _LIB = handle
    return _LIB


def check(code: int, what: str) -> None:
    if code != 0:
        kind = {-1: "invalid argument", -2: "workspace too small", -3: "unsupported"}.get(
            code, f"hipError_t {code}")
        raise NativeError(f"{what} failed: {kind}")


_LAUNCH_HOOK = None


def set_launch_hook(hook) -> None:
    """``hook()`` runs before every native launch (engine: enqueue a held finishing launch)."""
    global _LAUNCH_HOOK
    _LAUNCH_HOOK = hook


def stream_handle(device: torch.device) -> int:
    """
    hipStream_t of torch's current stream on ``device`` (kernels are ordered with torch's own).
    Every launch asks for it, so a held launch (engine._PendingStep) is enqueued here first.
    """
    if _LAUNCH_HOOK is not None:
        _LAUNCH_HOOK()
    index = getattr(device, "index", None)
    if index is None:
        return torch.cuda.current_stream(device).cuda_stream
    # the raw handle without constructing a torch.cuda.Stream (a few microseconds per launch)
    return torch._C._cuda_getCurrentRawStream(index)


def ptr(tensor: Optional[torch.Tensor]) -> Optional[int]:
    return None if tensor is None else tensor.data_ptr()


def require_device(tensor: torch.Tensor, what: str) -> None:
    if tensor.device.type != "cuda":
        raise NativeError(f"{what} must live on a ROCm device for the MI355X ELBO engine, got "
                          f"{tensor.device}. Move the data and the guide to 'cuda' (HIP).")
