"""
Build the oracle's C restatement (test infrastructure): oracle/philox.c -> oracle/liboracle.so.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCE = os.path.join(HERE, "philox.c")
TARGET = os.path.join(HERE, "liboracle.so")


def build(force: bool = False) -> str:
    if force or not os.path.exists(TARGET) or os.path.getmtime(TARGET) < os.path.getmtime(SOURCE):
        subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-o", TARGET, SOURCE, "-lm"], check=True)
    return TARGET


def load() -> ctypes.CDLL:
    lib = ctypes.CDLL(build())
    lib.oracle_philox4x32_10.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32,
                                         ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    lib.oracle_guide_normals.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64,
                                         ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int64,
                                         ctypes.c_void_p]
    f32, i32 = ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int32)
    lib.oracle_gamma_draws.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                       ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                       ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    lib.oracle_beta_draws.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                      ctypes.c_uint32, ctypes.c_int64] + [ctypes.c_void_p] * 5
    return lib


def gamma_draws(concentration, K, seed, step, stream_id, particle_offset=0):
    """
    Standard gamma draws [K, N] of ``mi_gamma_rsample`` (oracle_gamma_draws) and the Philox blocks
    each consumed.
    """
    import numpy as np
    conc = np.ascontiguousarray(concentration, dtype=np.float32).reshape(-1)
    N = conc.shape[0]
    g = np.empty((K, N), np.float32)
    blocks = np.empty((K, N), np.int32)
    load().oracle_gamma_draws(K, N, conc.ctypes.data, seed, step, stream_id, particle_offset,
                              g.ctypes.data, blocks.ctypes.data)
    return g, blocks


def beta_draws(c1, c0, K, seed, step, stream_id, particle_offset=0):
    """
    Beta draws [K, N] of ``mi_beta_rsample`` (oracle_beta_draws): (x, g1, g0, blocks1, blocks0).
    """
    import numpy as np
    a = np.ascontiguousarray(c1, dtype=np.float32).reshape(-1)
    b = np.ascontiguousarray(c0, dtype=np.float32).reshape(-1)
    N = a.shape[0]
    out = [np.empty((K, N), np.float32) for _ in range(3)] + \
        [np.empty((K, N), np.int32) for _ in range(2)]
    load().oracle_beta_draws(K, N, a.ctypes.data, b.ctypes.data, seed, step, stream_id,
                             particle_offset, *[o.ctypes.data for o in out])
    return tuple(out)
