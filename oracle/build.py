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
    return lib
