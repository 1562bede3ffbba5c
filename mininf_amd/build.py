"""
In-tree build of ``libmininf_amd.so`` (gfx950). Used by ``__graft_entry__.build()`` and the tests.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = [os.path.join(HERE, "csrc", name) for name in ("sites.hip", "guide.hip")]
HEADERS = [os.path.join(HERE, "csrc", "common.hpp"),
           os.path.join(os.path.dirname(HERE), "include", "mininf_amd.h")]
TARGET = os.path.join(HERE, "libmininf_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", f"--offload-arch={ARCH}"]


def up_to_date() -> bool:
    if not os.path.exists(TARGET):
        return False
    built = os.path.getmtime(TARGET)
    return all(os.path.getmtime(path) <= built for path in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = True) -> str:
    """
    Compile the HIP sources into ``mininf_amd/libmininf_amd.so`` unless it is up to date.
    """
    if not force and up_to_date():
        return TARGET
    command = [HIPCC, *FLAGS, "-o", TARGET, *SOURCES]
    if verbose:
        print(" ".join(command), file=sys.stderr)
    subprocess.run(command, check=True)
    return TARGET


if __name__ == "__main__":
    build(force="--force" in sys.argv)
