"""
In-tree build of ``libmininf_amd.so`` (gfx950). Used by ``__graft_entry__.build()`` and the tests.

The library holds the precompiled kernels (sites.hip, guide.hip, elbo.hip, linear.hip) and the host-side site-program
specialiser (jit.cpp), which embeds ``include/mininf_amd.h`` and ``csrc/device_math.hpp`` verbatim
so that kernels compiled at trace time by hiprtc share the exact device math of the precompiled
ones.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(ROOT, "include")
SOURCES = [os.path.join(CSRC, name)
           for name in ("sites.hip", "guide.hip", "elbo.hip", "linear.hip", "minibatch.hip",
                        "adam.hip", "mvn.hip", "jit.cpp")]
HEADERS = [os.path.join(CSRC, name) for name in ("common.hpp", "device_math.hpp", "beta_grad.hpp", "jit.hpp",
                                                 "internal.hpp")] + \
    [os.path.join(INCLUDE, "mininf_amd.h")]
EMBEDDED = {"embedded_header.inc": os.path.join(INCLUDE, "mininf_amd.h"),
            "embedded_math.inc": os.path.join(CSRC, "device_math.hpp")}
TARGET = os.path.join(HERE, "libmininf_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", f"--offload-arch={ARCH}",
         "-fno-slp-vectorize",  # SLP packing of independent fp32 chains into v_pk_* only adds moves
         f"-I{INCLUDE}", f"-I{CSRC}"]
LIBS = ["-lhiprtc"]


def write_embedded() -> None:
    """
    Generate csrc/embedded_*.inc: C++ raw-string literals of the headers hiprtc compiles against.
    """
    for name, source in EMBEDDED.items():
        with open(source) as fh:
            text = fh.read()
        if ")MIEMBED" in text:
            raise RuntimeError(f"{source} contains the raw-string delimiter")
        content = 'R"MIEMBED(' + text + ')MIEMBED"\n'
        target = os.path.join(CSRC, name)
        if not os.path.exists(target) or open(target).read() != content:
            with open(target, "w") as fh:
                fh.write(content)


def up_to_date() -> bool:
    if not os.path.exists(TARGET):
        return False
    built = os.path.getmtime(TARGET)
    return all(os.path.getmtime(path) <= built for path in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = True) -> str:
    """
    Compile the HIP sources into ``mininf_amd/libmininf_amd.so`` unless it is up to date.
    """
    write_embedded()
    if not force and up_to_date():
        return TARGET
    command = [HIPCC, *FLAGS, "-o", TARGET, *SOURCES, *LIBS]
    if verbose:
        print(" ".join(command), file=sys.stderr)
    subprocess.run(command, check=True)
    return TARGET


if __name__ == "__main__":
    build(force="--force" in sys.argv)
