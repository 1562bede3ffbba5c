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
                        "adam.hip", "mvn.hip", "peer.hip", "jit.cpp")]
HEADERS = [os.path.join(CSRC, name) for name in ("common.hpp", "device_math.hpp", "beta_grad.hpp", "jit.hpp",
                                                 "internal.hpp", "entropy.hpp", "adam_math.hpp")] + \
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


OBJ = os.path.join(HERE, "_obj")   # per-source objects (git- and gpurun-ignored)


def build(force: bool = False, verbose: bool = True) -> str:
    """
    Compile the HIP sources into ``mininf_amd/libmininf_amd.so`` unless it is up to date: one
    object per source, compiled in parallel (a source is recompiled when it or any header is newer
    than its object), then linked.
    """
    write_embedded()
    if not force and up_to_date():
        return TARGET
    os.makedirs(OBJ, exist_ok=True)
    headers = max(os.path.getmtime(path) for path in HEADERS)
    compile_flags = [f for f in FLAGS if f != "-shared"]
    jobs, objects = [], []
    for source in SOURCES:
        obj = os.path.join(OBJ, os.path.basename(source) + ".o")
        objects.append(obj)
        if force or not os.path.exists(obj) or \
                os.path.getmtime(obj) < max(headers, os.path.getmtime(source)):
            command = [HIPCC, *compile_flags, "-c", "-o", obj, source]
            if verbose:
                print(" ".join(command), file=sys.stderr)
            jobs.append(subprocess.Popen(command))
    failed = [job.args[-1] for job in jobs if job.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, f"hipcc {' '.join(failed)}")
    # linked beside the target, then renamed over it: a reader never sees a half-written library
    partial = TARGET + ".partial"
    command = [HIPCC, *FLAGS, "-o", partial, *objects, *LIBS]
    if verbose:
        print(" ".join(command), file=sys.stderr)
    subprocess.run(command, check=True)
    os.replace(partial, TARGET)
    return TARGET


if __name__ == "__main__":
    build(force="--force" in sys.argv)
