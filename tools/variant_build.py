"""
Variant builds of the library for A/B measurements on one box: every source as in the tree except
the substituted ones, into tools/_variants/<name>/libmininf_amd.so (git-ignored, sent to the GPU box) (select with MININF_AMD_LIB).

    python tools/variant_build.py <name> [csrc-file=replacement-path ...]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from mininf_amd import build as b
    name, subs = sys.argv[1], dict(a.split("=", 1) for a in sys.argv[2:])
    b.write_embedded()
    sources = [subs.get(os.path.basename(s), s) for s in b.SOURCES]
    out = os.path.join(ROOT, "tools", "_variants", name, "libmininf_amd.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    flags = [*b.FLAGS, f"-I{b.CSRC}"]
    subprocess.run([b.HIPCC, *flags, "-o", out, *sources, *b.LIBS], check=True)
    print(out)


if __name__ == "__main__":
    main()
