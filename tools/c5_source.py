"""
Write the specialised site program of the C5 group (the fused z draw with the z / y / b sites,
engine.describe's layout) to a file, on the CPU: mi_group_source is host code. Compile the result
offline to inspect its ISA, e.g.

    python tools/c5_source.py /tmp/c5.hip [K] [N]
    hipcc -O3 -std=c++17 -fno-slp-vectorize --offload-arch=gfx950 --cuda-device-only -S \
        -I include -I mininf_amd/csrc /tmp/c5.hip -o /tmp/c5.s
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mininf_amd import _native as nat  # noqa: E402


def c5_group(K: int, N: int, grads: bool = True, bench: bool = True) -> nat.Group:
    dummy = 1 << 20   # any aligned non-null address: only the signature matters here
    g = nat.Group()
    g.K, g.N = K, N
    g.num_sites, g.num_operands = 3, 4
    g.num_slots = 1 if grads else 0
    g.compute_grads = int(grads)
    g.grad_scale = -1.0 / K
    g.options = nat.GROUP_DRAW_PARTIALS if grads else 0
    z, mu, y, b = (g.operands[i] for i in range(4))
    z.stride_k, z.stride_i, z.grad_mode = N, 1, nat.GRAD_DENSE if grads else nat.GRAD_NONE
    mu.data, mu.stride_k, mu.stride_i = dummy, 1, 0
    mu.grad_mode, mu.slot = (nat.GRAD_PARTICLE if grads else nat.GRAD_NONE), 0
    y.data, y.stride_k, y.stride_i = dummy, 0, 1
    b.data, b.stride_k, b.stride_i = dummy, 0, 1
    d = g.draw
    d.operand, d.stream_id = 1, 1
    d.loc, d.loc_stride, d.scale, d.scale_stride = dummy, 1, dummy, 1
    d.scale_exp = dummy
    d.seed, d.step = 1, 0
    d.step_device = dummy
    sites = [(nat.NORMAL, (1, -1, 0), (0.0, 1.0, 0.0), False),
             (nat.NORMAL, (0, -1, 2), (0.0, 0.5, 0.0), True),
             (nat.BERNOULLI_LOGITS, (0, -1, 3), (0.0, 0.0, 0.0), True)]
    for s, (family, ops, consts, masked) in zip(g.sites, sites):
        s.family = family
        for q in range(3):
            s.operand[q] = ops[q]
            s.constant[q] = consts[q]
        if masked:
            s.mask, s.mask_stride_k, s.mask_stride_i = dummy, 0, 1
        s.scale = 1.0
    if bench:   # as benched: mu's prior folded in (mi_group.prior), mu drawn by the program (pdraw)
        g.prior.present, g.prior.family = 1, nat.NORMAL
        g.prior.constant[0], g.prior.constant[1] = 0.0, 1.0
        g.prior.scale, g.prior.flags = 1.0, dummy
        p = g.pdraw
        p.operand, p.stream_id = 2, 0
        p.loc, p.loc_stride, p.scale, p.scale_stride = dummy, 0, dummy, 0
        p.scale_exp = dummy
        p.seed, p.step, p.step_device = 1, 0, dummy
    return g


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "/tmp/c5.hip"
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000
    g = c5_group(K, N)
    need = ctypes.c_size_t()
    nat.check(nat.lib().mi_group_source(ctypes.byref(g), None, 0, ctypes.byref(need)), "source")
    buf = ctypes.create_string_buffer(need.value)
    nat.check(nat.lib().mi_group_source(ctypes.byref(g), buf, need.value, None), "source")
    with open(out, "w") as fh:
        fh.write(buf.value.decode())
    print(out, need.value)


if __name__ == "__main__":
    main()
