"""
Time mi_elbo_forward alone on synthetic descriptors (deferred reductions, tail Beta sums) to
attribute its cost: python tools/elbo_probe.py  (GPU).
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mininf_amd import _native as nat  # noqa: E402

dev = torch.device("cuda")
lib = nat.lib()
K = 4096


def job(nseg, slots=1):
    part = torch.randn((1 + slots) * nseg * K, device=dev)
    total = torch.empty(K, device=dev)
    slot = torch.empty((max(1, slots), K), device=dev)
    r = nat.Reduce()
    r.part, r.nseg, r.K, r.num_sites, r.num_slots = part.data_ptr(), nseg, K, 1, slots
    r.scale[0] = 1.0
    r.slot_scale = 1.0
    r.total, r.slot_grad = total.data_ptr(), slot.data_ptr()
    return r, (part, total, slot)


def beta_factor(E, j, slot_rows, keep):
    conc = torch.full((1, 2), 2.0, device=dev)
    dgrad = torch.randn(K, 1, 2, dtype=torch.float64, device=dev)
    saved = torch.empty(4, dtype=torch.float64, device=dev)
    d = E.factors[j]
    d.family, d.n, d.draw_kind = nat.BETA, 1, nat.DRAW_SOURCES
    d.param[0], d.param[1] = conc.data_ptr(), conc.data_ptr() + 4
    d.stride[0] = d.stride[1] = 2
    d.num_sources = len(slot_rows)
    for s, row in enumerate(slot_rows):
        d.source[s].ptr, d.source[s].stride_k, d.source[s].stride_i = row.data_ptr(), 1, 0
    d.dgrad, d.saved = dgrad.data_ptr(), saved.data_ptr()
    d.draws = conc.data_ptr()
    keep += [conc, dgrad, saved]


def run(name, jobs=(), tail=False, terms=0):
    keep = []
    E = nat.Elbo()
    E.K, E.g0, E.entropy_scale = K, -1.0 / K, 1.0
    rows = []
    for j, nseg in enumerate(jobs):
        r, t = job(nseg)
        keep += list(t)
        E.reduce[j] = r
        rows.append(t[2][0])
    E.num_reduce = len(jobs)
    for t in range(terms):
        x = torch.randn(K, device=dev)
        keep.append(x)
        E.terms[t] = x.data_ptr()
    E.num_terms = terms
    if tail:
        beta_factor(E, 0, rows or [torch.zeros(K, device=dev)], keep)
        E.num_factors = 1
    size = ctypes.c_size_t()
    nat.check(lib.mi_elbo_workspace_bytes(ctypes.byref(E), ctypes.byref(size)), "ws")
    ws = torch.zeros(max(size.value, 1 << 16), dtype=torch.uint8, device=dev)
    loss = torch.empty((), device=dev)
    s = nat.stream_handle(dev)
    for _ in range(20):
        nat.check(lib.mi_elbo_forward(ctypes.byref(E), ws.data_ptr(), ws.numel(), loss.data_ptr(), s), name)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    n = 200
    for _ in range(n):
        lib.mi_elbo_forward(ctypes.byref(E), ws.data_ptr(), ws.numel(), loss.data_ptr(), s)
    b.record()
    torch.cuda.synchronize()
    fwd = a.elapsed_time(b) / n * 1e3
    up = torch.ones((), device=dev)
    dterm = torch.empty(1, device=dev)
    grads = []
    for j in range(E.num_factors):
        g = torch.empty(4, device=dev)
        grads.append(g)
        E.factors[j].grad[0], E.factors[j].grad[1] = g.data_ptr(), g.data_ptr() + 4
        E.factors[j].grad_stride[0] = E.factors[j].grad_stride[1] = 1
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        lib.mi_elbo_backward(ctypes.byref(E), up.data_ptr(), dterm.data_ptr(), ws.data_ptr(),
                             ws.numel(), s)
    b.record()
    torch.cuda.synchronize()
    print(f"{name:40s} fwd {fwd:8.1f} us  bwd {a.elapsed_time(b) / n * 1e3:8.1f} us", flush=True)


run("terms only (1 term)", terms=1)
run("beta entropy, no sources", tail=False, terms=1)
run("1 job nseg=2", jobs=(2,))
run("1 job nseg=246", jobs=(246,))
run("2 jobs 2 + 246", jobs=(2, 246))
run("2 jobs + late beta", jobs=(2, 246), tail=True)
run("1 job nseg=2 + late beta", jobs=(2,), tail=True)
run("beta factor, no jobs", tail=True, terms=1)
