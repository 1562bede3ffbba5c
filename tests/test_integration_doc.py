"""
The reference-side ctypes binding shown in INTEGRATION.md must work as written: the CPU test
checks that its struct layouts match the library's; the GPU test runs its Bernoulli-logits site
against the oracle.
"""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from mininf_amd import _native as nat
from oracle import logprob as lpf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def binding_namespace():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = next(b for b in re.findall(r"```python\n(.*?)```", text, re.S) if "_mi355x.py" in b)
    os.environ["MININF_AMD_LIB"] = nat.LIB_PATH
    nat.lib()
    namespace: dict = {}
    exec(compile(block, "INTEGRATION.md", "exec"), namespace)
    return namespace


def test_binding_layouts_match_library():
    ns = binding_namespace()
    sizes = [ctypes.c_size_t() for _ in range(3)]
    assert nat.lib().mi_struct_sizes(*[ctypes.byref(s) for s in sizes]) == 0
    assert [s.value for s in sizes] == [ctypes.sizeof(ns["mi_operand"]),
                                        ctypes.sizeof(ns["mi_site"]),
                                        ctypes.sizeof(ns["mi_group"])]


@pytest.mark.gpu
def test_binding_bernoulli_site(device):
    ns = binding_namespace()
    rng = np.random.default_rng(3)
    K, n = 8, 1000
    logits = rng.normal(size=(K, n)).astype(np.float32)
    x = (rng.random(n) < 0.4).astype(np.float32)
    mask = rng.random(n) > 0.25
    total, dlogits, flags = ns["bernoulli_logits_site"](
        torch.as_tensor(logits, device=device), torch.as_tensor(x, device=device),
        torch.as_tensor(mask.astype(np.uint8), device=device), 1.0, -1.0,
        torch.cuda.current_stream(device).cuda_stream)
    torch.cuda.synchronize()
    lp, dl = lpf.bernoulli_logits(logits, x[None, :])
    np.testing.assert_allclose(total.cpu().numpy(), (lp * mask).sum(1), rtol=1e-5)
    np.testing.assert_allclose(-dlogits.cpu().numpy(), dl * mask, rtol=1e-5, atol=1e-6)
    assert int(flags.cpu()[0]) == 0
