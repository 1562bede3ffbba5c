"""
The linear-predictor site kernels (mi_linear_forward) through the C ABI: the matrix-core kernel
(k_linear_mfma, v_mfma_f32_32x32x2_f32) and the VALU kernel (MI_LINEAR_VALU) against an fp64 numpy
restatement of Normal(X @ theta, sigma) / Bernoulli(logits = X @ theta) log densities and their
gradients (normal.py:88-103, bernoulli.py:121-125), over ragged row counts, particle counts that are
not multiples of 32, feature counts with one and two 32-feature tiles, masks, strided X rows and a
transposed theta.

Tolerances: totals 1e-5 relative (the north-star ELBO tolerance); gradients 1e-5 relative of the
sum of |terms|, since they are sums of terms of both signs.
"""
import ctypes

import numpy as np
import pytest
import torch

from mininf_amd import _native as nat

pytestmark = pytest.mark.gpu


def reference(family, X, theta, y, mask, sigma, site_scale, g0):
    X64, th = X.astype(np.float64), theta.astype(np.float64)
    mu = X64 @ th.T                                   # [N, K]
    m = mask.astype(np.float64)[:, None]
    y64 = np.where(mask, y, 0.0).astype(np.float64)[:, None]   # masked lanes are never read
    if family == nat.NORMAL:
        s = sigma.astype(np.float64)[None, :]
        d = y64 - mu
        lp = -d ** 2 / (2 * s ** 2) - np.log(s) - 0.5 * np.log(2 * np.pi)
        dmu = d / s ** 2
        dsig = d ** 2 / s ** 3 - 1 / s
    else:
        lp = y64 * mu - np.logaddexp(0.0, mu)
        dmu = y64 - 1 / (1 + np.exp(-mu))
        dsig = np.zeros_like(mu)
    total = site_scale * (m * lp).sum(0)
    dtheta = g0 * site_scale * ((m * dmu).T @ X64)    # [K, P]
    dsigma = g0 * site_scale * (m * dsig).sum(0)
    bound = site_scale * (np.abs(m * dmu).T @ np.abs(X64)) + 1e-6
    sbound = site_scale * np.abs(m * dsig).sum(0) + 1e-6
    return total, dtheta, dsigma, bound, sbound


def run(family, X, theta, y, mask, sigma, sigma_per_particle, site_scale, g0, valu):
    device = X.device
    N, P = X.shape
    K = theta.shape[0]
    L = nat.Linear()
    L.K, L.N, L.P = K, N, P
    L.family = family
    L.options = nat.LINEAR_VALU if valu else 0
    L.x = X.data_ptr()
    L.x_stride_i, L.x_stride_j = X.stride()
    L.theta = theta.data_ptr()
    L.theta_stride_k, L.theta_stride_j = theta.stride()
    L.value = y.data_ptr()
    L.value_stride_i = y.stride(0)
    if mask is not None:
        L.mask = mask.data_ptr()
        L.mask_stride_i = mask.stride(0)
    if sigma_per_particle:
        L.scale = sigma.data_ptr()
        L.scale_stride_k = sigma.stride(0)
    else:
        L.scale_constant = float(sigma[0])
    L.grad_scale = g0
    L.site_scale = site_scale
    L.compute_grads = 1
    lib = nat.lib()
    size = ctypes.c_size_t()
    nat.check(lib.mi_linear_workspace_bytes(ctypes.byref(L), ctypes.byref(size)), "workspace")
    work = torch.empty(size.value, dtype=torch.uint8, device=device)
    total = torch.empty(K, device=device)
    nslots = P + (1 if sigma_per_particle else 0)
    dslots = torch.empty((nslots, K), device=device)
    flags = torch.empty(1, dtype=torch.int32, device=device)
    nat.check(lib.mi_linear_forward(ctypes.byref(L), work.data_ptr(), size.value, total.data_ptr(),
                                    dslots.data_ptr(), flags.data_ptr(),
                                    nat.stream_handle(device)), "mi_linear_forward")
    torch.cuda.synchronize()
    return total.cpu().numpy(), dslots.cpu().numpy(), int(flags.cpu()[0])


CASES = [
    # (N, P, K, masked, per-particle sigma, row stride, transposed theta)
    (1000, 32, 256, False, False, None, False),
    (777, 32, 40, True, True, None, False),
    (300, 64, 33, False, True, None, False),
    (5000, 36, 7, True, False, None, False),
    (256, 4, 1, False, False, None, True),
    (10, 8, 65, False, True, 12, True),
    (4099, 32, 96, True, False, 40, False),
    (20000, 60, 300, False, True, None, False),
]


@pytest.mark.parametrize("family", [nat.NORMAL, nat.BERNOULLI_LOGITS])
@pytest.mark.parametrize("case", CASES, ids=[f"N{c[0]}_P{c[1]}_K{c[2]}" for c in CASES])
@pytest.mark.parametrize("valu", [False, True], ids=["mfma", "valu"])
def test_linear_kernel_matches_fp64(device, family, case, valu):
    N, P, K, masked, per_particle, row_stride, transposed = case
    if family == nat.BERNOULLI_LOGITS and per_particle:
        per_particle = False
    rng = np.random.default_rng(N + P + K)
    stride = row_stride or P
    Xfull = rng.normal(size=(N, stride)).astype(np.float32)
    X = torch.as_tensor(Xfull, device=device)[:, :P]
    theta_np = (0.3 * rng.normal(size=(K, P))).astype(np.float32)
    theta = torch.as_tensor(theta_np.T.copy(), device=device).t() if transposed else \
        torch.as_tensor(theta_np, device=device)
    if family == nat.NORMAL:
        y_np = rng.normal(size=N).astype(np.float32)
    else:
        y_np = (rng.random(N) < 0.4).astype(np.float32)
    mask_np = rng.random(N) > 0.15 if masked else np.ones(N, bool)
    if masked:
        y_np[~mask_np] = np.nan if family == nat.NORMAL else 0.5   # masked lanes are never read
    y = torch.as_tensor(y_np, device=device)
    mask = torch.as_tensor(mask_np.astype(np.uint8), device=device) if masked else None
    sigma_np = (0.5 + rng.random(K)).astype(np.float32) if per_particle else \
        np.full(K, 0.8, np.float32)
    sigma = torch.as_tensor(sigma_np, device=device)
    site_scale, g0 = 3.0, -1.0 / K
    total, dslots, flags = run(family, X, theta, y, mask, sigma, per_particle, site_scale, g0, valu)
    want, dtheta, dsigma, bound, sbound = reference(family, Xfull[:, :P], theta_np, y_np, mask_np,
                                                    sigma_np, site_scale, g0)
    assert flags == 0
    np.testing.assert_allclose(total, want, rtol=1e-5, atol=1e-6 * np.abs(want).max())
    err = np.abs(dslots[:P].T - dtheta)
    assert (err <= 1e-5 * abs(g0) * bound + 1e-7).all(), err.max()
    if per_particle:
        assert (np.abs(dslots[P] - dsigma) <= 1e-5 * abs(g0) * sbound + 1e-7).all()


def test_linear_kernel_flags(device):
    """Support and parameter violations reach the flag word on the matrix-core path."""
    N, P, K = 512, 32, 32
    X = torch.randn(N, P, device=device)
    theta = torch.randn(K, P, device=device)
    y = torch.randn(N, device=device)
    y[17] = float("nan")
    sigma = torch.full((K,), 1.0, device=device)
    sigma[3] = -1.0
    _, _, flags = run(nat.NORMAL, X, theta, y, None, sigma, True, 1.0, -1.0, False)
    assert flags == (nat.FLAG_SUPPORT | nat.FLAG_PARAM)
    yb = (torch.rand(N, device=device) < 0.5).float()
    yb[5] = 2.0
    _, _, flags = run(nat.BERNOULLI_LOGITS, X, theta, yb, None, sigma, False, 1.0, -1.0, False)
    assert flags == nat.FLAG_SUPPORT
