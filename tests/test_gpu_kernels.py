"""
Kernel-level parity of the HIP path (through the C ABI / engine) against the oracle and the golden
per-family tables produced by the reference's torch.distributions arithmetic.
"""
import ctypes
import os

import numpy as np
import pytest
import torch
from torch.distributions import Bernoulli, Beta, Normal

import mininf_amd as mi
from mininf_amd import _native as nat, engine, guide
from mininf_amd.particles import SiteRecord
from oracle import build as oracle_build, elbo as oracle, logprob as lpf
from tests.conftest import golden

pytestmark = pytest.mark.gpu


def launch(family, roles, value, device, mask=None, scale=1.0, K=None, N=None, g0=-1.0):
    """
    Run a one-site group: `roles` are [K, 1] (per-particle) or [K, N] tensors, `value` [K, N] or
    [N] (shared). Returns (total [K], grads per role, slot grads).
    """
    views = []
    for t in roles + [value]:
        if t.dim() == 1:
            views.append(engine._View(t.reshape(1, -1).expand(K, t.shape[0]), 0, t.stride(0)))
        elif t.shape[1] == 1:
            views.append(engine._View(t, t.stride(0), 0))
        else:
            views.append(engine._View(t, t.stride(0), t.stride(1)))
    site = SiteRecord("s", family, [], torch.Size([N]), scale, None, family)
    launcher = engine._GroupLauncher(K, N, g0, device, per_site=True)
    mview = None if mask is None else engine._View(mask, 0, mask.stride(0))
    assert launcher.try_add(site, views, mview)
    total, site_lp, grads, slot_grad, flags = launcher.run(True)
    torch.cuda.synchronize()
    return total.cpu(), grads, slot_grad.cpu(), flags.cpu(), launcher


def test_philox_device_matches_c_oracle(device):
    lib = oracle_build.load()
    ctrs = np.array([[0, 0, 0, 0], [0xFFFFFFFF] * 4, [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
                     [1, 2, 3, 4]], dtype=np.uint32)
    keys = [(0, 0), (0xFFFFFFFF, 0xFFFFFFFF), (0xA4093822, 0x299F31D0), (5, 6)]
    for ctr, (k0, k1) in zip(ctrs, keys):
        c = torch.as_tensor(ctr.astype(np.int64)).to(torch.int32).to(device)
        out = torch.empty(4, dtype=torch.int32, device=device)
        nat.check(nat.lib().mi_philox4x32(c.data_ptr(), 1, k0, k1, out.data_ptr(), None), "philox")
        want = (ctypes.c_uint32 * 4)()
        lib.oracle_philox4x32_10((ctypes.c_uint32 * 4)(*ctr.tolist()), k0, k1, want)
        got = out.cpu().numpy().astype(np.uint32)
        assert got.tolist() == list(want)
    K, N = 8, 1000
    dev = torch.empty(K, N, device=device)
    nat.check(nat.lib().mi_philox_normal(K, N, 1234, 7, 2, 5, dev.data_ptr(), None), "normals")
    host = np.empty((K, N), np.float32)
    lib.oracle_guide_normals(K, N, 1234, 7, 2, 5, host.ctypes.data)
    np.testing.assert_allclose(dev.cpu().numpy(), host, rtol=0, atol=2e-5)


@pytest.mark.parametrize("mode", ["particle", "dense"])
def test_family_tables(device, mode):
    f = golden("families.npz")

    def rows(x):
        t = torch.as_tensor(x, dtype=torch.float32, device=device)
        return (t.reshape(-1, 1) if mode == "particle" else t.reshape(1, -1)).clone() \
            .requires_grad_()

    cases = [
        ("bernoulli_probs", [f["bern_p"]], f["bern_v"], f["bern_lp"], [f["bern_dp"]]),
        ("bernoulli_logits", [f["bernl_l"]], f["bernl_v"], f["bernl_lp"], [f["bernl_dl"]]),
        ("normal", [f["norm_loc"], f["norm_scale"]], f["norm_v"], f["norm_lp"],
         [f["norm_dloc"], f["norm_dscale"]]),
        ("beta", [f["beta_a"], f["beta_b"]], f["beta_v"], f["beta_lp"],
         [f["beta_da"], f["beta_db"]]),
    ]
    for family, params, value, want_lp, want_grads in cases:
        n = len(value)
        K, N = (n, 1) if mode == "particle" else (1, n)
        roles = [rows(p) for p in params]
        val = torch.as_tensor(value, dtype=torch.float32, device=device)
        val = val.reshape(K, N).contiguous()
        total, grads, slot_grad, flags, launcher = launch(family, roles, val, device, K=K, N=N)
        if mode == "particle":
            # 1e-5 relative (the north-star tolerance): Beta's lgamma(a+b) - lgamma(a) - lgamma(b)
            # cancels in float32 in both implementations.
            np.testing.assert_allclose(total.numpy(), want_lp, rtol=1e-5, atol=2e-6)
            for j, want in enumerate(want_grads):
                ok = np.isfinite(want)
                # slot gradients come pre-multiplied by the group's grad_scale (g0 = -1 here)
                np.testing.assert_allclose(-slot_grad[j].numpy()[ok], want[ok], rtol=2e-5, atol=2e-5)
        else:
            np.testing.assert_allclose(total.numpy()[0], want_lp.sum(), rtol=1e-5)
            for grad, want in zip(grads, want_grads):
                ok = np.isfinite(want)
                np.testing.assert_allclose(-grad.cpu().numpy()[0][ok], want[ok], rtol=2e-5,
                                           atol=2e-5)
        assert (flags == 0).all()


def test_bcast_site_matches_oracle(device):
    rng = np.random.default_rng(0)
    K, N = 300, 5000
    x = (rng.random(N) < 0.6).astype(np.float32)
    p = rng.random(K).astype(np.float32) * 0.98 + 0.01
    probs = torch.as_tensor(p, device=device).reshape(K, 1).requires_grad_()
    total, _, slot, flags, launcher = launch("bernoulli_probs", [probs],
                                             torch.as_tensor(x, device=device), device, K=K, N=N)
    want_lp, want_dp = lpf.bernoulli_probs(p[:, None], x[None, :])
    np.testing.assert_allclose(total.numpy(), want_lp.sum(1), rtol=1e-6)
    # slot gradients are pre-multiplied by grad_scale (g0 = -1 in `launch`)
    np.testing.assert_allclose(-slot[0].numpy(), want_dp.sum(1), rtol=1e-5)
    loc = torch.as_tensor(rng.normal(size=(K, 1)).astype(np.float32), device=device).requires_grad_()
    sd = torch.as_tensor(rng.random((K, 1)).astype(np.float32) + 0.5, device=device).requires_grad_()
    y = rng.normal(size=N).astype(np.float32)
    mask = torch.as_tensor(rng.random(N) > 0.3, device=device)
    total, _, slot, flags, _ = launch("normal", [loc, sd], torch.as_tensor(y, device=device),
                                      device, mask=mask, K=K, N=N)
    m = mask.cpu().numpy()
    lp, dl, ds, _ = lpf.normal(loc.detach().cpu().numpy(), sd.detach().cpu().numpy(), y[None, :])
    np.testing.assert_allclose(total.numpy(), (lp * m).sum(1), rtol=1e-6)
    # d/dscale = sum (z^2 - 1) / scale cancels for some particles: compare on the vector's scale.
    for got, want in ((-slot[0].numpy(), (dl * m).sum(1)), (-slot[1].numpy(), (ds * m).sum(1))):
        assert np.abs(got - want).max() <= 1e-5 * np.abs(want).max()


@pytest.mark.parametrize("family", ["bernoulli_probs", "bernoulli_logits"])
@pytest.mark.parametrize("N,K", [(5000, 300), (2048 + 257, 2100), (1024 + 1, 64), (4096 * 3, 513)])
@pytest.mark.parametrize("kernel", ["smem", "lds"])
def test_bcast_bernoulli_kernels(device, family, N, K, kernel):
    """
    Bernoulli BCAST sites (per-particle parameter against shared data) on both kernels: unmasked
    contiguous data runs k_site_bcast_smem (scalar-unit loads, whole 256-element blocks plus an
    odd or even tail), a mask -- all true here, so the answers are the same -- the LDS kernel.
    Particle counts cover a partial particle block and more than one block.
    """
    rng = np.random.default_rng(N + K)
    x = (rng.random(N) < 0.6).astype(np.float32)
    if family == "bernoulli_probs":
        a = rng.random(K).astype(np.float32) * 0.98 + 0.01
        want_lp, want_d = lpf.bernoulli_probs(a[:, None], x[None, :])
    else:
        a = (3 * rng.normal(size=K)).astype(np.float32)
        want_lp, want_d = lpf.bernoulli_logits(a[:, None], x[None, :])
    param = torch.as_tensor(a, device=device).reshape(K, 1).requires_grad_()
    mask = torch.ones(N, dtype=torch.bool, device=device) if kernel == "lds" else None
    total, _, slot, flags, _ = launch(family, [param], torch.as_tensor(x, device=device), device,
                                      mask=mask, K=K, N=N)
    np.testing.assert_allclose(total.numpy(), want_lp.sum(1), rtol=1e-6, atol=1e-6 * N)
    g = want_d.sum(1)
    assert np.abs(-slot[0].numpy() - g).max() <= 1e-5 * np.abs(g).max()
    assert (flags == 0).all()


def c5_case(device, n=3000, K=24):
    rng = np.random.default_rng(1)
    mask = torch.as_tensor(rng.random(n) > 0.2, device=device)
    y = torch.as_tensor(rng.normal(size=n).astype(np.float32), device=device)
    b = torch.as_tensor((rng.random(n) < 0.5).astype(np.float32), device=device)

    def model():
        mu = mi.sample("mu", Normal(0, 1))
        z = mi.sample("z", Normal(mu, 1), sample_shape=[n])
        mi.sample("y", Normal(z, 0.5))
        mi.sample("b", Bernoulli(logits=z))

    approx = mi.nn.ParameterizedFactorizedDistribution(
        mu=mi.nn.ParameterizedDistribution(Normal, loc=0.2, scale=0.7),
        z=mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(n), scale=torch.ones(n) * 0.9),
    ).to(device)
    noise = {"mu": torch.as_tensor(rng.normal(size=K).astype(np.float32), device=device),
             "z": torch.as_tensor(rng.normal(size=(K, n)).astype(np.float32), device=device)}
    cond = mi.condition(model, y=torch.masked.as_masked_tensor(y, mask),
                        b=torch.masked.as_masked_tensor(b, mask))
    return cond, approx, noise, (y, b, mask), K


def run_elbo(cond, approx, noise, K):
    for p in approx.parameters():
        p.grad = None
    value = mi.nn.EvidenceLowerBoundLoss(num_particles=K)(cond, approx(), _noise=noise)
    value.backward()
    return float(value), {n: p.grad.detach().cpu().numpy().copy()
                          for n, p in approx.named_parameters()}


def test_specialised_and_generic_kernels_agree(device):
    cond, approx, noise, _, K = c5_case(device)
    jit_loss, jit_grads = run_elbo(cond, approx, noise, K)
    os.environ["MININF_AMD_JIT"] = "0"
    try:
        gen_loss, gen_grads = run_elbo(cond, approx, noise, K)
    finally:
        del os.environ["MININF_AMD_JIT"]
    assert abs(jit_loss - gen_loss) <= 1e-6 * abs(gen_loss)
    for name in gen_grads:
        np.testing.assert_allclose(jit_grads[name], gen_grads[name], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("n", [3000, 2048, 300, 1])
def test_c5_against_oracle(device, n):
    """
    Row-layout site program at a ragged size (shifted last segment), an exact multiple of the
    segment, and sizes below one segment (clamped-index program).
    """
    cond, approx, noise, (y, b, mask), K = c5_case(device, n=n)
    loss, grads = run_elbo(cond, approx, noise, K)
    n = y.shape[0]
    ref = oracle.hierarchical_masked_elbo(y.cpu(), b.cpu(), mask.cpu(), 0.2, 0.7, np.zeros(n),
                                          np.full(n, 0.9, np.float32), noise["mu"].cpu(),
                                          noise["z"].cpu())
    assert abs(loss - ref["loss"]) <= 1e-5 * abs(ref["loss"])
    np.testing.assert_allclose(grads["z.distribution_parameters.loc"], ref["grad_z_loc"],
                               rtol=1e-5, atol=1e-5 * np.abs(ref["grad_z_loc"]).max())
    np.testing.assert_allclose(grads["z.distribution_parameters.scale"], ref["grad_z_scale"],
                               rtol=1e-5, atol=1e-5 * np.abs(ref["grad_z_scale"]).max())


def test_full_size_c2_closed_form(device):
    """
    C2 at full size (n = 1e6, K = 4096): the oracle evaluates the Bernoulli site through its
    sufficient statistics in float64, so it finishes instantly at this size.
    """
    n, K = 1_000_000, 4096
    gen = torch.Generator().manual_seed(0)
    x = (torch.rand(n, generator=gen) < 0.7).float()
    draws = torch.distributions.Beta(torch.tensor(2.5), torch.tensor(1.5)).sample((K,))

    def model():
        theta = mi.sample("theta", Beta(2, 2))
        mi.sample("x", Bernoulli(theta), sample_shape=[n])

    approx = mi.nn.ParameterizedDistribution(Beta, concentration1=2.5,
                                             concentration0=1.5).to(device)
    value = mi.nn.EvidenceLowerBoundLoss(num_particles=K)(
        mi.condition(model, x=x.to(device)), {"theta": approx()},
        _noise={"theta": draws.to(device)})
    value.backward()
    ref = oracle.beta_bernoulli_elbo(x.numpy(), 2, 2, 2.5, 1.5, draws.numpy())
    assert abs(float(value) - ref["loss"]) <= 1e-5 * abs(ref["loss"])
    g = approx.distribution_parameters
    assert abs(float(g["concentration1"].grad) - ref["grad_u_concentration1"]) <= \
        1e-5 * abs(ref["grad_u_concentration1"])
    assert abs(float(g["concentration0"].grad) - ref["grad_u_concentration0"]) <= \
        1e-5 * abs(ref["grad_u_concentration0"])


def test_beta_guide_backward_against_oracle(device):
    rng = np.random.default_rng(3)
    K, N = 512, 7
    c1 = torch.as_tensor(rng.random(N).astype(np.float32) * 5 + 0.3, device=device)
    c0 = torch.as_tensor(rng.random(N).astype(np.float32) * 9 + 0.3, device=device)
    x = torch.distributions.Beta(c1.cpu(), c0.cpu()).sample((K,)).clamp(1e-4, 1 - 1e-4)
    c1p, c0p = c1.clone().requires_grad_(), c0.clone().requires_grad_()
    cfg = guide.DrawConfig(K=K, seed=0, step=0, stream_id=0, particle_offset=0,
                           noise=x.to(device))
    draws = guide.draw(Beta(c1p, c0p), cfg)
    weights = torch.as_tensor(rng.normal(size=(K, N)).astype(np.float32), device=device)
    (draws * weights).sum().backward()
    xs, w = x.double().numpy(), weights.cpu().double().numpy()
    for i in range(N):
        d1, d0 = lpf.beta_draw_grads(xs[:, i], float(c1[i]), float(c0[i]))
        np.testing.assert_allclose(float(c1p.grad[i]), (w[:, i] * d1).sum(), rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(float(c0p.grad[i]), (w[:, i] * d0).sum(), rtol=1e-4, atol=1e-5)


def test_guide_draws_statistics_and_sharding(device):
    K, N = 4096, 64
    loc = torch.linspace(-1, 1, N, device=device)
    scale = torch.linspace(0.5, 2, N, device=device)
    full = guide.draw(Normal(loc, scale), guide.DrawConfig(K, 9, 3, 0, 0))
    halves = [guide.draw(Normal(loc, scale), guide.DrawConfig(K // 2, 9, 3, 0, off))
              for off in (0, K // 2)]
    torch.testing.assert_close(torch.cat(halves), full, rtol=0, atol=0)
    z = (full - loc) / scale
    assert abs(float(z.mean())) < 0.01 and abs(float(z.std()) - 1) < 0.01
    c1, c0 = torch.full((N,), 2.0, device=device), torch.full((N,), 5.0, device=device)
    x = guide.draw(Beta(c1, c0), guide.DrawConfig(K, 9, 3, 1, 0))
    assert abs(float(x.mean()) - 2 / 7) < 0.005
    assert abs(float(x.var()) - 2 * 5 / (49 * 8)) < 0.002
    assert float(x.min()) > 0 and float(x.max()) < 1


def test_validation_errors_are_raised(device):
    def model():
        theta = mi.sample("theta", Beta(2, 2))
        mi.sample("x", Bernoulli(theta), sample_shape=[5])

    approx = mi.nn.ParameterizedDistribution(Beta, concentration1=2.0,
                                             concentration0=2.0).to(device)
    bad = torch.tensor([0.0, 1.0, 2.0, 1.0, 0.0], device=device)
    with pytest.raises(ValueError, match="is not in the support"):
        mi.nn.EvidenceLowerBoundLoss(num_particles=8)(mi.condition(model, x=bad),
                                                      {"theta": approx()})

    def normal_model():
        mi.sample("y", Normal(0.0, mi.value("s")), sample_shape=[3])

    with pytest.raises(ValueError, match="satisfy"):
        loss = mi.nn.EvidenceLowerBoundLoss(num_particles=4)
        loss(mi.condition(normal_model, y=torch.zeros(3, device=device),
                          s=torch.tensor(-1.0, device=device)),
             {"q": Normal(torch.zeros((), device=device), 1.0)})


def _two_factor_case(device, n=700, K=16):
    rng = np.random.default_rng(5)
    x = torch.as_tensor((rng.random(n) < 0.6).astype(np.float32), device=device)
    y = torch.as_tensor(rng.normal(size=n).astype(np.float32), device=device)

    def model():
        a = mi.sample("a", Beta(2.0, 3.0), sample_shape=[n])
        b = mi.sample("b", Normal(0.0, 1.0), sample_shape=[n])
        mi.sample("x", Bernoulli(a))
        mi.sample("y", Normal(b, 1.0))

    approx = mi.nn.ParameterizedFactorizedDistribution(
        a=mi.nn.ParameterizedDistribution(Beta, concentration1=torch.full((n,), 1.5),
                                          concentration0=torch.linspace(0.5, 4.0, n)),
        b=mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(n),
                                          scale=torch.linspace(0.2, 2.0, n)),
    ).to(device)
    noise = {"a": torch.as_tensor(rng.beta(1.5, 2.0, size=(K, n)).astype(np.float32),
                                  device=device),
             "b": torch.as_tensor(rng.normal(size=(K, n)).astype(np.float32), device=device)}
    return mi.condition(model, x=x, y=y), approx, noise, K


def test_fused_elbo_matches_unfused_composition(device):
    """
    The fused ELBO node (site groups + mi_elbo_forward/backward entropy and reduction) against the
    unfused composition: per-particle log joint (engine.log_joint) and torch.distributions entropy.
    """
    from mininf_amd import engine, guide, particles
    cond, approx, noise, K = _two_factor_case(device)
    loss = mi.nn.EvidenceLowerBoundLoss(num_particles=K)(cond, approx(), _noise=noise)
    loss.backward()
    fused = {k: p.grad.clone() for k, p in approx.named_parameters()}
    for p in approx.parameters():
        p.grad = None

    q = approx()
    samples = guide.draw_all(q, K, 0, 0, 0, noise)
    trace = particles.trace_particles(cond, samples, K)
    g0 = float(torch.tensor(-1.0 / K, dtype=torch.float32))
    joint = engine.log_joint(trace, g0, device)
    ref = (joint.total * g0).sum() - q.entropy()
    ref.backward()
    assert abs(float(loss) - float(ref)) <= 1e-5 * abs(float(ref))
    for name, p in approx.named_parameters():
        torch.testing.assert_close(fused[name], p.grad, rtol=1e-5, atol=1e-6)


def test_fused_elbo_scales_with_upstream(device):
    cond, approx, noise, K = _two_factor_case(device, n=300, K=8)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K)
    loss_fn(cond, approx(), _noise=noise).backward()
    base = {k: p.grad.clone() for k, p in approx.named_parameters()}
    for p in approx.parameters():
        p.grad = None
    (2.5 * loss_fn(cond, approx(), _noise=noise)).backward()
    for name, p in approx.named_parameters():
        torch.testing.assert_close(p.grad, 2.5 * base[name], rtol=1e-5, atol=1e-6)


def test_log_likelihood_loss_on_device(device):
    """
    LogLikelihoodLoss with device parameters runs the site kernels (K = 1); it must match the
    reference-semantics host evaluation (LogProbTracer on the CPU) in value and gradients.
    """
    rng = np.random.default_rng(9)
    n, p = 2000, 4
    X = torch.as_tensor(rng.normal(size=(n, p)).astype(np.float32))
    y = torch.as_tensor(rng.normal(size=n).astype(np.float32))
    b = torch.as_tensor((rng.random(n) < 0.4).astype(np.float32))

    def make_model(Xd):
        def model():
            theta = mi.sample("theta", Normal(0.0, 1.0), sample_shape=p)
            q = mi.sample("q", Beta(2.0, 3.0))
            mi.sample("X", Normal(0.0, 1.0), sample_shape=(n, p))
            mi.sample("y", Normal(Xd @ theta, 1.5))
            mi.sample("b", Bernoulli(q), sample_shape=[n])
        return model

    def evaluate(dev):
        theta = torch.tensor([0.3, -0.2, 0.5, 1.0], device=dev, requires_grad=True)
        q = torch.tensor(0.35, device=dev, requires_grad=True)
        loss = mi.nn.LogLikelihoodLoss()(
            make_model(X.to(dev)),
            {"theta": theta, "q": q, "X": X.to(dev), "y": y.to(dev), "b": b.to(dev)})
        loss.backward()
        return float(loss), theta.grad.cpu(), q.grad.cpu()

    host = evaluate(torch.device("cpu"))
    dev = evaluate(device)
    assert abs(dev[0] - host[0]) <= 1e-5 * abs(host[0])
    torch.testing.assert_close(dev[1], host[1], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dev[2], host[2], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("family", ["normal_const", "normal_sigma", "bernoulli"])
@pytest.mark.parametrize("p,K", [(5, 12), (32, 40)], ids=["valu", "mfma"])
def test_linear_site_matches_materialised_product(device, family, p, K, monkeypatch):
    """
    The fused linear site (X @ theta evaluated in mi_linear_forward: the VALU kernel for P = 5, the
    matrix-core kernel for P = 32) against the same model with the product materialised by the
    model's matmul (MININF_AMD_DEFER_MATMUL=0): ELBO value and guide gradients, masked data and a
    minibatch scale included.
    """
    rng = np.random.default_rng(4)
    n = 3000
    X = torch.as_tensor(rng.normal(size=(n, p)).astype(np.float32), device=device)
    mask = torch.as_tensor(rng.random(n) > 0.1, device=device)
    if family == "bernoulli":
        y = torch.as_tensor((rng.random(n) < 0.4).astype(np.float32), device=device)
    else:
        y = torch.as_tensor(rng.normal(size=n).astype(np.float32), device=device)

    def model():
        theta = mi.sample("theta", Normal(0.0, 1.0), sample_shape=p)
        sigma = mi.sample("sigma", torch.distributions.Gamma(2.0, 2.0)) \
            if family == "normal_sigma" else 0.7
        with mi.batch(2 * n):
            if family == "bernoulli":
                mi.sample("y", Bernoulli(logits=X @ theta))
            else:
                mi.sample("y", Normal(X @ theta, sigma))

    guide = {"theta": mi.nn.ParameterizedDistribution(Normal, loc=torch.full((p,), 0.1),
                                                      scale=torch.full((p,), 0.5))}
    noise = {"theta": torch.as_tensor(rng.normal(size=(K, p)).astype(np.float32), device=device)}
    if family == "normal_sigma":
        guide["sigma"] = mi.nn.ParameterizedDistribution(Normal, loc=1.0, scale=0.1)
        noise["sigma"] = torch.as_tensor(rng.normal(size=K).astype(np.float32), device=device)
    approx = mi.nn.ParameterizedFactorizedDistribution(guide).to(device)
    data = y if family != "normal_const" else torch.masked.as_masked_tensor(y, mask)
    cond = mi.condition(model, y=data if family == "normal_const" else y)

    def run():
        for q in approx.parameters():
            q.grad = None
        loss = mi.nn.EvidenceLowerBoundLoss(num_particles=K)(cond, approx(), _noise=noise)
        loss.backward()
        return float(loss), {k: q.grad.detach().clone() for k, q in approx.named_parameters()}

    if family == "normal_const":
        # masked data and a batch scale cannot be combined (core.py:263-264): drop the batch
        def model():  # noqa: F811
            theta = mi.sample("theta", Normal(0.0, 1.0), sample_shape=p)
            mi.sample("y", Normal(X @ theta, 0.7))
        cond = mi.condition(model, y=data)
    fused = run()
    monkeypatch.setenv("MININF_AMD_DEFER_MATMUL", "0")
    plain = run()
    assert abs(fused[0] - plain[0]) <= 1e-5 * abs(plain[0])
    for name in plain[1]:
        # gradients are sums of terms of both signs: the absolute tolerance follows their scale
        scale = max(1.0, float(plain[1][name].abs().max()))
        torch.testing.assert_close(fused[1][name], plain[1][name], rtol=1e-5, atol=1e-5 * scale)


def _hierarchical(device, n, use_exp=False):
    rng = np.random.default_rng(6)
    mask = torch.as_tensor(rng.random(n) > 0.2, device=device)
    y = torch.as_tensor(rng.normal(size=n).astype(np.float32), device=device)
    b = torch.as_tensor((rng.random(n) < 0.5).astype(np.float32), device=device)

    def model():
        mu = mi.sample("mu", Normal(0.0, 1.0))
        z = mi.sample("z", Normal(mu, 1.0), sample_shape=[n])
        mi.sample("y", Normal(z.exp() if use_exp else z, 0.5))
        mi.sample("b", Bernoulli(logits=z))

    approx = mi.nn.ParameterizedFactorizedDistribution(
        mu=mi.nn.ParameterizedDistribution(Normal, loc=0.2, scale=0.7),
        z=mi.nn.ParameterizedDistribution(Normal, loc=torch.linspace(-1, 1, n),
                                          scale=torch.linspace(0.5, 1.5, n)),
    ).to(device)
    cond = mi.condition(model, y=torch.masked.as_masked_tensor(y, mask),
                        b=torch.masked.as_masked_tensor(b, mask))
    return cond, approx


@pytest.mark.parametrize("n,use_exp", [(4096, False), (3000, False), (3001, False),
                                       (4096, True)])
def test_fused_guide_draw_matches_materialised(device, n, use_exp, monkeypatch):
    """
    A large Normal guide factor drawn inside the site kernel (mi_draw: z and dz never stored)
    against the materialised draw (MININF_AMD_FUSE_DRAWS=0): the same Philox eps, so the ELBO
    and its gradients agree up to summation order. n = 3001 (not a multiple of 4) and a model
    that uses z outside a site (z.exp()) take the materialised path by themselves.
    """
    cond, approx = _hierarchical(device, n, use_exp)
    K = 24

    def run():
        for q in approx.parameters():
            q.grad = None
        loss = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=5)(cond, approx())
        loss.backward()
        return float(loss), {k: q.grad.detach().clone() for k, q in approx.named_parameters()}

    fused = run()
    monkeypatch.setenv("MININF_AMD_FUSE_DRAWS", "0")
    plain = run()
    assert abs(fused[0] - plain[0]) <= 1e-5 * abs(plain[0])
    for name in plain[1]:
        torch.testing.assert_close(fused[1][name], plain[1][name], rtol=1e-5, atol=1e-5)


def _absorb_cases(device, case):
    """Models whose guide draws the ELBO backward can absorb (or must not)."""
    rng = np.random.default_rng(12)
    if case == "beta_scalar":   # C2-shaped: one Beta factor, many particles (cross-slice sums)
        x = torch.as_tensor((rng.random(5000) < 0.7).astype(np.float32), device=device)

        def model():
            theta = mi.sample("theta", Beta(2.0, 2.0))
            mi.sample("x", Bernoulli(theta), sample_shape=[5000])
        approx = mi.nn.ParameterizedFactorizedDistribution(
            theta=mi.nn.ParameterizedDistribution(Beta, concentration1=1.7, concentration0=2.6))
        return mi.condition(model, x=x), approx.to(device), 2048
    if case == "two_factor":
        cond, approx, _, K = _two_factor_case(device, n=700, K=16)
        return cond, approx, K
    if case in ("linear", "linear_sigma"):
        n, p = 4000, 6
        X = torch.as_tensor(rng.normal(size=(n, p)).astype(np.float32), device=device)
        y = torch.as_tensor(rng.normal(size=n).astype(np.float32), device=device)

        def model():
            theta = mi.sample("theta", Normal(0.0, 1.0), sample_shape=p)
            sigma = mi.sample("sigma", Normal(1.0, 0.1)) if case == "linear_sigma" else 0.8
            mi.sample("y", Normal(X @ theta, sigma))
        guide = {"theta": mi.nn.ParameterizedDistribution(Normal, loc=torch.full((p,), 0.1),
                                                          scale=torch.full((p,), 0.5))}
        if case == "linear_sigma":
            guide["sigma"] = mi.nn.ParameterizedDistribution(Normal, loc=1.0, scale=0.05)
        return mi.condition(model, y=y), mi.nn.ParameterizedFactorizedDistribution(guide) \
            .to(device), 64
    if case == "hierarchical":    # fused draw (partials) + a scalar factor used as a loc (slot)
        cond, approx = _hierarchical(device, 4096)
        return cond, approx, 48
    cond, approx = _hierarchical(device, 2048, use_exp=True)   # z.exp(): must not be absorbed
    return cond, approx, 16


@pytest.mark.parametrize("case", ["beta_scalar", "beta_scalar_inline", "beta_scalar_dgrad",
                                  "two_factor", "linear",
                                  "linear_sigma", "hierarchical", "exp_use"])
def test_absorbed_draws_match_autograd(device, case, monkeypatch):
    """
    Guide draws whose backward the ELBO kernel absorbs (mi_factor draw_kind: Beta implicit
    gradient, Normal eps regeneration, fused-draw partials; entropy and exp transform folded in)
    against the same step with the draws' backward left to autograd (MININF_AMD_ABSORB=0).
    Beta: the implicit-gradient factors computed by extra workgroups of the site launch (mi_side,
    the default), inside mi_elbo_forward (beta_scalar_inline, MININF_AMD_BETA_SIDE=0), or by
    mi_beta_dgrad on a side stream (beta_scalar_dgrad, MININF_AMD_BETA_DGRAD=1).
    """
    if case == "beta_scalar_dgrad":
        monkeypatch.setenv("MININF_AMD_BETA_DGRAD", "1")
        case = "beta_scalar"
    if case == "beta_scalar_inline":
        monkeypatch.setenv("MININF_AMD_BETA_SIDE", "0")
        case = "beta_scalar"
    cond, approx, K = _absorb_cases(device, case)

    def run(scale=1.0):
        for q in approx.parameters():
            q.grad = None
        loss = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=3)(cond, approx())
        (scale * loss).backward()
        return float(loss), {k: q.grad.detach().clone() for k, q in approx.named_parameters()}

    absorbed = run()
    scaled = run(-1.5)
    monkeypatch.setenv("MININF_AMD_ABSORB", "0")
    plain = run()
    assert abs(absorbed[0] - plain[0]) <= 1e-5 * abs(plain[0])
    for name in plain[1]:
        torch.testing.assert_close(absorbed[1][name], plain[1][name], rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(scaled[1][name], -1.5 * plain[1][name], rtol=1e-5, atol=1e-5)


def test_absorption_plan(device):
    """Which factors the ELBO absorbs: all of the hierarchical model's, none when z is used
    outside the site kernels."""
    from mininf_amd import engine
    seen = []
    original = engine.plan_absorption

    def spy(*args, **kwargs):
        out = original(*args, **kwargs)
        seen.append(sorted((args[0][i].name, p.kind) for i, p in out.items()))
        return out
    engine.plan_absorption = spy
    try:
        for case in ("hierarchical", "exp_use", "beta_scalar", "linear"):
            cond, approx, K = _absorb_cases(device, case)
            mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=3)(cond, approx()).backward()
    finally:
        engine.plan_absorption = original
    import mininf_amd._native as nat
    assert seen[0] == [("mu", nat.DRAW_SOURCES), ("z", nat.DRAW_PARTIALS)]
    assert ("z", nat.DRAW_SOURCES) not in seen[1] and ("z", nat.DRAW_PARTIALS) not in seen[1]
    assert seen[2] == [("theta", nat.DRAW_SOURCES)]
    assert seen[3] == [("theta", nat.DRAW_SOURCES)]


def test_fused_beta_guide_matches_torch_construction(device):
    """
    ParameterizedDistribution(Beta) on the device builds its interleaved concentration array in one
    launch (mi_transform_params) and assembles the Beta as Beta.__init__ does: same parameters,
    shapes, log densities, entropy and gradients as the host module's torch construction.
    """
    c1 = torch.tensor([0.7, 2.5, 9.0])
    c0 = torch.tensor([1.3, 0.4, 6.0])
    host = mi.nn.ParameterizedDistribution(Beta, concentration1=c1, concentration0=c0)
    dev = mi.nn.ParameterizedDistribution(Beta, concentration1=c1, concentration0=c0).to(device)
    qh, qd = host(), dev()
    assert type(qd) is Beta and qd.batch_shape == qh.batch_shape and qd.event_shape == ()
    torch.testing.assert_close(qd.concentration1.cpu(), qh.concentration1, rtol=1e-6, atol=0)
    torch.testing.assert_close(qd.concentration0.cpu(), qh.concentration0, rtol=1e-6, atol=0)
    x = torch.tensor([0.2, 0.5, 0.9])
    (qh.log_prob(x).sum() + qh.entropy().sum()).backward()
    (qd.log_prob(x.to(device)).sum() + qd.entropy().sum()).backward()
    for name, p in host.distribution_parameters.items():
        torch.testing.assert_close(dev.distribution_parameters[name].grad.cpu(), p.grad,
                                   rtol=1e-5, atol=1e-6)
    bad = mi.nn.ParameterizedDistribution(Beta, concentration1=c1, concentration0=c0,
                                          validate_args=True).to(device)
    bad.distribution_parameters["concentration1"].data.fill_(float("nan"))
    with pytest.raises(ValueError, match="concentration"):   # Dirichlet's check, as in torch
        bad()


@pytest.mark.parametrize("N,K", [(5000, 2048), (3000, 96)])
def test_bcast_side_job_matches_beta_dgrad(device, N, K):
    """
    The Beta implicit-gradient factors carried as extra workgroups of the BCAST site launch
    (mi_side) are bit-identical to mi_beta_dgrad's, and the site results are unchanged by them.
    """
    rng = np.random.default_rng(N)
    x = (rng.random(N) < 0.6).astype(np.float32)
    conc = torch.as_tensor([[1.7, 2.6]], dtype=torch.float32, device=device)
    draws = torch.distributions.Beta(torch.tensor(1.7), torch.tensor(2.6)).sample((K, 1))
    draws = draws.to(device).contiguous()
    probs = draws.reshape(K, 1).clone().requires_grad_()
    base = launch("bernoulli_probs", [probs], torch.as_tensor(x, device=device), device, K=K, N=N)

    views = [engine._View(probs, probs.stride(0), 0),
             engine._View(torch.as_tensor(x, device=device).reshape(1, -1).expand(K, N), 0, 1)]
    site = SiteRecord("s", "bernoulli_probs", [], torch.Size([N]), 1.0, None, "bernoulli_probs")
    launcher = engine._GroupLauncher(K, N, -1.0, device, per_site=True)
    assert launcher.try_add(site, views, None)
    launcher.side = (draws, conc)
    total, _, _, slot, flags = launcher.run(True)
    torch.cuda.synchronize()
    assert launcher.side_out is not None, "the BCAST kernel should carry the side job"
    want = torch.empty((K, 1, 2), dtype=torch.float64, device=device)
    c = conc.data_ptr()
    nat.check(nat.lib().mi_beta_dgrad(draws.data_ptr(), c, 2, c + 4, 2, K, 1, want.data_ptr(),
                                      None), "mi_beta_dgrad")
    torch.cuda.synchronize()
    assert torch.equal(launcher.side_out, want)
    assert torch.equal(total.cpu(), base[0]) and torch.equal(slot.cpu(), base[2])
    assert int(flags.cpu().max()) == 0


def test_interleaved_beta_elbos_keep_their_own_sums(device):
    """
    Two ELBO evaluations with absorbed Beta draws before one backward (loss1 + loss2, gradient
    accumulation, a logging ELBO mid-step): each evaluation's forward sums (mi_factor.saved) stay
    its own, also when the second needs a larger ELBO workspace than the first.
    Gradients equal those of separate backwards.
    """
    rng = np.random.default_rng(5)
    n, nv = 5000, 3000
    x = torch.as_tensor((rng.random(n) < 0.7).astype(np.float32), device=device)
    xv = torch.as_tensor((rng.random((nv,)) < 0.4).astype(np.float32), device=device)

    def scalar_model():
        theta = mi.sample("theta", Beta(2.0, 2.0))
        mi.sample("x", Bernoulli(theta), sample_shape=[n])

    def vector_model():   # per-element Beta guide: more blocks, more workspace
        theta = mi.sample("theta", Beta(2.0, 2.0), sample_shape=[nv])
        mi.sample("x", Bernoulli(theta))

    a1 = mi.nn.ParameterizedFactorizedDistribution(
        theta=mi.nn.ParameterizedDistribution(Beta, concentration1=1.7, concentration0=2.6)
    ).to(device)
    a2 = mi.nn.ParameterizedFactorizedDistribution(
        theta=mi.nn.ParameterizedDistribution(Beta, concentration1=torch.full((nv,), 1.2),
                                              concentration0=torch.full((nv,), 3.1))).to(device)
    c1, c2 = mi.condition(scalar_model, x=x), mi.condition(vector_model, x=xv)

    def losses():
        l1 = mi.nn.EvidenceLowerBoundLoss(num_particles=2048, seed=3)(c1, a1())
        l2 = mi.nn.EvidenceLowerBoundLoss(num_particles=64, seed=4)(c2, a2())
        l3 = mi.nn.EvidenceLowerBoundLoss(num_particles=512, seed=5)(c1, a1())
        return l1, l2, l3

    def grads():
        out = {f"a1.{k}": q.grad.detach().clone() for k, q in a1.named_parameters()}
        out.update({f"a2.{k}": q.grad.detach().clone() for k, q in a2.named_parameters()})
        for q in list(a1.parameters()) + list(a2.parameters()):
            q.grad = None
        return out

    for l in losses():   # separate forward/backward pairs
        l.backward()
    separate = grads()
    l1, l2, l3 = losses()   # all forwards first, then one backward
    (l1 + l2 + l3).backward()
    joint = grads()
    for name in separate:
        torch.testing.assert_close(joint[name], separate[name], rtol=1e-6, atol=1e-7)


def _categorical_abi(logits, value, device, mask=None, scale=1.0, g0=-1.0):
    """mi_categorical_forward on [K, N, C] logits: (total [K], dlogits [K, N, C], flags)."""
    K, N, C = logits.shape
    lib = nat.lib()
    size = ctypes.c_size_t()
    assert lib.mi_categorical_workspace_bytes(K, N, ctypes.byref(size)) == 0
    ws = torch.empty(max(1, size.value), dtype=torch.uint8, device=device)
    total = torch.empty(K, dtype=torch.float32, device=device)
    dlogits = torch.full_like(logits, float("nan"))   # every entry must be written
    flags = torch.empty(1, dtype=torch.int32, device=device)
    nat.check(lib.mi_categorical_forward(
        logits.data_ptr(), *logits.stride(), K, N, C, value.data_ptr(), *value.stride(),
        None if mask is None else mask.data_ptr(), 0 if mask is None else mask.stride(0),
        scale, g0, dlogits.data_ptr(), ws.data_ptr(), size.value, total.data_ptr(),
        flags.data_ptr(), None), "mi_categorical_forward")
    torch.cuda.synchronize()
    return total.cpu(), dlogits.cpu(), int(flags.cpu()[0])


@pytest.mark.parametrize("mode", ["particle", "dense"])
def test_categorical_kernel_against_golden(device, mode):
    """
    k_categorical on the reference's raw logits (golden families.npz, torch Categorical(logits=.)
    .log_prob and its autograd, categorical.py:74-78, 150-156): the kernel normalises, gathers and
    writes g0 * (onehot - softmax), the gradient with respect to the raw logits.
    """
    f = golden("families.npz")
    raw = torch.as_tensor(f["cat_logits"], device=device)            # [6, 5]
    v = torch.as_tensor(f["cat_v"], device=device)
    if mode == "particle":   # six particles, one element each
        logits, value = raw.reshape(6, 1, 5).contiguous(), v.reshape(6, 1).contiguous()
    else:                    # one particle, six elements
        logits, value = raw.reshape(1, 6, 5).contiguous(), v.reshape(1, 6).contiguous()
    total, dlogits, flags = _categorical_abi(logits, value, device)
    assert flags == 0
    want = f["cat_lp"] if mode == "particle" else np.array([f["cat_lp"].sum()])
    np.testing.assert_allclose(total.numpy(), want, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(-dlogits.reshape(6, 5).numpy(), f["cat_dlogits"], rtol=1e-5,
                               atol=1e-6)


def test_categorical_kernel_mask_and_support(device):
    """Masked rows contribute 0 to value and gradient (util.py:85-90); an observed value outside
    [0, C) sets the support flag, a masked one does not."""
    rng = np.random.default_rng(3)
    K, N, C = 3, 2000, 7
    logits = torch.as_tensor(rng.normal(size=(K, N, C)).astype(np.float32), device=device)
    v = rng.integers(0, C, size=N)
    mask = rng.random(N) > 0.3
    value = torch.as_tensor(v, device=device).reshape(1, N).expand(K, N)
    m = torch.as_tensor(mask.astype(np.uint8), device=device)
    total, dlogits, flags = _categorical_abi(logits, value, device, mask=m, scale=2.5, g0=-0.5)
    assert flags == 0
    lp, dl = lpf.categorical(logits.cpu().numpy(), np.broadcast_to(v, (K, N)))
    np.testing.assert_allclose(total.numpy(), 2.5 * (lp * mask).sum(1), rtol=1e-5)
    np.testing.assert_allclose(dlogits.numpy(), -1.25 * dl * mask[None, :, None], rtol=1e-5,
                               atol=1e-6)
    bad = v.copy()
    bad[np.flatnonzero(~mask)[0]] = C          # masked: ignored
    _, _, flags = _categorical_abi(logits, torch.as_tensor(bad, device=device).reshape(1, N)
                                   .expand(K, N), device, mask=m)
    assert flags == 0
    bad[np.flatnonzero(mask)[0]] = -1          # observed: flagged
    _, _, flags = _categorical_abi(logits, torch.as_tensor(bad, device=device).reshape(1, N)
                                   .expand(K, N), device, mask=m)
    assert flags & nat.FLAG_SUPPORT


@pytest.mark.parametrize("float_values", [False, True])
def test_categorical_model_against_oracle(device, float_values):
    """
    A masked K-particle Categorical model through EvidenceLowerBoundLoss (mi_categorical_forward,
    injected Normal noise) against the fp64 oracle at 1e-5; fractional values raise the reference's
    support error (integer_interval, core.py:186-188) instead of being truncated.
    """
    from torch.distributions import Categorical
    rng = np.random.default_rng(8)
    n, C, K = 3000, 6, 32
    y = rng.integers(0, C, size=n)
    mask = rng.random(n) > 0.2
    yt = torch.as_tensor(y.astype(np.float32) if float_values else y, device=device)
    obs = torch.masked.as_masked_tensor(yt, torch.as_tensor(mask, device=device))

    def model():
        theta = mi.sample("theta", Normal(0.0, 1.0), sample_shape=[C])
        mi.sample("y", Categorical(logits=theta), sample_shape=[n])

    loc = rng.normal(size=C).astype(np.float32) * 0.3
    scale = np.full(C, 0.4, np.float32)
    approx = mi.nn.ParameterizedFactorizedDistribution(theta=mi.nn.ParameterizedDistribution(
        Normal, loc=torch.as_tensor(loc), scale=torch.as_tensor(scale))).to(device)
    eps = rng.normal(size=(K, C)).astype(np.float32)
    loss = mi.nn.EvidenceLowerBoundLoss(num_particles=K)(
        mi.condition(model, y=obs), approx(), _noise={"theta": torch.as_tensor(eps, device=device)})
    loss.backward()
    ref = oracle.categorical_masked_elbo(y, mask, loc, scale, eps)
    assert abs(float(loss) - ref["loss"]) <= 1e-5 * abs(ref["loss"])
    params = approx["theta"].distribution_parameters
    np.testing.assert_allclose(params["loc"].grad.cpu().numpy(), ref["grad_loc"], rtol=1e-5,
                               atol=1e-5 * np.abs(ref["grad_loc"]).max())
    np.testing.assert_allclose(params["scale"].grad.cpu().numpy(), ref["grad_u_scale"], rtol=1e-5,
                               atol=1e-5 * np.abs(ref["grad_u_scale"]).max())
    frac = yt.clone()
    if float_values:
        frac[np.flatnonzero(mask)[0]] = 1.5
        bad = torch.masked.as_masked_tensor(frac, torch.as_tensor(mask, device=device))
        with pytest.raises(ValueError, match="is not in the support"):
            mi.nn.EvidenceLowerBoundLoss(num_particles=K)(mi.condition(model, y=bad), approx())


def test_elbo_loss_tensor_and_guide_exp(device):
    """
    The fused ELBO's loss is a plain-looking 0-d tensor whose backward() seeds autograd with a
    cached device 1.0 (no fill launch): same gradients as an explicit ones seed, repr as a tensor,
    and operations on it give ordinary tensors. A positive guide parameter's exp runs in
    mi_transform_params: values equal torch.exp's, and its autograd backward is exp(u).
    """
    from torch.distributions import Bernoulli, Beta
    torch.manual_seed(0)
    x = (torch.rand(3000) < 0.6).float().to(device)

    def model():
        theta = mi.sample("theta", Beta(2, 2))
        mi.sample("x", Bernoulli(theta), sample_shape=[3000])

    grads = []
    for explicit in (False, True):
        guide_mod = mi.nn.ParameterizedDistribution(Beta, concentration0=2.0,
                                                    concentration1=3.0).to(device)
        loss = mi.nn.EvidenceLowerBoundLoss(num_particles=64, seed=3)(
            mi.condition(model, x=x), {"theta": guide_mod()})
        assert repr(loss).startswith("tensor(") and type(loss + 1) is torch.Tensor
        if explicit:
            torch.autograd.backward(loss, torch.ones((), device=device))
        else:
            loss.backward()
        grads.append([p.grad.clone() for p in guide_mod.parameters()])
    for a, b in zip(*grads):
        assert torch.equal(a, b)

    module = mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(1000),
                                             scale=torch.rand(1000) + 0.5).to(device)
    scale = module().scale
    u = module.distribution_parameters["scale"]
    torch.testing.assert_close(scale, torch.exp(u.detach()), rtol=2e-7, atol=0)
    scale.sum().backward()
    torch.testing.assert_close(u.grad, torch.exp(u.detach()), rtol=2e-7, atol=0)


def test_beta_guide_transform_fused_into_draw(device, monkeypatch):
    """
    A Beta guide's exp transform runs inside its draw (mi_beta_rsample_exp) unless something reads
    the concentrations first: the ELBO, gradients and the written concentrations equal the
    separate-launch path bit for bit, and a reader without a draw (no_grad, .mean) sees the values.
    """
    from torch.distributions import Bernoulli, Beta
    x = (torch.rand(2000, generator=torch.Generator().manual_seed(2)) < 0.3).float().to(device)

    def model():
        theta = mi.sample("theta", Beta(2, 2))
        mi.sample("x", Bernoulli(theta), sample_shape=[2000])

    # torch's own argument validation reads the concentrations (and so runs the transform); the
    # captured steps run without it, as here
    monkeypatch.setattr(torch.distributions.Distribution, "_validate_args", False)
    results = []
    for defer in ("0", "1"):
        monkeypatch.setenv("MININF_AMD_DEFER_EXP", defer)
        module = mi.nn.ParameterizedDistribution(Beta, concentration0=2.5,
                                                 concentration1=1.5).to(device)
        loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=128, seed=5, validate=False)
        guide_dist = module()
        pending = guide.pending_exp(guide_dist._dirichlet.concentration) is not None
        assert pending == (defer == "1")
        loss = loss_fn(mi.condition(model, x=x), {"theta": guide_dist})
        loss.backward()
        assert guide.pending_exp(guide_dist._dirichlet.concentration) is None
        results.append((float(loss), [p.grad.clone() for p in module.parameters()],
                        guide_dist._dirichlet.concentration.detach().clone()))
    (l0, g0, c0), (l1, g1, c1) = results
    assert l0 == l1
    assert all(torch.equal(a, b) for a, b in zip(g0, g1))
    assert torch.equal(c0, c1)
    monkeypatch.setenv("MININF_AMD_DEFER_EXP", "1")
    module = mi.nn.ParameterizedDistribution(Beta, concentration0=2.5,
                                             concentration1=1.5).to(device)
    with torch.no_grad():
        d = module()
    torch.testing.assert_close(d.mean.cpu(), torch.tensor(1.5 / 4.0), rtol=1e-6, atol=0)


def test_bcast_reducible_floor_matches_per_eval(device, monkeypatch):
    """
    The measurement-only closed form of the C2 site kernel (MININF_AMD_BCAST_SUFFSTAT=1: sum_i x_i
    l_k as l_k sum_i x_i, the bench's reducible floor) computes the same ELBO and gradients as the
    per-eval kernel, at 1e-5.
    """
    from torch.distributions import Bernoulli, Beta
    n = 300_000
    x = (torch.rand(n, generator=torch.Generator().manual_seed(9)) < 0.7).float().to(device)

    def model():
        theta = mi.sample("theta", Beta(2, 2))
        mi.sample("x", Bernoulli(theta), sample_shape=[n])

    out = []
    for suff in ("0", "1"):
        monkeypatch.setenv("MININF_AMD_BCAST_SUFFSTAT", suff)
        module = mi.nn.ParameterizedDistribution(Beta, concentration0=2.0,
                                                 concentration1=2.0).to(device)
        loss = mi.nn.EvidenceLowerBoundLoss(num_particles=1024, seed=11)(
            mi.condition(model, x=x), {"theta": module()})
        loss.backward()
        out.append((float(loss), [p.grad.clone() for p in module.parameters()]))
    (l0, g0), (l1, g1) = out
    assert abs(l0 - l1) <= 1e-5 * abs(l0)
    for a, b in zip(g0, g1):
        assert (a - b).abs().max() <= 1e-5 * a.abs().max()


def test_normal_guide_transform_fused_into_draw(device, monkeypatch):
    """A Normal guide's scale = exp(u) is computed and written by its draw
    (mi_normal_rsample_exp): the ELBO, gradients and scale equal the separate-launch path bit for
    bit, for a vector factor (a small materialised draw) and a scalar one (a broadcast scale)."""
    gen = torch.Generator().manual_seed(4)
    X = torch.randn(3000, 8, generator=gen).to(device)
    y = (X @ torch.randn(8, generator=gen).to(device)) + 0.3

    def model():
        mu = mi.sample("mu", Normal(0.0, 1.0))
        theta = mi.sample("theta", Normal(mu, 1.0), sample_shape=[8])
        mi.sample("y", Normal(X @ theta, 1.0))

    monkeypatch.setattr(torch.distributions.Distribution, "_validate_args", False)
    results = []
    for defer in ("0", "1"):
        monkeypatch.setenv("MININF_AMD_DEFER_EXP", defer)
        guide_mod = mi.nn.ParameterizedFactorizedDistribution(
            mu=mi.nn.ParameterizedDistribution(Normal, loc=0.1, scale=0.7),
            theta=mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(8),
                                                  scale=torch.full((8,), 0.5))).to(device)
        approx = guide_mod()
        assert (guide.pending_exp(approx["theta"].scale) is not None) == (defer == "1")
        loss = mi.nn.EvidenceLowerBoundLoss(num_particles=64, seed=2, validate=False)(
            mi.condition(model, y=y), approx)
        loss.backward()
        results.append((float(loss), [p.grad.clone() for p in guide_mod.parameters()],
                        approx["theta"].scale.detach().clone(), approx["mu"].scale.detach().clone()))
    (l0, g0, s0, m0), (l1, g1, s1, m1) = results
    assert l0 == l1
    assert all(torch.equal(a, b) for a, b in zip(g0, g1))
    assert torch.equal(s0, s1) and torch.equal(m0, m1)


@pytest.mark.gpu
def test_normal_guide_transform_fused_into_site_program(device, monkeypatch):
    """A vector Normal guide whose draw is evaluated inside the site program (mi_draw) reads its
    unconstrained scale through mi_draw.scale_exp: the program computes exp(u), writes the scale
    and draws from it. ELBO, gradients and the written scale equal the separate transform launch
    bit for bit."""
    n = 1024
    gen = torch.Generator().manual_seed(5)
    y = torch.randn(n, generator=gen).to(device)
    b = (torch.rand(n, generator=gen) < 0.4).float().to(device)

    def model():
        mu = mi.sample("mu", Normal(0.0, 1.0))
        z = mi.sample("z", Normal(mu, 1.0), sample_shape=[n])
        mi.sample("y", Normal(z, 0.5))
        mi.sample("b", Bernoulli(logits=z))

    monkeypatch.setattr(torch.distributions.Distribution, "_validate_args", False)
    results = []
    for defer in ("0", "1"):
        monkeypatch.setenv("MININF_AMD_DEFER_EXP", defer)
        guide_mod = mi.nn.ParameterizedFactorizedDistribution(
            mu=mi.nn.ParameterizedDistribution(Normal, loc=0.1, scale=0.7),
            z=mi.nn.ParameterizedDistribution(Normal, loc=torch.linspace(-1, 1, n),
                                              scale=torch.linspace(0.2, 0.9, n))).to(device)
        approx = guide_mod()
        pending = guide.pending_exp(approx["z"].scale)
        assert (pending is not None) == (defer == "1")
        loss = mi.nn.EvidenceLowerBoundLoss(num_particles=64, seed=3, validate=False)(
            mi.condition(model, y=y, b=b), approx)
        if pending is not None:
            assert pending.filled   # written by the site program, no transform launch
        loss.backward()
        results.append((float(loss), [p.grad.clone() for p in guide_mod.parameters()],
                        approx["z"].scale.detach().clone()))
    (l0, g0, s0), (l1, g1, s1) = results
    assert l0 == l1
    assert all(torch.equal(a, c) for a, c in zip(g0, g1))
    assert torch.equal(s0, s1)
