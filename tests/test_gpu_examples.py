"""
The reference's example models and its LogLikelihoodLoss on the MI355X path, against fixtures the
reference itself produced (tests/golden/make_golden.py): the models in tests/example_models.py are
the examples' code unchanged, so this is the north-star promise "existing model functions run
unchanged" checked at 1e-5 (ELBO / log likelihood values, gradients by max-norm).

Also: the Gamma / Poisson / InverseGamma site kernels against the reference's per-family tables,
the Gamma guide sampler's backward against torch._standard_gamma_grad, and broadcast_samples on the
particle machinery (one vmapped run) against the reference's per-sample loop.
"""
import numpy as np
import pytest
import torch
from torch.distributions import Gamma, Normal

import mininf_amd as mi
from mininf_amd import _native as nat, guide
from tests import example_models as ex
from tests.conftest import golden
from tests.test_gpu_kernels import launch

pytestmark = pytest.mark.gpu


def close(got, want, name, rtol=1e-5):
    got = np.asarray(got.detach().cpu() if isinstance(got, torch.Tensor) else got, np.float64)
    want = np.asarray(want, np.float64)
    err = np.abs(got - want).max() / max(np.abs(want).max(), 1e-30)
    assert err <= rtol, f"{name}: relative error {err:.3g}"


@pytest.mark.parametrize("mode", ["particle", "dense"])
def test_extra_family_tables(device, mode):
    f = golden("families_extra.npz")

    def rows(x):
        t = torch.as_tensor(x, dtype=torch.float32, device=device)
        return (t.reshape(-1, 1) if mode == "particle" else t.reshape(1, -1)).clone() \
            .requires_grad_()

    cases = [
        ("gamma", [f["gamma_a"], f["gamma_r"]], f["gamma_v"], f["gamma_lp"],
         [f["gamma_da"], f["gamma_dr"]]),
        ("poisson", [f["pois_rate"]], f["pois_v"], f["pois_lp"], [f["pois_drate"]]),
        ("inverse_gamma", [f["igamma_a"], f["igamma_r"]], f["igamma_v"], f["igamma_lp"],
         [f["igamma_da"], f["igamma_dr"]]),
    ]
    for family, params, value, want_lp, want_grads in cases:
        n = len(value)
        K, N = (n, 1) if mode == "particle" else (1, n)
        roles = [rows(p) for p in params]
        val = torch.as_tensor(value, dtype=torch.float32, device=device).reshape(K, N).contiguous()
        total, grads, slot_grad, flags, _ = launch(family, roles, val, device, K=K, N=N)
        assert (flags == 0).all(), family
        if mode == "particle":
            np.testing.assert_allclose(total.numpy(), want_lp, rtol=1e-5, atol=2e-6,
                                       err_msg=family)
            for j, want in enumerate(want_grads):
                np.testing.assert_allclose(-slot_grad[j].numpy(), want, rtol=2e-5, atol=2e-5,
                                           err_msg=f"{family} d{j}")
        else:
            np.testing.assert_allclose(total.numpy()[0], want_lp.sum(), rtol=1e-5, err_msg=family)
            for j, (grad, want) in enumerate(zip(grads, want_grads)):
                np.testing.assert_allclose(-grad.cpu().numpy()[0], want, rtol=2e-5, atol=2e-5,
                                           err_msg=f"{family} d{j}")


def test_extra_family_support_and_parameter_flags(device):
    """Out-of-support values (Gamma: v <= 0; Poisson: non-integer or negative) and invalid
    parameters reach the flag words."""
    ones = torch.ones(4, 1, device=device)
    v = torch.tensor([[0.5], [-1.0], [2.0], [3.0]], device=device)
    *_, flags, _ = launch("gamma", [ones, ones], v, device, K=4, N=1)
    assert int(flags.max()) & nat.FLAG_SUPPORT
    v = torch.tensor([[0.0], [1.5], [2.0], [3.0]], device=device)
    *_, flags, _ = launch("poisson", [ones], v, device, K=4, N=1)
    assert int(flags.max()) & nat.FLAG_SUPPORT
    bad = torch.tensor([[1.0], [-2.0], [1.0], [1.0]], device=device)
    *_, flags, _ = launch("gamma", [bad, ones], torch.ones(4, 1, device=device), device, K=4, N=1)
    assert int(flags.max()) & nat.FLAG_PARAM


def test_gamma_guide_sampler(device):
    """mi_gamma_rsample / backward: the implicit gradient of injected standard draws equals
    torch._standard_gamma_grad over all three regimes (golden), and generated draws have the
    Gamma(a, r) mean and variance."""
    f = golden("families_extra.npz")
    alpha = torch.as_tensor(f["sgg_alpha"], device=device).requires_grad_()
    rate = torch.ones_like(alpha).requires_grad_()
    g = torch.as_tensor(f["sgg_x"], device=device).reshape(1, -1)
    cfg = guide.DrawConfig(K=1, seed=0, step=0, stream_id=0, particle_offset=0, noise=g)
    x = guide.draw(Gamma(alpha, rate), cfg)
    x.sum().backward()
    np.testing.assert_allclose(alpha.grad.cpu().numpy(), f["sgg_grad"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(rate.grad.cpu().numpy(), -f["sgg_x"], rtol=1e-6)

    a = torch.tensor([0.3, 1.0, 2.5, 12.0], device=device)
    r = torch.tensor([2.0, 0.5, 1.0, 3.0], device=device)
    K = 1 << 16
    cfg = guide.DrawConfig(K=K, seed=5, step=0, stream_id=1, particle_offset=0)
    draws = guide.draw(Gamma(a, r), cfg).double()
    mean, var = (a / r).double(), (a / r ** 2).double()
    assert torch.all((draws.mean(0) - mean).abs() < 5 * (var / K).sqrt())
    assert torch.all((draws.var(0) / var - 1).abs() < 0.05)


# ------------------------------------------------------------------------------------------------
# LogLikelihoodLoss (nn.py:231-257)
# ------------------------------------------------------------------------------------------------
def test_log_likelihood_loss_against_reference(device):
    f = golden("loglik.npz")
    n = 2000
    theta = torch.tensor(float(f["coin_theta"]), device=device, requires_grad=True)

    def coin():
        t = mi.sample("theta", torch.distributions.Beta(2, 2))
        mi.sample("x", torch.distributions.Bernoulli(t), sample_shape=[n])
    value = mi.nn.LogLikelihoodLoss()(coin, {"theta": theta, "x": torch.as_tensor(
        f["coin_x"], device=device)})
    value.backward()
    close(value, f["coin_loss"], "coin loss")
    close(theta.grad, f["coin_dtheta"], "coin dtheta")

    th = torch.as_tensor(f["reg_theta"], device=device).requires_grad_()

    def regression():
        t = mi.sample("theta", Normal(0, 1), sample_shape=8)
        with mi.batch(10000):
            with mi.no_log_prob():
                Xs = mi.sample("X", Normal(0, 1), sample_shape=(10000, 8))
            mi.sample("y", Normal(Xs @ t, 1))
    value = mi.nn.LogLikelihoodLoss()(regression, {
        "theta": th, "X": torch.as_tensor(f["reg_X"], device=device),
        "y": torch.as_tensor(f["reg_y"], device=device)})
    value.backward()
    close(value, f["reg_loss"], "regression loss")
    close(th.grad, f["reg_dtheta"], "regression dtheta")

    m = 1000
    mu = torch.tensor(float(f["hier_mu"]), device=device, requires_grad=True)
    z = torch.as_tensor(f["hier_z"], device=device).requires_grad_()
    mask = torch.as_tensor(f["hier_mask"], device=device)

    def hier():
        mm = mi.sample("mu", Normal(0, 1))
        zz = mi.sample("z", Normal(mm, 1), sample_shape=[m])
        mi.sample("y", Normal(zz, 0.5))
        mi.sample("b", torch.distributions.Bernoulli(logits=zz))
    value = mi.nn.LogLikelihoodLoss()(hier, {
        "mu": mu, "z": z,
        "y": torch.masked.as_masked_tensor(torch.as_tensor(f["hier_y"], device=device), mask),
        "b": torch.masked.as_masked_tensor(torch.as_tensor(f["hier_b"], device=device), mask)})
    value.backward()
    close(value, f["hier_loss"], "hierarchical loss")
    close(mu.grad, f["hier_dmu"], "hierarchical dmu")
    close(z.grad, f["hier_dz"], "hierarchical dz")

    # the feature-uncertainty example at fixed parameters: Gamma and Poisson site kernels
    params = {k: torch.as_tensor(f[f"feat_{k}"], device=device).requires_grad_()
              for k in ("population_scale", "z", "intercept", "slope")}
    data = {k: torch.as_tensor(f[f"feat_{k}"], device=device) for k in ("x", "y", "noise_scale")}
    value = mi.nn.LogLikelihoodLoss()(ex.feature_model, {**params, **data})
    value.backward()
    close(value, f["feat_loss"], "feature model loss")
    for k, p in params.items():
        close(p.grad, f[f"feat_d{k}"], f"feature model d{k}")


# ------------------------------------------------------------------------------------------------
# The examples' ELBOs over K injected particles
# ------------------------------------------------------------------------------------------------
def _check_guide_grads(approximation, f, prefix=""):
    for factor in approximation:
        for pname, p in approximation[factor].distribution_parameters.items():
            close(p.grad, f[f"grad_{factor}_{pname}"], f"grad {factor}.{pname}")


def test_feature_uncertainty_example_elbo(device):
    f = golden("feature_uncertainty.npz")
    n, K = ex.FEATURE_N, f["eps_z"].shape[0]
    approximation = mi.nn.ParameterizedFactorizedDistribution(
        z=mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(n), scale=torch.ones(n)),
        intercept=mi.nn.ParameterizedDistribution(Normal, loc=0.0, scale=1.0),
        slope=mi.nn.ParameterizedDistribution(Normal, loc=0.0, scale=1.0),
        population_scale=mi.nn.ParameterizedDistribution(Gamma, concentration=2.0, rate=2.0),
    ).to(device)
    data = {"x": torch.as_tensor(f["x"], device=device),
            "y": torch.as_tensor(f["y"], device=device),
            "noise_scale": torch.tensor(float(f["noise_scale"]), device=device)}
    noise = {"z": f["eps_z"], "intercept": f["eps_intercept"], "slope": f["eps_slope"],
             "population_scale": f["g_population_scale"]}
    loss = mi.nn.EvidenceLowerBoundLoss(num_particles=K)(
        mi.condition(ex.feature_model, data), approximation(),
        _noise={k: torch.as_tensor(v, device=device) for k, v in noise.items()})
    loss.backward()
    close(loss, f["loss"], "loss")
    _check_guide_grads(approximation, f)


def test_missing_observations_example_elbo(device):
    f = golden("missing_observations.npz")
    n, K = ex.MISSING_N, f["eps_z"].shape[0]
    kappa = torch.tensor(float(f["kappa"]))
    approximation = mi.nn.ParameterizedFactorizedDistribution(
        z=mi.nn.ParameterizedDistribution(Normal, loc=torch.as_tensor(f["z_loc"]),
                                          scale=torch.ones(n) * kappa),
        sigma=mi.nn.ParameterizedDistribution(Gamma, concentration=2, rate=2),
        length_scale=mi.nn.ParameterizedDistribution(Gamma, concentration=2, rate=2),
    ).to(device)
    mask = torch.as_tensor(f["mask"], device=device)
    y = torch.masked.as_masked_tensor(torch.as_tensor(f["y"], device=device), mask)
    noise = {"z": f["eps_z"], "sigma": f["g_sigma"], "length_scale": f["g_length_scale"]}
    loss = mi.nn.EvidenceLowerBoundLoss(num_particles=K)(
        mi.condition(ex.missing_model, {"kappa": kappa.to(device)}, y=y), approximation(),
        _noise={k: torch.as_tensor(v, device=device) for k, v in noise.items()})
    loss.backward()
    # The GP prior's covariance is built by the model in float32 and is ill-conditioned (1e-3
    # jitter), so no float32 implementation reproduces another's rounding: the reference's own
    # fixture is 6.6e-6 (loss) to 1.1e-3 (gradients) away from the float64 evaluation of the same
    # ELBO (oracle.examples). The engine refactorises the MultivariateNormal in float64 (loss
    # 2.5e-6 from float64); the gradients still carry the model's float32 covariance arithmetic.
    # Each quantity must be within 1e-5 of the float64 truth, or within 4x the reference's own
    # distance from it (measured on MI355X: at most 2.4x, grad sigma.concentration).
    from oracle import examples
    truth = examples.missing_observations_elbo(f, torch.float64)

    def held(got, key):
        got = np.asarray(got.detach().cpu().double() if isinstance(got, torch.Tensor) else got)
        want, ref = np.asarray(truth[key], np.float64), np.asarray(f[key], np.float64)
        norm = max(np.abs(want).max(), 1e-30)
        ours, theirs = np.abs(got - want).max() / norm, np.abs(ref - want).max() / norm
        print(f"{key}: ours {ours:.3g}, reference {theirs:.3g} (relative to float64)")
        assert ours <= max(1e-5, 4 * theirs), (key, ours, theirs)
    held(loss, "loss")
    for factor in approximation:
        for pname, p in approximation[factor].distribution_parameters.items():
            held(p.grad, f"grad_{factor}_{pname}")


def test_missing_observations_example_trains(device):
    """The example's training loop (three steps, as under IN_CI) runs unchanged on the device."""
    n = ex.MISSING_N
    approximation = mi.nn.ParameterizedFactorizedDistribution(
        z=mi.nn.ParameterizedDistribution(Normal, loc=torch.randn(n), scale=torch.ones(n) * 0.1),
        sigma=mi.nn.ParameterizedDistribution(Gamma, concentration=2, rate=2),
        length_scale=mi.nn.ParameterizedDistribution(Gamma, concentration=2, rate=2),
    ).to(device)
    optimizer = torch.optim.Adam(approximation.parameters(), 0.05)
    loss = mi.nn.EvidenceLowerBoundLoss(num_particles=16)
    conditioned = mi.condition(ex.missing_model, kappa=torch.tensor(0.1, device=device),
                               y=torch.randn(n, device=device))
    for _ in range(3):
        optimizer.zero_grad()
        value = loss(conditioned, approximation())
        value.backward()
        optimizer.step()
        assert torch.isfinite(value)
    samples = approximation().sample([200])
    assert samples["z"].shape == (200, n)


# ------------------------------------------------------------------------------------------------
# broadcast_samples (core.py:548-584) on the particle machinery
# ------------------------------------------------------------------------------------------------
def test_predictive_broadcast_matches_reference(device):
    f = golden("predictive.npz")
    S, nlin = f["theta"].shape[0], f["lin"].shape[0]
    samples = mi.State({"theta": torch.as_tensor(f["theta"], device=device),
                        "sigma": torch.as_tensor(f["sigma"], device=device)})
    out = mi.broadcast_samples(mi.condition(ex.predictive_model, n=nlin,
                                            x=torch.as_tensor(f["lin"])), samples)
    assert sorted(out) == sorted(str(k) for k in f["keys"])
    for key in ("theta", "sigma", "n", "p", "x", "X"):
        got = out[key]
        assert got.device.type == device.type and got.shape == f[f"out_{key}"].shape, key
        # X = x ** arange(p): the device pow rounds within 1 ulp of the host's
        np.testing.assert_allclose(got.cpu().numpy(), f[f"out_{key}"], rtol=3e-7, atol=0,
                                   err_msg=key)
    np.testing.assert_allclose(out["prediction"].cpu().numpy(), f["out_prediction"], rtol=1e-5,
                               atol=1e-5)
    # y ~ Normal(prediction, sigma) is drawn anew: standardised residuals are N(0, 1)
    resid = ((out["y"] - out["prediction"]) / out["sigma"][:, None]).double()
    assert resid.shape == (S, nlin)
    assert abs(float(resid.mean())) < 5 / np.sqrt(S * nlin)
    assert abs(float(resid.std()) - 1) < 0.05


def test_predictive_broadcast_checks_parameters(device):
    """An invalid distribution parameter in a device broadcast_samples raises, as the reference's
    per-sample run does (torch distribution.py:68-80, 'Expected parameter scale'), instead of
    drawing from it."""
    from torch.distributions import Normal

    def model():
        sigma = mi.sample("sigma", Normal(0, 1))
        mi.sample("y", Normal(0.0, sigma), sample_shape=[3])

    good = mi.State({"sigma": torch.tensor([0.5, 1.0, 2.0], device=device)})
    assert mi.broadcast_samples(model, good)["y"].shape == (3, 3)
    bad = mi.State({"sigma": torch.tensor([0.5, -1.0, 2.0], device=device)})
    with pytest.raises(ValueError, match="Expected parameter scale"):
        mi.broadcast_samples(model, bad)


def test_predictive_draws_on_hip_samplers(device):
    """Missing sites of a device broadcast_samples are drawn by the HIP samplers (VERDICT r02
    item 8): reproducible under torch.manual_seed, one counter block per sample, and equal to the
    generator's own normals (mi_philox_normal) through z = loc + eps * scale; Gamma and Beta
    draws have the right moments."""
    from torch.distributions import Beta
    from mininf_amd import predictive
    S, n = 400, 5

    def model():
        loc = mi.sample("loc", Normal(0, 1))
        mi.sample("y", Normal(loc, 2.0), sample_shape=[n])
        mi.sample("g", Gamma(3.0, 2.0), sample_shape=[n])
        mi.sample("b", Beta(2.0, 5.0), sample_shape=[n])

    states = mi.State({"loc": torch.linspace(-1, 1, S, device=device)})
    torch.manual_seed(3)
    first = mi.broadcast_samples(model, states)
    torch.manual_seed(3)
    again = mi.broadcast_samples(model, states)
    for key in ("y", "g", "b"):
        assert first[key].shape == (S, n) and torch.equal(first[key], again[key]), key
    torch.manual_seed(3)
    seed = int(torch.randint(0, 2 ** 62, ()).item())
    eps = torch.empty(S * n, dtype=torch.float32, device=device)
    nat.check(nat.lib().mi_philox_normal(1, S * n, seed, 0, predictive.STREAM_BASE + 0, 0,
                                         eps.data_ptr(), nat.stream_handle(device)),
              "mi_philox_normal")
    want = states["loc"][:, None] + eps.reshape(S, n) * 2.0
    torch.testing.assert_close(first["y"], want, rtol=1e-6, atol=1e-6)
    g, b = first["g"].double(), first["b"].double()
    assert abs(float(g.mean()) - 1.5) < 0.08 and abs(float(g.var()) - 0.75) < 0.12
    assert abs(float(b.mean()) - 2 / 7) < 0.02
    assert float(g.min()) > 0 and 0 < float(b.min()) and float(b.max()) < 1
