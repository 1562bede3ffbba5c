"""
Host (CPU) paths against the reference's fixtures: LogLikelihoodLoss with host parameters keeps
the reference's torch-CPU evaluation (nn.py:231-257), and broadcast_samples with host samples keeps
the reference's per-sample loop (core.py:548-584). The device paths are in test_gpu_examples.py.
"""
import numpy as np
import torch
from torch.distributions import Bernoulli, Beta, Normal

import mininf_amd as mi
from tests import example_models as ex
from tests.conftest import golden


def test_host_log_likelihood_loss_matches_reference():
    f = golden("loglik.npz")
    theta = torch.tensor(float(f["coin_theta"]), requires_grad=True)

    def coin():
        t = mi.sample("theta", Beta(2, 2))
        mi.sample("x", Bernoulli(t), sample_shape=[2000])
    value = mi.nn.LogLikelihoodLoss()(coin, {"theta": theta, "x": torch.as_tensor(f["coin_x"])})
    value.backward()
    np.testing.assert_allclose(float(value), f["coin_loss"], rtol=1e-6)
    np.testing.assert_allclose(float(theta.grad), f["coin_dtheta"], rtol=1e-6)

    params = {k: torch.as_tensor(f[f"feat_{k}"]).requires_grad_()
              for k in ("population_scale", "z", "intercept", "slope")}
    data = {k: torch.as_tensor(f[f"feat_{k}"]) for k in ("x", "y", "noise_scale")}
    value = mi.nn.LogLikelihoodLoss()(ex.feature_model, {**params, **data})
    value.backward()
    np.testing.assert_allclose(float(value), f["feat_loss"], rtol=1e-6)
    for k, p in params.items():
        np.testing.assert_allclose(p.grad.numpy(), f[f"feat_d{k}"], rtol=1e-5, atol=1e-6)


def test_host_broadcast_samples_matches_reference():
    f = golden("predictive.npz")
    nlin = f["lin"].shape[0]
    samples = mi.State({"theta": torch.as_tensor(f["theta"]),
                        "sigma": torch.as_tensor(f["sigma"])})
    out = mi.broadcast_samples(mi.condition(ex.predictive_model, n=nlin,
                                            x=torch.as_tensor(f["lin"])), samples)
    assert sorted(out) == sorted(str(k) for k in f["keys"])
    for key in ("theta", "sigma", "n", "p", "x", "X", "prediction"):
        np.testing.assert_allclose(out[key].numpy(), f[f"out_{key}"], rtol=1e-6, err_msg=key)


def test_vmapped_broadcast_equals_loop_on_host():
    """broadcast_particles (one vmapped run) gives the loop's deterministic values."""
    from mininf_amd.particles import broadcast_particles
    f = golden("predictive.npz")
    nlin = f["lin"].shape[0]
    model = mi.condition(ex.predictive_model, n=nlin, x=torch.as_tensor(f["lin"]))
    states = {"theta": torch.as_tensor(f["theta"]), "sigma": torch.as_tensor(f["sigma"])}
    out = broadcast_particles(model, dict(states))
    for key in ("n", "p", "x", "X"):
        np.testing.assert_array_equal(out[key].numpy(), f[f"out_{key}"], err_msg=key)
    # batched X @ theta rounds in a different order than the per-sample products
    np.testing.assert_allclose(out["prediction"].numpy(), f["out_prediction"], rtol=1e-5,
                               atol=1e-5)
    lin = torch.as_tensor(f["lin"]).clone()
    lin[3] = float("nan")                                     # outside Normal's (real) support
    try:
        broadcast_particles(mi.condition(ex.predictive_model, n=nlin, x=lin), dict(states))
    except ValueError as error:   # deferred site checks: X's default-value check fires first
        assert "support" in str(error)
    else:
        raise AssertionError("expected a support error")
