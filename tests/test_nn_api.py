"""
Guide modules and losses (reference tests/test_nn.py, test_util.py, test_mininf.py,
test_distributions.py), written against mininf_amd. The ELBO tests that launch HIP kernels are
marked gpu; the rest run on the CPU.
"""
import numpy as np
import pytest
import torch
from torch import distributions

import mininf_amd as mi
from mininf_amd.distributions import InverseGamma
from mininf_amd.nn import EvidenceLowerBoundLoss, FactorizedDistribution, LogLikelihoodLoss, \
    ParameterizedDistribution, ParameterizedFactorizedDistribution
from mininf_amd.util import _normalize_shape, check_constraint, get_masked_data_with_dense_grad


@pytest.mark.parametrize("cls, params, const, learnable", [
    (distributions.Normal, {"loc": 0.0, "scale": 1.0}, set(), {"loc", "scale"}),
    (distributions.Normal, {"loc": torch.randn(3), "scale": torch.ones(2, 1)}, {"loc"}, {"scale"}),
    (distributions.LKJCholesky, {"dim": 3, "concentration": 9}, set(), {"concentration"}),
])
def test_parameterized_distribution(cls, params, const, learnable):
    module = ParameterizedDistribution(cls, _const=const, **params)
    dist = module()
    assert isinstance(dist, cls)
    draw = dist.sample()
    lp = dist.log_prob(draw)
    assert torch.isfinite(lp).all()
    lp.sum().backward()
    assert set(module.distribution_parameters) == learnable
    for name in learnable:
        assert module.distribution_parameters[name].grad is not None


def test_parameters_are_not_exposed():
    dist = ParameterizedDistribution(distributions.Normal, loc=0.0, scale=1.0)()
    assert not isinstance(dist.loc, torch.nn.Parameter)
    assert not isinstance(dist.scale, torch.nn.Parameter)


@pytest.mark.parametrize("clone", [False, True])
def test_clone_protects_inputs(clone):
    loc = torch.randn(3)
    snapshot = loc.clone()
    module = ParameterizedDistribution(distributions.Normal, loc=loc, scale=1, _clone=clone)
    optimizer = torch.optim.Adam(module.parameters(), 0.1)
    module().rsample().square().sum().backward()
    optimizer.step()
    if clone:
        np.testing.assert_allclose(loc, snapshot)
    else:
        assert ((loc - snapshot).abs() > 1e-6).all()


def test_factorized_distribution():
    x = distributions.Normal(0, 1)
    y = distributions.Gamma(2 * torch.ones(5), 2)
    joint = FactorizedDistribution(x=x, y=y)
    assert joint.entropy() == x.entropy() + y.entropy().sum()
    draws = joint.rsample([3])
    assert draws["x"].shape == (3,) and draws["y"].shape == (3, 5)
    draws = joint.sample([7])
    assert draws["x"].shape == (7,) and draws["y"].shape == (7, 5)


def test_parameterized_factorized_distribution():
    module = ParameterizedFactorizedDistribution(
        {"a": ParameterizedDistribution(distributions.Normal, loc=0.0, scale=1.0)},
        b=ParameterizedDistribution(distributions.Gamma, concentration=3.0, rate=2.0),
    )
    assert set(module) == {"a", "b"}
    assert isinstance(module()["a"], distributions.Normal)
    assert isinstance(module()["b"], distributions.Gamma)


def test_elbo_rejects_non_dict_samples():
    with pytest.raises(TypeError, match="dictionaries of tensors"):
        EvidenceLowerBoundLoss()(None, distributions.Normal(0, 1))


def test_elbo_requires_device_tensors():
    approximation = ParameterizedDistribution(distributions.Normal, loc=0.0, scale=1.0)
    with pytest.raises(RuntimeError, match="ROCm device"):
        EvidenceLowerBoundLoss()(lambda: mi.sample("x", distributions.Normal(0, 1)),
                                 {"x": approximation()})


def test_log_likelihood_loss_with_grad():
    estimate = torch.nn.Parameter(torch.ones(3))
    value = LogLikelihoodLoss()(lambda: mi.sample("x", distributions.Normal(0, 1), 3),
                                {"x": estimate})
    assert value.grad_fn is not None and value.ndim == 0 and np.isfinite(value.item())
    assert estimate.grad is None
    value.backward()
    assert estimate.grad is not None


def test_inverse_gamma_shapes():
    assert InverseGamma(torch.rand(3, 1), torch.rand(4)).sample([7]).shape == (7, 3, 4)


def test_linear_regression_prior_and_log_prob_shapes():
    def model(n, p):
        features = mi.sample("features", distributions.Normal(0, 1), (n, p))
        coefs = mi.sample("coefs", distributions.Normal(0, 1), p)
        sigma = mi.sample("sigma", distributions.Gamma(2, 2))
        mi.sample("outcomes", distributions.Normal(features @ coefs, sigma))

    assert model(5, 2) is None
    with mi.State() as state:
        model(50, 3)
    shapes = {"features": (50, 3), "coefs": (3,), "sigma": (), "outcomes": (50,)}
    assert {k: v.shape for k, v in state.items()} == shapes
    with mi.core.LogProbTracer() as lp, state:
        model(50, 3)
    assert {k: v[0].shape for k, v in lp.items()} == shapes


# ---- util (reference mininf/util.py) ----------------------------------------------------------

@pytest.mark.parametrize("dist", [
    distributions.MultivariateNormal(torch.randn(5), torch.randn(5).exp() * torch.eye(5)),
    distributions.LKJCholesky(3),
    distributions.Uniform(-torch.rand(5), torch.rand(5)),
])
def test_check_constraint_with_masks(dist):
    support = dist.support
    x = dist.sample([7, 13])
    mask = torch.rand(*x.shape[:x.ndim - support.event_dim]) > 0.5
    assert support.check(x).all()
    torch.testing.assert_close(check_constraint(support, x), support.check(x))
    x[~mask] = torch.nan
    torch.testing.assert_close(check_constraint(support, x), mask)
    expanded = mask.reshape(mask.shape + (1,) * support.event_dim)
    result = check_constraint(support, torch.masked.as_masked_tensor(
        *torch.broadcast_tensors(x, expanded)))
    torch.testing.assert_close(result.get_mask(), mask)
    assert result.all()


def test_masked_data_dense_grad():
    x = torch.randn(20)
    mask = torch.randn(20) < 0.5
    param = torch.nn.Parameter(torch.zeros_like(x))
    get_masked_data_with_dense_grad(torch.masked.as_masked_tensor(x * param, mask)).sum() \
        .backward()
    assert param.grad.is_sparse is False
    torch.testing.assert_close(param.grad, torch.where(mask, x, 0))
    param = torch.nn.Parameter(torch.zeros_like(x))
    data = get_masked_data_with_dense_grad(torch.masked.as_masked_tensor(x * param, mask))
    torch.masked.as_masked_tensor(data, mask).sum().backward()
    assert param.grad.is_sparse is False


@pytest.mark.parametrize("shape, expected", [
    (None, ()), (0, (0,)), (7, (7,)), ((0,), (0,)), ((3, 4), (3, 4)),
    (torch.as_tensor(5), (5,)), (torch.as_tensor([3, 7]), (3, 7)),
])
def test_normalize_shape(shape, expected):
    assert _normalize_shape(shape) == torch.Size(expected)


# ---- ELBO on the GPU (reference tests/test_nn.py:50-66) -----------------------------------------

@pytest.mark.gpu
def test_elbo_value_and_backprop(device):
    approximation = ParameterizedDistribution(distributions.Normal, loc=0.0,
                                              scale=torch.ones(3)).to(device)
    value = EvidenceLowerBoundLoss()(lambda: mi.sample("x", distributions.Normal(0, 1), 3),
                                     {"x": approximation()})
    assert value.grad_fn is not None and value.ndim == 0 and np.isfinite(value.item())
    assert all(p.grad is None for p in approximation.distribution_parameters.values())
    value.backward()
    assert all(p.grad is not None for p in approximation.distribution_parameters.values())


def test_optim_adam_argument_checks():
    import mininf_amd.optim as optim
    p = [torch.zeros(2, requires_grad=True)]
    with pytest.raises(ValueError, match="learning rate"):
        optim.Adam(p, lr=-1.0)
    with pytest.raises(ValueError, match="beta parameter at index 1"):
        optim.Adam(p, betas=(0.9, 1.0))
    with pytest.raises(NotImplementedError):
        optim.Adam(p, amsgrad=True)
