"""
Generate the golden fixtures in this directory by running the REFERENCE implementation
(tillahoffmann/mininf at /root/reference, imported read-only) on small instances of configs C1-C5.

Only this script touches the reference; it runs in the build container (the reference does not exist
on the GPU box) and only its outputs -- inputs and expected outputs as .npz data -- are committed.

Sample-injection protocol: the reference's EvidenceLowerBoundLoss draws ONE guide
sample internally (mininf/nn.py:217), so the guide factors are replaced by subclasses whose rsample
returns a supplied draw with the reference's own reparameterisation gradient:
  * Normal: loc + eps * scale with supplied eps;
  * Beta:   the supplied x, with torch's _Dirichlet_backward (implicit reparameterisation);
  * Gamma:  g / rate with the supplied standard draw g, with torch's _standard_gamma_grad.
A K-particle fixture is (1/K) * sum_k loss(model, guide with injected draw k), then backward().

Run:  PYTHONPATH=/root/reference python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np
import torch
from torch.distributions import Bernoulli, Beta, Gamma, MultivariateNormal, Normal, Poisson
from torch.distributions.dirichlet import _Dirichlet_backward

import mininf  # the reference (PYTHONPATH=/root/reference)

HERE = os.path.dirname(os.path.abspath(__file__))
assert mininf.__file__.startswith("/root/reference"), mininf.__file__


class InjectedNormal(Normal):
    def __init__(self, loc, scale, eps, validate_args=None):
        super().__init__(loc, scale, validate_args=validate_args)
        self._eps = eps

    def rsample(self, sample_shape=torch.Size()):
        return self.loc + self._eps * self.scale


class _InjectedDirichlet(torch.autograd.Function):
    @staticmethod
    def forward(ctx, concentration, x2):
        ctx.save_for_backward(x2, concentration)
        return x2.clone()

    @staticmethod
    def backward(ctx, grad):
        x2, concentration = ctx.saved_tensors
        return _Dirichlet_backward(x2, concentration, grad), None


class InjectedBeta(Beta):
    def __init__(self, concentration1, concentration0, x, validate_args=None):
        super().__init__(concentration1, concentration0, validate_args=validate_args)
        self._x = x

    def rsample(self, sample_shape=torch.Size()):
        x2 = torch.stack([self._x, 1.0 - self._x], -1)
        return _InjectedDirichlet.apply(self._dirichlet.concentration, x2).select(-1, 0)


class _InjectedStandardGamma(torch.autograd.Function):
    """torch._standard_gamma with a supplied result g (backward: _standard_gamma_grad)."""
    @staticmethod
    def forward(ctx, concentration, g):
        ctx.save_for_backward(concentration, g)
        return g.clone()

    @staticmethod
    def backward(ctx, grad):
        concentration, g = ctx.saved_tensors
        return grad * torch._standard_gamma_grad(concentration, g), None


class InjectedGamma(Gamma):
    """Gamma whose rsample is Gamma.rsample (gamma.py:80-88) with the standard draw g supplied."""
    def __init__(self, concentration, rate, g, validate_args=None):
        super().__init__(concentration, rate, validate_args=validate_args)
        self._g = g

    def rsample(self, sample_shape=torch.Size()):
        shape = self._extended_shape(sample_shape)
        g = _InjectedStandardGamma.apply(self.concentration.expand(shape), self._g.expand(shape))
        return g / self.rate.expand(shape)


def k_particle_loss(conditioned, make_guide, draws):
    """
    Mean over particles of the reference's single-draw ELBO loss.
    """
    loss = mininf.nn.EvidenceLowerBoundLoss()
    total = 0
    for draw in draws:
        total = total + loss(conditioned, make_guide(draw))
    return total / len(draws)


def grads_of(module):
    return {name: p.grad.detach().numpy().copy() for name, p in
            module.distribution_parameters.items()}


# ----------------------------------------------------------------------------------------------
# C1: the README biased coin, 3 Adam steps (README.md:40-69), injected draws.
# ----------------------------------------------------------------------------------------------
def c1():
    def model():
        n = 10
        theta = mininf.sample("theta", Beta(2, 2))
        x = mininf.sample("x", Bernoulli(theta), sample_shape=[n])
        return theta, x

    torch.manual_seed(0)
    _, x = model()
    approximation = mininf.nn.ParameterizedDistribution(Beta, concentration0=2, concentration1=2)
    conditioned = mininf.condition(model, x=x)
    optimizer = torch.optim.Adam(approximation.parameters(), lr=0.02)
    loss = mininf.nn.EvidenceLowerBoundLoss()
    draws = torch.distributions.Beta(torch.tensor(2.0), torch.tensor(2.0)).sample((3,))
    losses, params = [], []
    for step in range(3):
        optimizer.zero_grad()
        dist = approximation()
        guide = InjectedBeta(dist.concentration1, dist.concentration0, draws[step])
        value = loss(conditioned, {"theta": guide})
        value.backward()
        optimizer.step()
        losses.append(float(value))
        params.append([float(p) for p in approximation.distribution_parameters.values()])
    names = list(approximation.distribution_parameters)
    np.savez_compressed(os.path.join(HERE, "c1_readme.npz"), x=x.numpy(), draws=draws.numpy(),
                        losses=np.array(losses), params=np.array(params),
                        param_names=np.array(names))


# ----------------------------------------------------------------------------------------------
# C2 (small): Beta-Bernoulli, n = 4096, K = 64.
# ----------------------------------------------------------------------------------------------
def c2(n=4096, K=64):
    def model():
        theta = mininf.sample("theta", Beta(2, 2))
        mininf.sample("x", Bernoulli(theta), sample_shape=[n])

    torch.manual_seed(2)
    x = (torch.rand(n) < 0.7).float()
    c1_, c0_ = 2.5, 1.7
    approximation = mininf.nn.ParameterizedDistribution(Beta, concentration1=c1_,
                                                        concentration0=c0_)
    draws = torch.distributions.Beta(torch.tensor(c1_), torch.tensor(c0_)).sample((K,))
    dist = approximation()
    value = k_particle_loss(
        mininf.condition(model, x=x),
        lambda d: {"theta": InjectedBeta(dist.concentration1, dist.concentration0, d)}, draws)
    value.backward()
    g = grads_of(approximation)
    np.savez_compressed(os.path.join(HERE, "c2_beta_bernoulli.npz"), x=x.numpy(),
                        draws=draws.numpy(), c1=c1_, c0=c0_, loss=float(value),
                        grad_concentration1=g["concentration1"],
                        grad_concentration0=g["concentration0"])


# ----------------------------------------------------------------------------------------------
# C3 / C4 (small): linear regression (tests/test_mininf.py:13-18, examples/minibatch.md:24-33).
# ----------------------------------------------------------------------------------------------
def regression(name, n_total, n_obs, p, K, batched):
    def model():
        theta = mininf.sample("theta", Normal(0, 1), sample_shape=p)
        if batched:
            with mininf.batch(n_total):
                with mininf.no_log_prob():
                    X = mininf.sample("X", Normal(0, 1), sample_shape=(n_total, p))
                mininf.sample("y", Normal(X @ theta, 1))
        else:
            with mininf.no_log_prob():
                X = mininf.sample("X", Normal(0, 1), sample_shape=(n_total, p))
            mininf.sample("y", Normal(X @ theta, 1))

    torch.manual_seed(3)
    X = torch.randn(n_obs, p)
    true = torch.randn(p)
    y = X @ true + torch.randn(n_obs)
    loc0 = 1e-1 * torch.randn(p)
    scale0 = (1e-1 * torch.randn(p)).exp()
    approximation = mininf.nn.ParameterizedDistribution(Normal, loc=loc0.clone(),
                                                        scale=scale0.clone())
    eps = torch.randn(K, p)
    dist = approximation()
    value = k_particle_loss(mininf.condition(model, X=X, y=y),
                            lambda e: {"theta": InjectedNormal(dist.loc, dist.scale, e)}, eps)
    value.backward()
    g = grads_of(approximation)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), X=X.numpy(), y=y.numpy(),
                        loc0=loc0.numpy(), scale0=scale0.numpy(), eps=eps.numpy(),
                        n_total=n_total, loss=float(value), grad_loc=g["loc"],
                        grad_scale=g["scale"])


# ----------------------------------------------------------------------------------------------
# C5 (small): masked hierarchical model (examples/missing-observations.md:33-45, 53-54, restated).
# ----------------------------------------------------------------------------------------------
def c5(n=4096, K=16):
    def model():
        mu = mininf.sample("mu", Normal(0, 1))
        z = mininf.sample("z", Normal(mu, 1), sample_shape=[n])
        mininf.sample("y", Normal(z, 0.5))
        mininf.sample("b", Bernoulli(logits=z))

    torch.manual_seed(5)
    with mininf.State() as state:
        model()
    mask = torch.rand(n) > 0.2
    y = torch.masked.as_masked_tensor(state["y"], mask)
    b = torch.masked.as_masked_tensor(state["b"], mask)
    approximation = mininf.nn.ParameterizedFactorizedDistribution(
        mu=mininf.nn.ParameterizedDistribution(Normal, loc=0.1, scale=0.9),
        z=mininf.nn.ParameterizedDistribution(Normal, loc=0.1 * torch.randn(n),
                                              scale=torch.ones(n) * 0.8),
    )
    eps_mu = torch.randn(K)
    eps_z = torch.randn(K, n)
    dists = approximation()
    value = k_particle_loss(
        mininf.condition(model, y=y, b=b),
        lambda k: {"mu": InjectedNormal(dists["mu"].loc, dists["mu"].scale, eps_mu[k]),
                   "z": InjectedNormal(dists["z"].loc, dists["z"].scale, eps_z[k])},
        list(range(K)))
    value.backward()
    out = dict(y=state["y"].numpy(), b=state["b"].numpy(), mask=mask.numpy(),
               z_loc0=approximation["z"].distribution_parameters["loc"].detach().numpy(),
               eps_mu=eps_mu.numpy(), eps_z=eps_z.numpy(), loss=float(value))
    for factor in ("mu", "z"):
        for pname, p in approximation[factor].distribution_parameters.items():
            out[f"grad_{factor}_{pname}"] = p.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "c5_masked_hierarchical.npz"), **out)


# ----------------------------------------------------------------------------------------------
# Per-family elementwise tables with edge values, and the reference's error messages.
# ----------------------------------------------------------------------------------------------
def families():
    out = {}
    # Bernoulli via probs (clamped path) including p near 0 and 1.
    p = torch.tensor([1e-9, 1e-7, 0.01, 0.3, 0.5, 0.9, 1 - 1e-7, 1.0 - 2 ** -24, 0.999999],
                     requires_grad=True)
    v = torch.tensor([0.0, 1.0, 1.0, 0.0, 1.0, 1.0, 0.0, 1.0, 0.0])
    lp = Bernoulli(probs=p).log_prob(v)
    lp.sum().backward()
    out.update(bern_p=p.detach().numpy(), bern_v=v.numpy(), bern_lp=lp.detach().numpy(),
               bern_dp=p.grad.numpy())
    l = torch.tensor([-30.0, -5.0, -0.1, 0.0, 0.2, 4.0, 25.0], requires_grad=True)
    v = torch.tensor([1.0, 0.0, 1.0, 0.0, 1.0, 1.0, 0.0])
    lp = Bernoulli(logits=l).log_prob(v)
    lp.sum().backward()
    out.update(bernl_l=l.detach().numpy(), bernl_v=v.numpy(), bernl_lp=lp.detach().numpy(),
               bernl_dl=l.grad.numpy())
    loc = torch.tensor([0.0, -1.5, 2.0, 10.0], requires_grad=True)
    scale = torch.tensor([1.0, 0.1, 3.0, 0.5], requires_grad=True)
    v = torch.tensor([0.3, -1.4, -4.0, 9.0], requires_grad=True)
    lp = Normal(loc, scale).log_prob(v)
    lp.sum().backward()
    out.update(norm_loc=loc.detach().numpy(), norm_scale=scale.detach().numpy(),
               norm_v=v.detach().numpy(), norm_lp=lp.detach().numpy(),
               norm_dloc=loc.grad.numpy(), norm_dscale=scale.grad.numpy(), norm_dv=v.grad.numpy())
    a = torch.tensor([2.0, 0.5, 1.0, 7.0, 30.0], requires_grad=True)
    b = torch.tensor([2.0, 0.7, 3.0, 9.0, 2.0], requires_grad=True)
    v = torch.tensor([0.3, 0.01, 0.5, 0.45, 0.97], requires_grad=True)
    lp = Beta(a, b).log_prob(v)
    lp.sum().backward()
    out.update(beta_a=a.detach().numpy(), beta_b=b.detach().numpy(), beta_v=v.detach().numpy(),
               beta_lp=lp.detach().numpy(), beta_da=a.grad.numpy(), beta_db=b.grad.numpy(),
               beta_dv=v.grad.numpy())
    # Implicit reparameterisation gradient of Beta draws over all regimes of dirichlet_grad_one.
    xs, alphas, totals = [], [], []
    for x_ in (1e-4, 0.02, 0.3, 0.5, 0.7, 0.98, 0.9999):
        for a_ in (0.3, 1.0, 2.5, 8.0, 40.0):
            for b_ in (0.4, 1.0, 3.0, 12.0, 50.0):
                xs.append(x_)
                alphas.append(a_)
                totals.append(a_ + b_)
    xs, alphas, totals = (torch.tensor(t) for t in (xs, alphas, totals))
    out.update(dg_x=xs.numpy(), dg_alpha=alphas.numpy(), dg_total=totals.numpy(),
               dg_grad=torch._dirichlet_grad(xs, alphas, totals).numpy())
    # Categorical (normalised logits gather).
    logits = torch.randn(6, 5, generator=torch.Generator().manual_seed(7), requires_grad=True)
    v = torch.tensor([0, 4, 2, 2, 1, 3])
    lp = torch.distributions.Categorical(logits=logits).log_prob(v)
    lp.sum().backward()
    out.update(cat_logits=logits.detach().numpy(), cat_v=v.numpy(), cat_lp=lp.detach().numpy(),
               cat_dlogits=logits.grad.numpy())
    np.savez_compressed(os.path.join(HERE, "families.npz"), **out)


# ----------------------------------------------------------------------------------------------
# Round 2: the families the examples use, LogLikelihoodLoss, the example models, broadcast_samples.
# ----------------------------------------------------------------------------------------------
def families_extra():
    """Gamma / Poisson / InverseGamma (the reference's own class) log densities and gradients."""
    from mininf.distributions import InverseGamma
    out = {}
    a = torch.tensor([2.0, 0.5, 1.0, 7.0, 30.0, 2.0], requires_grad=True)
    r = torch.tensor([2.0, 0.7, 3.0, 0.1, 2.0, 10.0], requires_grad=True)
    v = torch.tensor([0.3, 0.01, 0.5, 45.0, 14.0, 0.2], requires_grad=True)
    lp = Gamma(a, r).log_prob(v)
    lp.sum().backward()
    out.update(gamma_a=a.detach().numpy(), gamma_r=r.detach().numpy(), gamma_v=v.detach().numpy(),
               gamma_lp=lp.detach().numpy(), gamma_da=a.grad.numpy(), gamma_dr=r.grad.numpy(),
               gamma_dv=v.grad.numpy())
    rate = torch.tensor([0.5, 3.0, 12.0, 0.01, 40.0, 1.0], requires_grad=True)
    v = torch.tensor([0.0, 2.0, 15.0, 1.0, 38.0, 0.0], requires_grad=True)
    lp = Poisson(rate).log_prob(v)
    lp.sum().backward()
    out.update(pois_rate=rate.detach().numpy(), pois_v=v.detach().numpy(),
               pois_lp=lp.detach().numpy(), pois_drate=rate.grad.numpy(), pois_dv=v.grad.numpy())
    a = torch.tensor([10.0, 2.0, 0.7, 5.0], requires_grad=True)
    r = torch.tensor([1.0, 2.0, 0.3, 8.0], requires_grad=True)
    v = torch.tensor([0.1, 1.5, 3.0, 2.2], requires_grad=True)
    lp = InverseGamma(a, r).log_prob(v)
    lp.sum().backward()
    out.update(igamma_a=a.detach().numpy(), igamma_r=r.detach().numpy(),
               igamma_v=v.detach().numpy(), igamma_lp=lp.detach().numpy(),
               igamma_da=a.grad.numpy(), igamma_dr=r.grad.numpy(), igamma_dv=v.grad.numpy())
    # Gamma entropy and its gradient (gamma.py:101-107)
    a = torch.tensor([0.4, 1.0, 2.0, 9.0], requires_grad=True)
    r = torch.tensor([0.5, 2.0, 2.0, 3.0], requires_grad=True)
    h = Gamma(a, r).entropy()
    h.sum().backward()
    out.update(gent_a=a.detach().numpy(), gent_r=r.detach().numpy(), gent_h=h.detach().numpy(),
               gent_da=a.grad.numpy(), gent_dr=r.grad.numpy())
    # implicit gradient of standard Gamma draws over the three regimes of standard_gamma_grad_one
    alphas, xs = [], []
    for a_ in (0.3, 1.0, 2.5, 7.9, 8.5, 40.0):
        for x_ in (0.05, 0.5, 0.79, 0.81, 2.0, 7.5, 9.0, 36.0, 41.0, 60.0):
            alphas.append(a_)
            xs.append(x_)
    alphas, xs = torch.tensor(alphas), torch.tensor(xs)
    out.update(sgg_alpha=alphas.numpy(), sgg_x=xs.numpy(),
               sgg_grad=torch._standard_gamma_grad(alphas, xs).numpy())
    np.savez_compressed(os.path.join(HERE, "families_extra.npz"), **out)


def loglik():
    """LogLikelihoodLoss (nn.py:231-257) at fixed parameters: values and parameter gradients."""
    out = {}
    torch.manual_seed(21)
    # (a) Beta-Bernoulli
    x = (torch.rand(2000) < 0.3).float()
    theta = torch.tensor(0.37, requires_grad=True)

    def coin():
        t = mininf.sample("theta", Beta(2, 2))
        mininf.sample("x", Bernoulli(t), sample_shape=[2000])
    value = mininf.nn.LogLikelihoodLoss()(coin, {"theta": theta, "x": x})
    value.backward()
    out.update(coin_x=x.numpy(), coin_theta=0.37, coin_loss=float(value),
               coin_dtheta=float(theta.grad))
    # (b) regression under batch(10000) with X not evaluated
    X, y = torch.randn(500, 8), torch.randn(500)
    th = torch.randn(8).requires_grad_()

    def regression():
        t = mininf.sample("theta", Normal(0, 1), sample_shape=8)
        with mininf.batch(10000):
            with mininf.no_log_prob():
                Xs = mininf.sample("X", Normal(0, 1), sample_shape=(10000, 8))
            mininf.sample("y", Normal(Xs @ t, 1))
    value = mininf.nn.LogLikelihoodLoss()(regression, {"theta": th, "X": X, "y": y})
    value.backward()
    out.update(reg_X=X.numpy(), reg_y=y.numpy(), reg_theta=th.detach().numpy(),
               reg_loss=float(value), reg_dtheta=th.grad.numpy())
    # (c) masked hierarchical
    n = 1000
    mu = torch.tensor(0.3, requires_grad=True)
    z = torch.randn(n).requires_grad_()
    yv, bv = torch.randn(n), (torch.rand(n) < 0.5).float()
    mask = torch.rand(n) > 0.2

    def hier():
        m = mininf.sample("mu", Normal(0, 1))
        zz = mininf.sample("z", Normal(m, 1), sample_shape=[n])
        mininf.sample("y", Normal(zz, 0.5))
        mininf.sample("b", Bernoulli(logits=zz))
    value = mininf.nn.LogLikelihoodLoss()(hier, {
        "mu": mu, "z": z, "y": torch.masked.as_masked_tensor(yv, mask),
        "b": torch.masked.as_masked_tensor(bv, mask)})
    value.backward()
    out.update(hier_z=z.detach().numpy(), hier_y=yv.numpy(), hier_b=bv.numpy(),
               hier_mask=mask.numpy(), hier_mu=0.3, hier_loss=float(value),
               hier_dmu=float(mu.grad), hier_dz=z.grad.numpy())
    # (d) the feature-uncertainty example model at fixed parameters (Gamma and Poisson sites)
    model, state = feature_model()
    params = {k: state[k].clone().requires_grad_() for k in
              ("population_scale", "z", "intercept", "slope")}
    value = mininf.nn.LogLikelihoodLoss()(model, {**params, **state.subset("x", "y",
                                                                           "noise_scale")})
    value.backward()
    out.update(feat_loss=float(value), **{f"feat_{k}": state[k].numpy() for k in state},
               **{f"feat_d{k}": p.grad.numpy() for k, p in params.items()})
    np.savez_compressed(os.path.join(HERE, "loglik.npz"), **out)


def feature_model():
    """examples/regression-with-feature-uncertainty.md:26-38 verbatim, data as at :46-48."""
    n = 30

    def model():
        population_scale = mininf.sample("population_scale", Gamma(2, 2))
        z = mininf.sample("z", Normal(0, population_scale), n)
        noise_scale = mininf.sample("noise_scale", Gamma(2, 2))
        x = mininf.sample("x", Normal(z, noise_scale))
        intercept = mininf.sample("intercept", Normal(0, 1))
        slope = mininf.sample("slope", Normal(0, 1))
        y = mininf.sample("y", Poisson((intercept + z * slope).exp()))  # noqa: F841

    torch.manual_seed(13)
    with mininf.State() as state:
        model()
    return model, state


def feature_uncertainty(K=8):
    """The example's ELBO (:75-90) over K injected particles: guide as at :76-81."""
    model, state = feature_model()
    n = 30
    approximation = mininf.nn.ParameterizedFactorizedDistribution(
        z=mininf.nn.ParameterizedDistribution(Normal, loc=torch.zeros(n), scale=torch.ones(n)),
        intercept=mininf.nn.ParameterizedDistribution(Normal, loc=0.0, scale=1.0),
        slope=mininf.nn.ParameterizedDistribution(Normal, loc=0.0, scale=1.0),
        population_scale=mininf.nn.ParameterizedDistribution(Gamma, concentration=2.0, rate=2.0),
    )
    conditioned = mininf.condition(model, state.subset("x", "y", "noise_scale"))
    gen = torch.Generator().manual_seed(31)
    eps_z, eps_i, eps_s = (torch.randn(K, n, generator=gen), torch.randn(K, generator=gen),
                           torch.randn(K, generator=gen))
    g_pop = torch._standard_gamma(torch.full((K,), 2.0), generator=gen)
    d = approximation()
    value = k_particle_loss(conditioned, lambda k: {
        "z": InjectedNormal(d["z"].loc, d["z"].scale, eps_z[k]),
        "intercept": InjectedNormal(d["intercept"].loc, d["intercept"].scale, eps_i[k]),
        "slope": InjectedNormal(d["slope"].loc, d["slope"].scale, eps_s[k]),
        "population_scale": InjectedGamma(d["population_scale"].concentration,
                                          d["population_scale"].rate, g_pop[k])},
        list(range(K)))
    value.backward()
    out = dict(x=state["x"].numpy(), y=state["y"].numpy(), noise_scale=float(state["noise_scale"]),
               eps_z=eps_z.numpy(), eps_intercept=eps_i.numpy(), eps_slope=eps_s.numpy(),
               g_population_scale=g_pop.numpy(), loss=float(value))
    for factor in approximation:
        for pname, p in approximation[factor].distribution_parameters.items():
            out[f"grad_{factor}_{pname}"] = p.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "feature_uncertainty.npz"), **out)


def missing_observations(K=8):
    """examples/missing-observations.md:28-45 verbatim; the masked data and guide of :53-54, :77-83."""
    import mininf.distributions
    n = 50
    x = torch.linspace(0, 1, n)

    def model() -> None:
        sigma = mininf.sample("sigma", Gamma(2, 2))
        length_scale = mininf.sample("length_scale", mininf.distributions.InverseGamma(10, 1))
        kappa = mininf.sample("kappa", Gamma(2, 10))
        residuals = (x[:, None] - x) / length_scale
        cov = sigma * sigma * (- residuals ** 2 / 2).exp() + 1e-3 * torch.eye(n)
        z = mininf.sample("z", MultivariateNormal(torch.zeros(n), cov))
        mininf.sample("y", Normal(z, kappa))

    torch.manual_seed(13)
    with mininf.State() as state:
        model()
    mask = torch.rand(n) > 0.2
    z_loc = torch.randn(n)
    approximation = mininf.nn.ParameterizedFactorizedDistribution(
        z=mininf.nn.ParameterizedDistribution(Normal, loc=z_loc.clone(),
                                              scale=torch.ones(n) * state["kappa"]),
        sigma=mininf.nn.ParameterizedDistribution(Gamma, concentration=2, rate=2),
        length_scale=mininf.nn.ParameterizedDistribution(Gamma, concentration=2, rate=2),
    )
    y = torch.masked.as_masked_tensor(state["y"], mask)
    conditioned = mininf.condition(model, state.subset("kappa"), y=y)
    gen = torch.Generator().manual_seed(41)
    eps_z = torch.randn(K, n, generator=gen)
    g_sigma = torch._standard_gamma(torch.full((K,), 2.0), generator=gen)
    g_length = torch._standard_gamma(torch.full((K,), 2.0), generator=gen)
    d = approximation()
    value = k_particle_loss(conditioned, lambda k: {
        "z": InjectedNormal(d["z"].loc, d["z"].scale, eps_z[k]),
        "sigma": InjectedGamma(d["sigma"].concentration, d["sigma"].rate, g_sigma[k]),
        "length_scale": InjectedGamma(d["length_scale"].concentration, d["length_scale"].rate,
                                      g_length[k])},
        list(range(K)))
    value.backward()
    out = dict(y=state["y"].numpy(), mask=mask.numpy(), kappa=float(state["kappa"]),
               z_loc=z_loc.numpy(), eps_z=eps_z.numpy(), g_sigma=g_sigma.numpy(),
               g_length_scale=g_length.numpy(), loss=float(value))
    for factor in approximation:
        for pname, p in approximation[factor].distribution_parameters.items():
            out[f"grad_{factor}_{pname}"] = p.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "missing_observations.npz"), **out)


def predictive(S=40):
    """examples/predictive.md:22-38 verbatim; broadcast_samples (:86) over fixed samples."""
    from torch.distributions.constraints import nonnegative_integer

    def model():
        n = mininf.value("n", 30, support=nonnegative_integer)
        p = mininf.value("p", 3, support=nonnegative_integer)
        x = mininf.sample("x", torch.distributions.Normal(0, 1), n)
        X = mininf.value("X", x[:, None] ** torch.arange(p))
        theta = mininf.sample("theta", torch.distributions.Normal(0, 1), p)
        prediction = mininf.value("prediction", X @ theta)
        sigma = mininf.sample("sigma", torch.distributions.Gamma(2, 2))
        y = mininf.sample("y", torch.distributions.Normal(prediction, sigma))  # noqa: F841

    torch.manual_seed(0)
    with mininf.State() as state:
        model()
    gen = torch.Generator().manual_seed(51)
    samples = {"theta": torch.randn(S, 3, generator=gen),
               "sigma": torch._standard_gamma(torch.full((S,), 10.0), generator=gen) / 10.0}
    nlin = 101
    lin = torch.linspace(state["x"].min() - 0.1, state["x"].max() + 0.1, nlin)
    torch.manual_seed(52)
    out_state = mininf.broadcast_samples(mininf.condition(model, n=nlin, x=lin),
                                         mininf.State(dict(samples)))
    out = {f"out_{k}": v.numpy() for k, v in out_state.items()}
    out.update(theta=samples["theta"].numpy(), sigma=samples["sigma"].numpy(), lin=lin.numpy(),
               keys=np.array(sorted(out_state)))
    np.savez_compressed(os.path.join(HERE, "predictive.npz"), **out)


def messages():
    """
    Error messages the reference raises on the hot path's negative cases.
    """
    found = {}

    def capture(key, fn):
        try:
            fn()
        except Exception as ex:  # noqa: BLE001
            found[key] = f"{type(ex).__name__}: {ex}"

    def twice():
        mininf.sample("x", Normal(0, 1))
        mininf.sample("x", Normal(0, 1))
    def twice_case():
        with mininf.State():
            twice()
            with mininf.core.LogProbTracer():
                twice()
    capture("twice", twice_case)
    capture("missing", lambda: mininf.nn.LogLikelihoodLoss()(
        lambda: mininf.sample("q", Normal(0, 1)), {}))
    capture("support", lambda: mininf.nn.LogLikelihoodLoss()(
        lambda: mininf.sample("x", Bernoulli(0.5), [3]), {"x": torch.tensor([0.0, 2.0, 1.0])}))
    capture("shape", lambda: mininf.nn.LogLikelihoodLoss()(
        lambda: mininf.sample("x", Normal(0, 1), [3]), {"x": torch.zeros(4)}))
    capture("type", lambda: mininf.nn.EvidenceLowerBoundLoss()(None, Normal(0, 1)))
    with open(os.path.join(HERE, "messages.txt"), "w") as fh:
        for key in sorted(found):
            fh.write(f"{key}\t{found[key]}\n")


FIXTURES = {
    "c1": c1, "c2": c2,
    "c3": lambda: regression("c3_regression", n_total=4096, n_obs=4096, p=32, K=16,
                             batched=False),
    "c4": lambda: regression("c4_minibatch", n_total=1_000_000, n_obs=1024, p=32, K=16,
                             batched=True),
    "c5": c5, "families": families, "messages": messages,
    "families_extra": families_extra, "loglik": loglik, "feature_uncertainty": feature_uncertainty,
    "missing_observations": missing_observations, "predictive": predictive,
}

if __name__ == "__main__":
    # all fixtures, or only those named on the command line
    for name in sys.argv[1:] or list(FIXTURES):
        FIXTURES[name]()
    print("golden fixtures written to", HERE, file=sys.stderr)
