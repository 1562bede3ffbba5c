"""
Generate the golden fixtures in this directory by running the REFERENCE implementation
(tillahoffmann/mininf at /root/reference, imported read-only) on small instances of configs C1-C5.

Only this script touches the reference; it runs in the build container (the reference does not exist
on the GPU box) and only its outputs -- inputs and expected outputs as .npz data -- are committed.

Sample-injection protocol: the reference's EvidenceLowerBoundLoss draws ONE guide
sample internally (mininf/nn.py:217), so the guide factors are replaced by subclasses whose rsample
returns a supplied draw with the reference's own reparameterisation gradient:
  * Normal: loc + eps * scale with supplied eps;
  * Beta:   the supplied x, with torch's _Dirichlet_backward (implicit reparameterisation).
A K-particle fixture is (1/K) * sum_k loss(model, guide with injected draw k), then backward().

Run:  PYTHONPATH=/root/reference python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np
import torch
from torch.distributions import Bernoulli, Beta, Normal
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


if __name__ == "__main__":
    c1()
    c2()
    regression("c3_regression", n_total=4096, n_obs=4096, p=32, K=16, batched=False)
    regression("c4_minibatch", n_total=1_000_000, n_obs=1024, p=32, K=16, batched=True)
    c5()
    families()
    messages()
    print("golden fixtures written to", HERE, file=sys.stderr)
