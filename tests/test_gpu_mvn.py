"""
MultivariateNormal site density on mi_mvn_tril_forward (csrc/mvn.hip, mininf_amd/mvn.py) against
torch's float64 MultivariateNormal.log_prob and its autograd (multivariate_normal.py:255-262), at
1e-10 relative (both float64): values and gradients with respect to value, loc and the covariance
(through torch's Cholesky), event sizes below, at and above one wave (lane loops), broadcast batch
shapes, the vmap rule of the particle trace, and the missing-observations example's GP site running
on the kernel (its ELBO parity against the reference's fixture is tests/test_gpu_examples.py).
"""
import numpy as np
import pytest
import torch
from torch.distributions import MultivariateNormal

from mininf_amd import mvn

pytestmark = pytest.mark.gpu


def spd(batch, n, device, gen):
    a = torch.randn(*batch, n, n, generator=gen, dtype=torch.float64).to(device)
    return a @ a.transpose(-1, -2) / n + 0.5 * torch.eye(n, dtype=torch.float64, device=device)


def rel(got, want):
    return float((got - want).abs().max() / max(float(want.abs().max()), 1e-300))


@pytest.mark.parametrize("n,vbatch,cbatch", [(1, (3,), (3,)), (50, (8,), (8,)),
                                             (64, (2, 5), (5,)), (130, (4,), ()),
                                             (7, (), (6,))])
def test_mvn_kernel_matches_torch(device, n, vbatch, cbatch):
    gen = torch.Generator().manual_seed(n)
    cov = spd(cbatch, n, device, gen)
    loc = torch.randn(n, generator=gen, dtype=torch.float64).to(device)
    value = torch.randn(*vbatch, n, generator=gen, dtype=torch.float64).to(device)
    out = []
    for kernel in (True, False):
        c = cov.clone().requires_grad_()
        m = loc.clone().requires_grad_()
        v = value.clone().requires_grad_()
        d = MultivariateNormal(m, covariance_matrix=c, validate_args=False)
        assert mvn.enabled(d)
        lp = mvn.log_prob(d, v) if kernel else d.log_prob(v)
        (lp * torch.linspace(0.5, 1.5, lp.numel(), dtype=torch.float64,
                             device=device).reshape(lp.shape)).sum().backward()
        out.append((lp.detach(), v.grad, m.grad, c.grad))
    for got, want, name in zip(out[0], out[1], ("log_prob", "dvalue", "dloc", "dcov")):
        assert got.shape == want.shape, name
        assert rel(got, want) <= 1e-10, (name, rel(got, want))


def test_mvn_kernel_under_vmap(device):
    """The particle trace's vmap rule: batched covariance and value, shared loc."""
    gen = torch.Generator().manual_seed(3)
    K, n = 16, 50
    cov = spd((K,), n, device, gen)
    value = torch.randn(K, n, generator=gen, dtype=torch.float64).to(device)
    loc = torch.zeros(n, dtype=torch.float64, device=device)

    def per_particle(c, v):
        return mvn.log_prob(MultivariateNormal(loc, covariance_matrix=c, validate_args=False), v)

    got = torch.func.vmap(per_particle)(cov, value)
    want = MultivariateNormal(loc, covariance_matrix=cov).log_prob(value)
    assert rel(got, want) <= 1e-10


@pytest.mark.parametrize("n,batch,dtype", [(1, (3,), torch.float64), (7, (2, 3), torch.float64),
                                            (50, (16,), torch.float64), (80, (4,), torch.float32),
                                            (81, (2,), torch.float64), (130, (), torch.float32)])
def test_cholesky_kernel_matches_torch(device, n, batch, dtype):
    """mi_cholesky (float64 arithmetic) against torch.linalg.cholesky, and its backward against
    torch's autograd of the factorisation (float64 at 1e-10)."""
    gen = torch.Generator().manual_seed(n)
    A = spd(batch, n, device, gen)
    L, info = mvn.cholesky_ex(A.to(dtype))
    want = torch.linalg.cholesky(A)
    assert L.dtype == dtype and L.shape == A.shape and info.shape == batch
    assert int(info.abs().sum()) == 0
    tol = 1e-10 if dtype == torch.float64 else 1e-6
    assert rel(L.double(), want) <= tol, rel(L.double(), want)
    if dtype == torch.float64:
        weight = torch.randn(A.shape, generator=gen, dtype=torch.float64).to(device)
        grads = []
        for ours in (True, False):
            a = A.clone().requires_grad_()
            out = mvn.cholesky_ex(a)[0] if ours else torch.linalg.cholesky(a)
            (out * weight).sum().backward()
            grads.append(a.grad)
        assert rel(grads[0], grads[1]) <= 1e-9, rel(grads[0], grads[1])


def test_cholesky_kernel_reports_non_positive_pivots(device):
    A = torch.eye(5, dtype=torch.float64, device=device).repeat(3, 1, 1)
    A[1, 3, 3] = -1.0
    _, info = mvn.cholesky_ex(A)
    _, want = torch.linalg.cholesky_ex(A)
    assert info.tolist() == want.tolist() == [0, 4, 0]


def test_cholesky_kernel_under_vmap(device):
    gen = torch.Generator().manual_seed(9)
    A = spd((12,), 20, device, gen)
    L, info = torch.func.vmap(mvn.cholesky_ex)(A)
    assert rel(L, torch.linalg.cholesky(A)) <= 1e-10 and info.shape == (12,)


def test_mvn_kernel_rejects_oversized_events(device):
    from mininf_amd import _native as nat
    buf = torch.zeros(8, dtype=torch.float64, device=device).data_ptr()
    assert nat.lib().mi_mvn_tril_forward(buf, buf, buf, 1, mvn.MAX_N + 1, buf, buf, buf,
                                         None) == -1


def test_missing_observations_gp_site_runs_on_kernel(device, monkeypatch):
    """The example's GP prior (MultivariateNormal over 50 points) goes through mi_mvn_tril_forward
    once per ELBO evaluation, for all particles at once."""
    import mininf_amd as mi
    from torch.distributions import Gamma, Normal
    from tests import example_models as ex
    calls = []
    launch = mvn._launch

    def counted(value, loc, scale_tril):
        calls.append(tuple(scale_tril.shape))
        return launch(value, loc, scale_tril)
    monkeypatch.setattr(mvn, "_launch", counted)
    n, K = ex.MISSING_N, 8
    approximation = mi.nn.ParameterizedFactorizedDistribution(
        z=mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(n), scale=torch.ones(n)),
        sigma=mi.nn.ParameterizedDistribution(Gamma, concentration=2, rate=2),
        length_scale=mi.nn.ParameterizedDistribution(Gamma, concentration=2, rate=2),
    ).to(device)
    y = torch.randn(n, device=device)
    loss = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=0)(
        mi.condition(ex.missing_model, {"kappa": torch.tensor(0.1, device=device)}, y=y),
        approximation())
    loss.backward()
    assert np.isfinite(float(loss))
    assert calls and all(shape[-2:] == (n, n) and shape[0] == K for shape in calls), calls



def test_missing_observations_step_under_graph_replay(device):
    """The GP example's training step (examples/missing-observations.md:28-45: a host
    `x[:, None] - x` and `torch.eye` inside the model, the Cholesky factorisation of the
    covariance, mi_mvn_tril_forward) captured by StepGraph: replays reproduce eager steps at 1e-6.
    The host intermediate is copied to the device once, keyed by its contents; the factorisation
    runs as cholesky_ex with its status in the step's validation words."""
    import mininf_amd as mi
    from mininf_amd.graph import StepGraph
    from torch.distributions import Gamma, Normal
    from tests import example_models as ex

    def setup():
        n = ex.MISSING_N
        approximation = mi.nn.ParameterizedFactorizedDistribution(
            z=mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(n), scale=torch.ones(n)),
            sigma=mi.nn.ParameterizedDistribution(Gamma, concentration=2, rate=2),
            length_scale=mi.nn.ParameterizedDistribution(Gamma, concentration=2, rate=2),
        ).to(device)
        optimizer = torch.optim.Adam(approximation.parameters(), lr=0.05, capturable=True)
        loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=16, seed=5)
        y = torch.linspace(-1, 1, n, device=device)
        conditioned = mi.condition(ex.missing_model, {"kappa": torch.tensor(0.1, device=device)},
                                   y=y)

        def step():
            optimizer.zero_grad(set_to_none=True)
            loss = loss_fn(conditioned, approximation())
            loss.backward()
            optimizer.step()
            return loss
        return step, approximation

    eager_step, eager_q = setup()
    graph_body, graph_q = setup()
    eager = [float(eager_step()) for _ in range(5)]
    captured = StepGraph(graph_body, warmup=2)
    replays = []
    for _ in range(3):
        replays.append(float(captured()))
    captured.check()
    np.testing.assert_allclose(replays, eager[2:], rtol=1e-6)
    for a, b in zip(eager_q.parameters(), graph_q.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
