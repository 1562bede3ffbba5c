"""
The HIP Marsaglia-Tsang samplers (csrc/guide.hip: k_gamma_rsample, k_beta_rsample) against their
plain-C restatement (oracle/philox.c: oracle_gamma_draws, oracle_beta_draws), draw by draw.

The reference draws its Beta / Gamma guide factors with torch's own sampler
(`approximation.rsample()`, /root/reference/mininf/nn.py:217 -> torch Beta.rsample -> _sample_dirichlet,
Gamma.rsample -> _standard_gamma). That generator cannot be reproduced bit for bit, so this build has
its own (Philox-4x32-7 blocks, Marsaglia-Tsang with the alpha < 1 boost), and these tests pin it:
- the same accept / reject path: a draw whose path differed would use a different normal and land
  far away, so agreement of every draw to a few ulp means every decision agreed; the inputs are
  chosen so that rejections, the alpha < 1 boost and several Philox blocks per draw all occur
  (checked on the oracle's block counts, so the comparison is not vacuous);
- values within REL_TOL relative: the device evaluates log / sqrt / cos / pow on the float
  hardware and OCML routines, the oracle in double precision rounded to float. Most draws agree to
  a few ulp; the algorithm amplifies the generator's ulp-level differences where it is
  ill-conditioned -- v = (1 + c x)^3 near y = 0 (tens of ulp), the alpha < 1 boost U^(1/alpha)
  at alpha = 0.05 (hundreds) -- so the bound is relative, far below the O(1) difference a single
  differing accept / reject decision makes (a different normal).
The full-size C2 step without injected draws ("Next round" 1b) then checks the bench's
own path end to end: the ELBO over the device's Beta draws against the oracle ELBO over the
restated draws.
"""
import numpy as np
import pytest
import torch
from torch.distributions import Bernoulli, Beta, Gamma

import mininf_amd as mi
from mininf_amd import _native as nat
from oracle import build as oracle_build, elbo as oracle

pytestmark = pytest.mark.gpu

# first GPU run: max 88 ulp (gamma, alpha = 1, y near 0), 1039 ulp (beta 0.05 / 0.05: the boost);
# relative 6e-5 at most
REL_TOL = 2e-4


def check_draws(got, want):
    """Every draw within REL_TOL relative; the bulk within a few ulp."""
    got = np.asarray(got, np.float32)
    want = np.asarray(want, np.float32)
    rel = np.abs(got.astype(np.float64) - want) / np.maximum(np.abs(want.astype(np.float64)),
                                                              1e-37)
    at = np.unravel_index(rel.argmax(), rel.shape)
    assert rel.max() <= REL_TOL, f"max relative {rel.max():.3g} at {at}: {got[at]} vs {want[at]}"
    d = ulps(got, want)
    assert np.median(d) <= 2 and (d <= 8).mean() >= 0.99, (np.median(d), (d <= 8).mean())


def ulps(a, b):
    """Distance in float32 units in the last place (sign-aware ordering of the bit patterns)."""
    def key(x):
        i = np.asarray(x, np.float32).view(np.int32).astype(np.int64)
        return np.where(i < 0, np.int64(-(2 ** 31)) - i, i)
    return np.abs(key(a) - key(b))


ALPHAS = np.array([0.3, 1.0, 2.5, 12.0, 0.05, 0.999, 1.001, 100.0], np.float32)


@pytest.mark.parametrize("seed,step,stream_id,offset", [(0, 0, 0, 0), (1234567, 9, 3, 1000),
                                                        (2 ** 40 + 7, 2 ** 33 + 5, 255, 77)])
def test_gamma_sampler_matches_restatement(device, seed, step, stream_id, offset):
    K = 4096
    conc = torch.as_tensor(ALPHAS, device=device)
    rate = torch.ones_like(conc)
    N = conc.shape[0]
    g = torch.empty(K, N, device=device)
    x = torch.empty(K, N, device=device)
    nat.check(nat.lib().mi_gamma_rsample(conc.data_ptr(), 1, rate.data_ptr(), 1, K, N, seed, step,
                                         None, stream_id, offset, None, g.data_ptr(), x.data_ptr(),
                                         None), "mi_gamma_rsample")
    want, blocks = oracle_build.gamma_draws(ALPHAS, K, seed, step, stream_id, offset)
    got = g.cpu().numpy()
    check_draws(got, want)
    # the comparison covers rejections (more than one block for alpha >= 1) and several blocks
    assert (blocks[:, ALPHAS >= 1] > 1).sum() > 10
    assert blocks.max() >= 3
    # x = g / rate (rate 1), floored at the smallest normal float
    np.testing.assert_array_equal(x.cpu().numpy(), np.maximum(got, np.float32(1.17549435e-38)))


def test_gamma_sampler_device_step_counter(device):
    """The step read from the device counter (graph replays) is the same stream as the argument."""
    K, seed = 512, 99
    conc = torch.as_tensor(ALPHAS, device=device)
    rate = torch.full_like(conc, 2.0)
    N = conc.shape[0]
    counter = torch.tensor([5], dtype=torch.int64, device=device)
    g = torch.empty(K, N, device=device)
    x = torch.empty(K, N, device=device)
    nat.check(nat.lib().mi_gamma_rsample(conc.data_ptr(), 1, rate.data_ptr(), 1, K, N, seed, 2,
                                         counter.data_ptr(), 4, 0, None, g.data_ptr(), x.data_ptr(),
                                         None), "mi_gamma_rsample")
    want, _ = oracle_build.gamma_draws(ALPHAS, K, seed, 7, 4, 0)
    got = g.cpu().numpy()
    check_draws(got, want)
    np.testing.assert_array_equal(x.cpu().numpy(), np.maximum(got / np.float32(2), np.float32(1.17549435e-38)))


C1 = np.array([0.3, 1.0, 2.5, 12.0, 0.3, 2.5, 0.05, 40.0], np.float32)
C0 = np.array([0.3, 2.5, 1.0, 12.0, 12.0, 0.3, 0.05, 0.5], np.float32)


@pytest.mark.parametrize("seed,step,stream_id,offset", [(0, 0, 0, 0), (31337, 4, 1, 2048)])
def test_beta_sampler_matches_restatement(device, seed, step, stream_id, offset):
    K = 4096
    c1 = torch.as_tensor(C1, device=device)
    c0 = torch.as_tensor(C0, device=device)
    N = C1.shape[0]
    x = torch.empty(K, N, device=device)
    nat.check(nat.lib().mi_beta_rsample(c1.data_ptr(), 1, c0.data_ptr(), 1, K, N, seed, step, None,
                                        stream_id, offset, None, x.data_ptr(), None),
              "mi_beta_rsample")
    want, g1, g0, b1, b0 = oracle_build.beta_draws(C1, C0, K, seed, step, stream_id, offset)
    got = x.cpu().numpy()
    # x = g1 / (g1 + g0): x near 0 (alpha = 0.05) carries the relative error of g1 itself
    check_draws(got, want)
    assert (b1 > 1).sum() > 10 and (b0 > 1).sum() > 10
    # (the 0.05 / 0.05 and 0.3 / 12 columns put many draws at exactly 0 or 1 in float32)
    assert ((got > 0) & (got < 1)).mean() > 0.9


def test_beta_sampler_exp_variant_matches_restatement(device):
    """mi_beta_rsample_exp (the C2 bench draw): expf of the unconstrained parameters, written
    interleaved, and the draws of those concentrations."""
    K, seed, step = 4096, 42, 3
    u1 = torch.log(torch.as_tensor(C1, device=device))
    u0 = torch.log(torch.as_tensor(C0, device=device))
    N = C1.shape[0]
    conc = torch.empty(N, 2, device=device)
    x = torch.empty(K, N, device=device)
    nat.check(nat.lib().mi_beta_rsample_exp(u1.data_ptr(), 1, u0.data_ptr(), 1, conc.data_ptr(), K,
                                            N, seed, step, None, 2, 0, None, x.data_ptr(), None),
              "mi_beta_rsample_exp")
    c = conc.cpu().numpy()
    np.testing.assert_allclose(c[:, 0], np.exp(u1.cpu().double().numpy()), rtol=3e-7)
    np.testing.assert_allclose(c[:, 1], np.exp(u0.cpu().double().numpy()), rtol=3e-7)
    want = oracle_build.beta_draws(c[:, 0], c[:, 1], K, seed, step, 2, 0)[0]
    check_draws(x.cpu().numpy(), want)


def test_gamma_guide_draw_through_the_elbo(device):
    """A Gamma guide factor drawn by the ELBO (stream 0, step 0 of a fresh loss) is the restated
    draw: the loss of a model with one Gamma site equals the oracle log-density sum."""
    K = 1024
    approx = mi.nn.ParameterizedDistribution(Gamma, concentration=0.7, rate=1.5).to(device)
    q = approx()

    def model():
        mi.sample("s", Gamma(2.0, 1.0))

    loss = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=11)(model, {"s": q})
    conc = float(q.concentration.detach().cpu())
    rate = float(q.rate.detach().cpu())
    g, _ = oracle_build.gamma_draws([conc], K, 11, 0, 0, 0)
    s = np.maximum(g[:, 0].astype(np.float64) / np.float32(rate), 1.17549435e-38)
    from scipy.special import gammaln
    lp = np.log(1.0) * 2 - gammaln(2.0) + (2 - 1) * np.log(s) - s
    ent = conc - np.log(rate) + gammaln(conc) + (1 - conc) * float(
        torch.special.digamma(torch.tensor(conc, dtype=torch.float64)))
    want = -(lp.mean() + ent)
    assert abs(float(loss) - want) <= 1e-5 * abs(want)


def test_full_size_c2_on_device_draws(device):
    """
    C2 exactly as the bench runs it (n = 1e6, K = 4096, Beta guide drawn by mi_beta_rsample_exp on
    the loss's own seed, the prior folded into the site launch, final gradients written by the ELBO
    forward), with nothing injected: loss and gradients against the oracle ELBO evaluated on the
    restated draws, at 1e-5 (VERDICT r03 "Next round" 1b). Two consecutive calls: the second uses
    step 1 of the generator.
    """
    n, K, seed = 1_000_000, 4096, 2024
    gen = torch.Generator().manual_seed(0)
    x = (torch.rand(n, generator=gen) < 0.7).float()

    def model():
        theta = mi.sample("theta", Beta(2, 2))
        mi.sample("x", Bernoulli(theta), sample_shape=[n])

    approx = mi.nn.ParameterizedDistribution(Beta, concentration1=2.5,
                                             concentration0=1.5).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=seed)
    cond = mi.condition(model, x=x.to(device))
    xs = x.numpy()
    for step in range(2):
        for p in approx.parameters():
            p.grad = None
        q = approx()
        value = loss_fn(cond, {"theta": q})
        value.backward()
        c1 = float(q.concentration1.detach().cpu())
        c0 = float(q.concentration0.detach().cpu())
        draws = oracle_build.beta_draws([c1], [c0], K, seed, step, 0, 0)[0][:, 0]
        ref = oracle.beta_bernoulli_elbo(xs, 2, 2, c1, c0, draws)
        assert abs(float(value) - ref["loss"]) <= 1e-5 * abs(ref["loss"]), step
        g = approx.distribution_parameters
        for name in ("concentration1", "concentration0"):
            want = ref[f"grad_u_{name}"]
            assert abs(float(g[name].grad) - want) <= 1e-5 * abs(want), (step, name)


@pytest.mark.parametrize("n", [1_000_017, 600_001, 2_100_000])
def test_c2_chunk_plans_against_the_oracle(device, n):
    """
    The C2 site kernel's chunk length follows the grid (r06: chunks evened out to one round of
    workgroup slots when the 4096-element grid fills between half a round and one round): n =
    1_000_017 gives 3936-element chunks with a 273-element last chunk (a whole 256-block, then an
    odd tail of 17 through the pair loop), 600_001 gives 2368-element chunks (groups of 32 past
    the last whole block), 2_100_000 keeps 4096 (two rounds). Loss and gradients against the oracle
    at 1e-5, on the device's own Beta draws.
    """
    K, seed = 4096, 77
    gen = torch.Generator().manual_seed(1)
    x = (torch.rand(n, generator=gen) < 0.3).float()

    def model():
        theta = mi.sample("theta", Beta(2, 2))
        mi.sample("x", Bernoulli(theta), sample_shape=[n])

    approx = mi.nn.ParameterizedDistribution(Beta, concentration1=1.7,
                                             concentration0=3.1).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=seed)
    q = approx()
    value = loss_fn(mi.condition(model, x=x.to(device)), {"theta": q})
    value.backward()
    c1 = float(q.concentration1.detach().cpu())
    c0 = float(q.concentration0.detach().cpu())
    draws = oracle_build.beta_draws([c1], [c0], K, seed, 0, 0, 0)[0][:, 0]
    ref = oracle.beta_bernoulli_elbo(x.numpy(), 2, 2, c1, c0, draws)
    assert abs(float(value) - ref["loss"]) <= 1e-5 * abs(ref["loss"])
    g = approx.distribution_parameters
    for name in ("concentration1", "concentration0"):
        want = ref[f"grad_u_{name}"]
        assert abs(float(g[name].grad) - want) <= 1e-5 * abs(want), name
