"""Time mi_mvn_tril_forward against torch's MultivariateNormal.log_prob (float64, HIP events)."""
import torch
from torch.distributions import MultivariateNormal

from mininf_amd import mvn


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return 1e3 * a.elapsed_time(b) / reps


for K, n in [(64, 50), (1024, 50), (64, 200)]:
    g = torch.Generator().manual_seed(0)
    x = torch.randn(K, n, n, generator=g, dtype=torch.float64).cuda()
    cov = x @ x.transpose(-1, -2) / n + 0.5 * torch.eye(n, dtype=torch.float64, device="cuda")
    d = MultivariateNormal(torch.zeros(n, dtype=torch.float64, device="cuda"), covariance_matrix=cov)
    v = torch.randn(K, n, dtype=torch.float64, device="cuda")
    d._unbroadcasted_scale_tril  # factorised once, outside the timing
    print(f"K={K} n={n}: kernel {timed(lambda: mvn.log_prob(d, v)):.1f} us, "
          f"torch log_prob {timed(lambda: d.log_prob(v)):.1f} us", flush=True)
