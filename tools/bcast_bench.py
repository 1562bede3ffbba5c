"""
Microbenchmark of the Bernoulli BCAST site kernel (C2's k_site_bcast_smem / k_site_bcast) through
the engine's group launcher, over particle and element counts: mean kernel time (HIP events
recorded by mi_group_forward_deferred around the site kernel) and packed-FMA rate.

    python tools/bcast_bench.py           (MININF_AMD_LIB=<variant build> compares launch shapes,
                                           tools/variant_build.py)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mininf_amd import engine  # noqa: E402
from mininf_amd.particles import SiteRecord  # noqa: E402


class Timer:
    def __init__(self):
        self.pairs = []

    def pair(self, launcher):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        b.record()
        self.pairs.append((a, b))
        return a, b

    def stamps(self, launcher):
        return None


def main():
    dev = torch.device("cuda:0")
    for K, N in [(4096, 1_000_000), (2048, 1_000_000), (8192, 1_000_000), (4096, 500_000),
                 (4096, 2_000_000), (1024, 1_000_000)]:
        probs = (torch.rand(K, 1, device=dev) * 0.9 + 0.05).requires_grad_()
        x = (torch.rand(N, device=dev) < 0.7).float()
        views = [engine._View(probs, probs.stride(0), 0),
                 engine._View(x.reshape(1, -1).expand(K, N), 0, 1)]
        site = SiteRecord("x", "bernoulli_probs", [], torch.Size([N]), 1.0, None, "bernoulli_probs")
        launcher = engine._GroupLauncher(K, N, -1.0 / K, dev, per_site=True)
        assert launcher.try_add(site, views, None)
        timer = Timer()
        for rep in range(25):
            engine.KERNEL_TIMER = timer if rep >= 5 else None
            launcher.run(True)
        engine.KERNEL_TIMER = None
        torch.cuda.synchronize()
        ms = sum(a.elapsed_time(b) for a, b in timer.pairs) / len(timer.pairs)
        tf = 2.0 * K * N / (ms * 1e-3) / 1e12
        print(f"K={K:5d} N={N:8d}: {1e3 * ms:8.1f} us  {tf:6.1f} TFLOP/s ({tf / 157.3:.3f})",
              flush=True)


if __name__ == "__main__":
    main()
