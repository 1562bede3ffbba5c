"""
Where an ELBO-finishing launch spends its time (mi_group_elbo_forward for C2,
mi_linear_elbo_forward for C4): per-block wall-clock stamps (100 MHz) from a build of the library
with -DMI_FINISH_TIMING=1 (csrc/fin_timing.hpp).

    python tools/finish_timing.py build      (on the CPU: tools/_timing/libmininf_amd_fin.so)
    python tools/finish_timing.py run        (on the GPU)

Stamps per block: 0 kernel entry, 1 main work done (finish entry), 2 arrival ticket returned,
3 helper released from the wait, 4 helper's jobs done, 5 final block starts the tail, 6 tail
done, 7 optimizer step done. Prints, per config, the phases in microseconds relative to the
earliest entry.
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "_timing", "libmininf_amd_fin.so")


def build():
    from mininf_amd import build as b
    b.write_embedded()
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [b.HIPCC, *b.FLAGS, "-DMI_FINISH_TIMING=1", "-o", OUT, *b.SOURCES, *b.LIBS]
    subprocess.run(cmd, check=True)
    print(OUT)


def _c2(device):
    import torch
    from torch.distributions import Bernoulli, Beta
    import mininf_amd as mi
    n, K = 1_000_000, 4096
    x = (torch.rand(n, generator=torch.Generator().manual_seed(0)) < 0.7).float().to(device)

    def model():
        theta = mi.sample("theta", Beta(2.0, 2.0))
        mi.sample("x", Bernoulli(theta), sample_shape=[n])
    module = mi.nn.ParameterizedDistribution(Beta, concentration1=2.0,
                                             concentration0=2.0).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, validate=False)
    cond = mi.condition(model, x=x)
    return module, loss_fn, lambda: cond, lambda: {"theta": module()}


def _c4(device):
    import torch
    from torch.distributions import Normal
    import mininf_amd as mi
    from mininf_amd.data import DeviceDataLoader
    n, p, B, K = 1_000_000, 32, 65536, 32
    gen = torch.Generator().manual_seed(0)
    X = torch.randn(n, p, generator=gen).to(device)
    y = X @ torch.randn(p, generator=gen).to(device) + torch.randn(n, device=device)

    def model():
        theta = mi.sample("theta", Normal(0, 1), sample_shape=p)
        with mi.batch(n):
            with mi.no_log_prob():
                Xs = mi.sample("X", Normal(0, 1), sample_shape=(n, p))
            mi.sample("y", Normal(Xs @ theta, 1))
    loader = DeviceDataLoader(X, y, batch_size=B, shuffle=True, drop_last=True, seed=0)
    module = mi.nn.ParameterizedDistribution(Normal, loc=torch.zeros(p),
                                             scale=torch.ones(p)).to(device)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, validate=False)

    def cond():
        Xb, yb = loader.next()
        return mi.condition(model, X=Xb, y=yb)
    return module, loss_fn, cond, lambda: {"theta": module()}


def _phases(stamps):
    import numpy as np
    t = stamps.reshape(-1, 8).astype(np.int64)
    live = t[:, 0] > 0
    t = t[live]
    t0 = t[:, 0].min()
    us = lambda v: (v - t0) / 100.0   # 100 MHz -> microseconds

    def stat(name, v):
        v = v[~np.isnan(v)]
        if v.size:
            print(f"  {name:34s} n={v.size:5d}  min {v.min():7.2f}  p50 {np.median(v):7.2f}  "
                  f"p90 {np.percentile(v, 90):7.2f}  max {v.max():7.2f}")
    f = lambda c: np.where(t[:, c] > 0, t[:, c], np.nan).astype(float)
    stat("entry (us from first entry)", us(f(0)))
    stat("main work done", us(f(1)))
    stat("ticket latency", (f(2) - f(1)) / 100.0)
    stat("ticket returned", us(f(2)))
    stat("helper released", us(f(3)))
    stat("helper wait", (f(3) - f(2)) / 100.0)
    stat("helper jobs", (f(4) - f(3)) / 100.0)
    stat("final tail start", us(f(5)))
    stat("final tail", (f(6) - f(5)) / 100.0)
    stat("optimizer step", (f(7) - f(6)) / 100.0)
    print(f"  blocks {t.shape[0]}, span {us(t.max()):.2f} us")


def run():
    import numpy as np
    import torch
    from mininf_amd import _native as nat
    from mininf_amd.optim import Adam
    nat.LIB_PATH = OUT
    lib = nat.lib()
    device = torch.device("cuda:0")
    for name, setup, setter in (("c2", _c2, "mi_group_finish_timing"),
                                ("c4", _c4, "mi_linear_finish_timing")):
        fn = getattr(lib, setter)
        fn.argtypes, fn.restype = [ctypes.c_void_p], ctypes.c_int
        buf = torch.zeros(8 * 8192, dtype=torch.int64, device=device)
        nat.check(fn(buf.data_ptr()), setter)
        module, loss_fn, cond, approx = setup(device)
        optimizer = Adam(module.parameters(), lr=1e-3)
        for it in range(6):
            buf.zero_()
            optimizer.zero_grad(set_to_none=True)
            loss = loss_fn(cond(), approx())
            loss.backward()
            optimizer.step()
            torch.cuda.synchronize()
            if it >= 3:
                print(f"{name} step {it}: fusions {loss_fn.last_fusions}")
                _phases(buf.cpu().numpy())
        nat.check(fn(None), setter)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
