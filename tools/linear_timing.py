"""
Where a k_linear_mfma block spends its time: phase timestamps (wall clock, 100 MHz) from a build
of the library with -DMI_LINEAR_TIMING=1, at the C4 shape.

    python tools/linear_timing.py build        (on the CPU: tools/_timing/libmininf_amd_lin.so)
    python tools/linear_timing.py run [N P K]  (on the GPU)
    python tools/linear_timing.py bench [c4]   (on the GPU: the bench step's own launch)

Stamps per wave: 0 entry, 1 before staging, 2 staged (loads issued, LDS written), 3 after the
staging barrier, 4 after the tiles, 5 after the tile barrier, 6 after the row-subset combine,
7 after the partial stores. Prints the mean of each phase and the spread of entry times.
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "_variants", "lintiming", "libmininf_amd.so")   # (sent to the GPU box)


def build():
    from mininf_amd import build as b
    b.write_embedded()
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [b.HIPCC, *b.FLAGS, "-DMI_LINEAR_TIMING=1", "-o", OUT, *b.SOURCES, *b.LIBS]
    subprocess.run(cmd, check=True)
    print(OUT)


def run(N=65536, P=32, K=32):
    import torch
    from mininf_amd import _native as nat
    nat.LIB_PATH = OUT
    lib = nat.lib()
    dev = torch.device("cuda:0")
    X = torch.randn(N, P, device=dev)
    theta = 0.3 * torch.randn(K, P, device=dev)
    y = torch.randn(N, device=dev)
    L = nat.Linear()
    L.K, L.N, L.P, L.family = K, N, P, nat.NORMAL
    L.x, (L.x_stride_i, L.x_stride_j) = X.data_ptr(), X.stride()
    L.theta, (L.theta_stride_k, L.theta_stride_j) = theta.data_ptr(), theta.stride()
    L.value, L.value_stride_i = y.data_ptr(), 1
    L.scale_constant, L.grad_scale, L.site_scale, L.compute_grads = 1.0, -1.0 / K, 1.0, 1
    size = ctypes.c_size_t()
    nat.check(lib.mi_linear_workspace_bytes(ctypes.byref(L), ctypes.byref(size)), "ws")
    work = torch.zeros(size.value, dtype=torch.uint8, device=dev)
    total = torch.empty(K, device=dev)
    dslots = torch.empty((P, K), device=dev)
    flags = torch.zeros(1, dtype=torch.int32, device=dev)
    stream = nat.stream_handle(dev)
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        b.record()
        nat.check(lib.mi_linear_forward_deferred(
            ctypes.byref(L), work.data_ptr(), size.value, total.data_ptr(), dslots.data_ptr(),
            flags.data_ptr(), a.cuda_event, b.cuda_event, stream, None), "fwd")
    torch.cuda.synchronize()
    try:
        kernel_ms = a.elapsed_time(b)
    except ValueError:   # (events recorded by the library on its stream)
        kernel_ms = float('nan')
    # the stamps sit at the end of the workspace: the last nonzero rows of 8 u64
    raw = work.view(torch.int64).cpu()
    rows = raw[raw.numel() % 8:].reshape(-1, 8)
    # stamp rows: positive, nondecreasing, under 10 ms end to end (the float partials in front of
    # the stamp area, read as int64, practically never look like that)
    ok = (rows[:, 0] > 0) & ((rows[:, 1:] - rows[:, :-1]) >= 0).all(dim=1) & \
        ((rows[:, 7] - rows[:, 0]) < 1_000_000)
    rows = rows[ok]
    rows = rows[(rows[:, 0] - rows[:, 0].median()).abs() < 1_000_000]
    t = rows.double() / 100.0   # 100 MHz -> microseconds
    base = t[:, 0].min()
    names = ["entry->stage", "stage issue", "stage barrier", "tiles", "tile barrier", "combine",
             "partials"]
    print(f"waves {rows.shape[0]}  kernel+finalize {kernel_ms * 1e3:.1f} us  "
          f"entry spread {float(t[:, 0].max() - base):.2f} us  "
          f"last exit {float(t[:, 7].max() - base):.2f} us")
    for i, name in enumerate(names):
        d = t[:, i + 1] - t[:, i]
        print(f"  {name:14s} mean {float(d.mean()):6.2f} us  max {float(d.max()):6.2f} us")
    life = t[:, 7] - t[:, 0]
    print(f"  wave lifetime  mean {float(life.mean()):6.2f} us  max {float(life.max()):6.2f} us")


def _phases(raw, label):
    import torch
    rows = raw[raw.numel() % 8:].reshape(-1, 8)
    ok = (rows[:, 0] > 0) & ((rows[:, 1:] - rows[:, :-1]) >= 0).all(dim=1) & \
        ((rows[:, 7] - rows[:, 0]) < 1_000_000)
    if not ok.any():
        return
    ok &= (rows[:, 0] - rows[ok][:, 0].median()).abs() < 1_000_000
    rows = rows[ok]
    t = rows.double() / 100.0
    base = t[:, 0].min()
    names = ["entry->stage", "stage issue", "stage barrier", "tiles", "tile barrier", "combine",
             "partials"]
    print(f"{label}: waves {rows.shape[0]}  entry spread {float(t[:, 0].max() - base):.2f} us  "
          f"last exit {float(t[:, 7].max() - base):.2f} us", flush=True)
    for i, name in enumerate(names):
        d = t[:, i + 1] - t[:, i]
        q = torch.quantile(d, torch.tensor([0.5, 0.9], dtype=torch.float64))
        print(f"  {name:14s} mean {float(d.mean()):6.2f}  p50 {float(q[0]):6.2f}  "
              f"p90 {float(q[1]):6.2f}  max {float(d.max()):6.2f} us")
    life = t[:, 7] - t[:, 0]
    print(f"  wave lifetime  mean {float(life.mean()):6.2f} us  max {float(life.max()):6.2f} us")
    start = t[:, 0] - base
    print(f"  entry          p50 {float(start.median()):6.2f}  max {float(start.max()):6.2f} us")
    # the last waves to exit: (block, wave) and their phase durations
    idx = torch.nonzero(ok).flatten()
    exit_t = t[:, 7] - base
    order = torch.argsort(exit_t, descending=True)[:6]
    for j in order.tolist():
        w = int(idx[j])
        ph = " ".join(f"{float(t[j, i + 1] - t[j, i]):5.2f}" for i in range(7))
        print(f"  late: block {w // 4:4d} wave {w % 4}  entry {float(start[j]):5.2f}  exit "
              f"{float(exit_t[j]):6.2f}  phases {ph}")
    blocks = idx // 4
    for lo, hi in ((0, 1), (1, 16), (16, 256), (256, 512)):
        sel = (blocks >= lo) & (blocks < hi)
        if sel.any():
            print(f"  blocks [{lo},{hi}): exit p50 {float(exit_t[sel].median()):6.2f} max "
                  f"{float(exit_t[sel].max()):6.2f} us")


def run_bench(config="c4"):
    """The bench's own step (rows, theta draw and prior in the launch): stamps of its linear
    launch, read from the launcher's workspace after each eager step."""
    import torch
    from mininf_amd import _native as nat
    nat.LIB_PATH = OUT
    nat.lib()
    import bench
    import mininf_amd
    device = torch.device("cuda", 0)
    w = bench.workload(config, device, 1, 0)
    optimizer = mininf_amd.optim.Adam(w["module"].parameters(), lr=w["lr"])
    loss_fn = mininf_amd.nn.EvidenceLowerBoundLoss(num_particles=w["k_local"], seed=1)
    for step in range(8):
        optimizer.zero_grad(set_to_none=True)
        loss = loss_fn(w["conditioned"](), w["guide"]())
        plan = loss.grad_fn.plan
        work = plan.linears[0].workspace
        torch.cuda.synchronize()
        raw = work.view(torch.int64).cpu()
        loss.backward()
        optimizer.step()
        if step >= 5:
            _phases(raw, f"{config} step {step}")
            fn = getattr(nat.lib(), "mi_debug_linear_prior", None)
            if fn is not None:   # the folded prior's sub-phases (timing builds)
                import numpy as np
                buf = np.zeros(64 * 6, dtype=np.uint64)
                fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
                fn(buf.ctypes.data, buf.nbytes)
                r = buf.reshape(64, 6).astype(np.int64)
                r = r[r[:, 1] > 0]
                for row in r:
                    d = np.diff(row[:5]) / 100.0
                    print(f"  prior wave (block {row[5]}): partials-start->prior {d[0]:5.2f}  "
                          f"kernargs {d[1]:5.2f}  evals {d[2]:5.2f}  stores+flags {d[3]:5.2f} us")
    torch.cuda.synchronize()


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    elif sys.argv[1] == "bench":
        run_bench(*(sys.argv[2:3]))
    else:
        run(*(int(v) for v in sys.argv[2:5]))
