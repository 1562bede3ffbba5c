"""
Microbenchmark of mi_linear_forward (the linear-predictor site kernel) at the C3 / C4 shapes.

    python tools/linear_bench.py [--valu]      (MININF_AMD_LIB=<variant build> compares launch
                                               shapes, tools/variant_build.py)
Prints one line per shape: mean kernel+finalize time and achieved TFLOP/s (4 P FLOP per eval).
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mininf_amd import _native as nat  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--valu", action="store_true")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--only", default=None, help="run one shape (C3, C3-bern, C4, P64)")
    ap.add_argument("--gather", choices=("none", "seq", "random"), default="none",
                    help="rows through mi_linear.row_index over a 10M-row X: sequential or random")
    ap.add_argument("--shape", action="append", default=[],
                    help="extra N,P,K shape (Normal); repeatable")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = nat.lib()
    shapes = [("C3", 1_000_000, 32, 256, nat.NORMAL),
              ("C3-bern", 1_000_000, 32, 256, nat.BERNOULLI_LOGITS),
              ("C4", 65536, 32, 32, nat.NORMAL),
              ("P64", 1_000_000, 64, 128, nat.NORMAL)]
    for text in args.shape:
        N, P, K = (int(v) for v in text.split(","))
        shapes.append((text, N, P, K, nat.NORMAL))
    if args.shape and args.only is None:
        args.only = "__shapes__"
    for name, N, P, K, fam in shapes:
        if args.only == "__shapes__" and name in ("C3", "C3-bern", "C4", "P64"):
            continue
        if args.only not in (None, "__shapes__") and name != args.only:
            continue
        if args.gather == "none":
            X = torch.randn(N, P, device=dev)
            rows = None
        else:
            X = torch.randn(10_000_000, P, device=dev)
            rows = (torch.arange(N, device=dev, dtype=torch.int32) if args.gather == "seq" else
                    torch.randperm(10_000_000, device=dev)[:N].to(torch.int32))
        theta = 0.3 * torch.randn(K, P, device=dev)
        ny = X.shape[0]
        y = torch.randn(ny, device=dev) if fam == nat.NORMAL else \
            (torch.rand(ny, device=dev) < 0.5).float()
        L = nat.Linear()
        L.K, L.N, L.P, L.family = K, N, P, fam
        L.options = nat.LINEAR_VALU if args.valu else 0
        L.x, (L.x_stride_i, L.x_stride_j) = X.data_ptr(), X.stride()
        L.theta, (L.theta_stride_k, L.theta_stride_j) = theta.data_ptr(), theta.stride()
        L.value, L.value_stride_i = y.data_ptr(), 1
        if rows is not None:
            L.row_index = rows.data_ptr()
        L.scale_constant, L.grad_scale, L.site_scale, L.compute_grads = 1.0, -1.0 / K, 1.0, 1
        size = ctypes.c_size_t()
        nat.check(lib.mi_linear_workspace_bytes(ctypes.byref(L), ctypes.byref(size)), "ws")
        work = torch.empty(size.value, dtype=torch.uint8, device=dev)
        total = torch.empty(K, device=dev)
        dslots = torch.empty((P, K), device=dev)
        flags = torch.empty(1, dtype=torch.int32, device=dev)
        stream = nat.stream_handle(dev)
        times = []
        for rep in range(args.reps + 3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            b.record()
            nat.check(lib.mi_linear_forward_deferred(
                ctypes.byref(L), work.data_ptr(), size.value, total.data_ptr(), dslots.data_ptr(),
                flags.data_ptr(), a.cuda_event, b.cuda_event, stream, None), "fwd")
            if rep >= 3:
                times.append((a, b))
        torch.cuda.synchronize()
        ms = sum(a.elapsed_time(b) for a, b in times) / len(times)
        tf = 4 * P * K * N / (ms * 1e-3) / 1e12
        print(f"{name:8s} gather={args.gather} N={N} P={P} K={K}: {ms * 1e3:8.1f} us  {tf:6.1f} TFLOP/s "
              f"({tf / 157.3:.3f} of 157.3)", flush=True)


if __name__ == "__main__":
    main()
