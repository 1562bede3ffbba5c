"""Which torch linear-algebra ops a capturing stream accepts on this ROCm stack (GP example)."""
import sys
import torch

dev = torch.device("cuda", 0)
a = torch.randn(16, 50, 50, dtype=torch.float64, device=dev)
spd = a @ a.transpose(-1, -2) + 50 * torch.eye(50, dtype=torch.float64, device=dev)
which = sys.argv[1] if len(sys.argv) > 1 else "cholesky_ex"
ops = {
    "cholesky_ex": lambda: torch.linalg.cholesky_ex(spd),
    "cholesky_ex32": lambda: torch.linalg.cholesky_ex(spd.float()),
    "solve_triangular": lambda: torch.linalg.solve_triangular(spd.tril(), a, upper=False),
}
f = ops[which]
f()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
ok = True
with torch.cuda.stream(s):
    g.capture_begin()
    try:
        out = f()
    except Exception as e:
        ok = False
        print(which, "FAILED inside capture:", type(e).__name__, str(e).splitlines()[0])
    try:
        g.capture_end()
    except Exception as e:
        ok = False
        print(which, "capture_end FAILED:", str(e).splitlines()[0])
print(which, "ok" if ok else "not capturable", flush=True)
