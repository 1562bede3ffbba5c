"""
Do the independent branches of a captured hipGraph run concurrently on this stack? Two streams
forked from the capture stream each run a chain of small elementwise kernels (latency-bound: a few
blocks each); the replay time of the forked graph is compared with the same chains captured on one
stream. Prints one JSON line.
"""
import json
import time

import torch


def chain(x, n):
    for _ in range(n):
        x = x * 1.0001 + 0.5
    return x


def main():
    dev = torch.device("cuda", 0)
    a = torch.randn(256 * 64, device=dev)
    b = torch.randn(256 * 64, device=dev)
    n = 200
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def forked():
        main = torch.cuda.current_stream()
        s1.wait_stream(main)
        s2.wait_stream(main)
        with torch.cuda.stream(s1):
            ya = chain(a, n)
        with torch.cuda.stream(s2):
            yb = chain(b, n)
        main.wait_stream(s1)
        main.wait_stream(s2)
        return ya, yb

    def serial():
        return chain(a, n), chain(b, n)

    out = {}
    for name, fn in (("forked", forked), ("serial", serial)):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            g.replay()
        torch.cuda.synchronize()
        out[name + "_us"] = (time.perf_counter() - t0) / 50 * 1e6
    out["ratio"] = out["forked_us"] / out["serial_us"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
