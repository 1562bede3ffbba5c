import torch, time
torch.cuda.init()
s1 = torch.cuda.current_stream()
s2 = torch.cuda.Stream()
a = torch.randn(1536, 1536, device="cuda")
def work():
    s2.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s2):
        torch.cuda._sleep(200000)    # ~100 us spin, one wave
    b = a @ a                         # ~ tens of us
    c = b @ a
    torch.cuda.current_stream().wait_stream(s2)
    return c
def serial():
    torch.cuda._sleep(200000)
    b = a @ a
    return b @ a
for name, fn in [("parallel", work), ("serial", serial)]:
    for _ in range(3): fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        fn()
    for _ in range(5): g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(50): g.replay()
    torch.cuda.synchronize()
    print(name, "graph us/replay", 1e6 * (time.perf_counter() - t) / 50)
# components
for name, fn in [("sleep", lambda: torch.cuda._sleep(200000)), ("mm", lambda: (a @ a) @ a)]:
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(50): fn()
    torch.cuda.synchronize(); print(name, "eager us", 1e6 * (time.perf_counter() - t) / 50)
