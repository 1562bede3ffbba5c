"""
Where C2's site kernel (k_site_bcast_smem) spends its time, per workgroup: a variant build of
sites.hip that stamps thread 0's wall clock (s_memrealtime, 100 MHz) at entry, after the
per-particle logits, after the FMA loops, after the chunk sum and at exit into a device array.
`run` replays the C2 bench step (24 steps per graph replay, as bench.py), then one more replay with
the array cleared, and prints the phase statistics of the last launch of that replay -- by dispatch
rank (block b is the b / 256-th workgroup of its CU in a one-round grid) and by XCD.

    python tools/c2_timeline.py build [name]   (on the CPU: tools/_variants/<name, c2tl>/)
    MININF_AMD_LIB=tools/_variants/c2tl/libmininf_amd.so python tools/c2_timeline.py run [rows.npy]
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch
from torch.distributions import Bernoulli, Beta

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import mininf_amd as mi  # noqa: E402
from mininf_amd import _native as nat  # noqa: E402
from mininf_amd.graph import StepGraph  # noqa: E402


def build_variant(name="c2tl"):
    """The timeline variant of the tree's sites.hip, through tools/variant_build.py."""
    import subprocess
    import tempfile
    src = open(os.path.join(ROOT, "mininf_amd", "csrc", "sites.hip")).read()

    def rep(old, new):
        nonlocal src
        assert src.count(old) == 1, old[:60]
        src = src.replace(old, new)
    rep("constexpr int kSmemMaxChunk", "__device__ unsigned long long g_tl[8192 * 8];\nconstexpr int kSmemMaxChunk")
    rep("""  const int64_t b = blockIdx.x;
  if (b >= padded * gy) {   // workgroups past the chunks: the side job (mi_side)
    const unsigned long long ts = span_begin(G.stamps);   // (the launch's span includes them)
    beta_side_block(G.side, b - padded * gy);
    span_end(G.stamps, ts);
    return;
  }""", """  const int64_t b = blockIdx.x;
  const unsigned long long T0 = __builtin_amdgcn_s_memrealtime();
  if (b >= padded * gy) {   // workgroups past the chunks: the side job (mi_side)
    const unsigned long long ts = span_begin(G.stamps);
    beta_side_block(G.side, b - padded * gy);
    span_end(G.stamps, ts);
    __syncthreads();
    if (threadIdx.x == 0) { g_tl[b * 8] = T0; g_tl[b * 8 + 4] = __builtin_amdgcn_s_memrealtime(); g_tl[b * 8 + 5] = 1; }
    return;
  }""")
    rep("""  double acc[kSmemP];
#pragma unroll
  for (int p = 0; p < kSmemP; ++p) acc[p] = 0.0;""", """  if (threadIdx.x == 0) { float z = 0.f;
#pragma unroll
    for (int p = 0; p < kSmemP; ++p) z += ld[p].x;
    __asm__ volatile("" :: "v"(z)); }
  const unsigned long long T1 = __builtin_amdgcn_s_memrealtime();
  double acc[kSmemP];
#pragma unroll
  for (int p = 0; p < kSmemP; ++p) acc[p] = 0.0;""")
    rep("""  // ---- chunk sum and support flags (vector loads, L2-resident by now)""",
        """  const unsigned long long T2 = __builtin_amdgcn_s_memrealtime();
  // ---- chunk sum and support flags (vector loads, L2-resident by now)""")
    rep("""  s_a = block_sum(s_a, scratch);
  if (SUFF) {""", """  s_a = block_sum(s_a, scratch);
  const unsigned long long T3 = __builtin_amdgcn_s_memrealtime();
  if (SUFF) {""")
    rep("""  if (G.prior.present != 0) publish_flags(G.prior.flags, fl_prior);
  span_end(G.stamps, t0);
}""", """  if (G.prior.present != 0) publish_flags(G.prior.flags, fl_prior);
  span_end(G.stamps, t0);
  __syncthreads();
  if (threadIdx.x == 0) {
    g_tl[b * 8] = T0; g_tl[b * 8 + 1] = T1; g_tl[b * 8 + 2] = T2; g_tl[b * 8 + 3] = T3;
    g_tl[b * 8 + 4] = __builtin_amdgcn_s_memrealtime(); g_tl[b * 8 + 5] = 0; g_tl[b * 8 + 6] = c;
    g_tl[b * 8 + 7] = kblock;
  }
}""")
    src += """
extern "C" int mi_debug_timeline(void* out, size_t bytes) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(mi::g_tl), bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int mi_debug_timeline_clear() {
  static unsigned long long zeros[8192 * 8];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(mi::g_tl), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice);
}
"""
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "sites.hip")
        open(path, "w").write(src)
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "variant_build.py"), name,
                        f"sites.hip={path}"], check=True)


def main():
    dev = torch.device("cuda:0")
    n, K = 1_000_000, 4096
    gy = K // 1024
    x = (torch.rand(n, generator=torch.Generator().manual_seed(0)) < 0.7).float().to(dev)

    def model():
        theta = mi.sample("theta", Beta(2, 2))
        mi.sample("x", Bernoulli(theta), sample_shape=[n])

    guide = mi.nn.ParameterizedDistribution(Beta, concentration0=2.0, concentration1=2.0).to(dev)
    cond = mi.condition(model, x=x)
    loss_fn = mi.nn.EvidenceLowerBoundLoss(num_particles=K, seed=3)
    opt = mi.optim.Adam(guide.parameters(), lr=0.02)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = loss_fn(cond, {"theta": guide()})
        loss.backward()
        opt.step()
        return loss

    lib = nat.lib()
    lib.mi_debug_timeline.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    graph = StepGraph(step, warmup=2, repeat=24)
    for _ in range(40):   # ~40 ms of device time: clocks up
        graph()
    torch.cuda.synchronize()
    assert lib.mi_debug_timeline_clear() == 0
    graph()
    torch.cuda.synchronize()
    raw = np.zeros(8192 * 8, dtype=np.uint64)
    assert lib.mi_debug_timeline(raw.ctypes.data, raw.nbytes) == 0
    rows = raw.reshape(-1, 8).astype(np.int64)
    rows = rows[rows[:, 0] > 0]
    main_rows = rows[rows[:, 5] == 0]
    side = rows[rows[:, 5] == 1]
    base = rows[:, 0].min()
    us = lambda v: (v - base) / 100.0   # noqa: E731
    t = [us(main_rows[:, i]) for i in range(5)]
    out = {"workgroups": int(main_rows.shape[0]), "side_workgroups": int(side.shape[0]),
           "kernel_span_us": float((rows[:, 4].max() - base) / 100.0)}

    def stats(v):
        return [round(float(np.min(v)), 2), round(float(np.percentile(v, 10)), 2),
                round(float(np.median(v)), 2), round(float(np.percentile(v, 90)), 2),
                round(float(np.max(v)), 2)]
    out["min/p10/median/p90/max (us)"] = {
        "entry": stats(t[0]), "logits (prologue)": stats(t[1] - t[0]),
        "fma loops": stats(t[2] - t[1]), "chunk sum + block sum": stats(t[3] - t[2]),
        "partials + flags (epilogue)": stats(t[4] - t[3]), "exit": stats(t[4]),
    }
    if side.shape[0]:
        out["side job (entry, exit)"] = {"entry": stats(us(side[:, 0])), "exit": stats(us(side[:, 4]))}
    c0 = main_rows[main_rows[:, 6] == 0]
    if c0.shape[0]:
        out["chunk-0 workgroups epilogue (us)"] = [round(float(v), 2) for v in (c0[:, 4] - c0[:, 3]) / 100.0]
    late = np.argsort(-t[4])[:8]
    out["last 8 to exit: (chunk, kblock, entry, loop, exit)"] = [
        (int(main_rows[i, 6]), int(main_rows[i, 7]), round(float(t[0][i]), 2),
         round(float(t[2][i] - t[1][i]), 2), round(float(t[4][i]), 2)) for i in late]
    xcd = main_rows[:, 6] % 8
    out["per XCD (c % 8): median prologue, loop, epilogue, exit; max exit"] = {
        int(q): [round(float(np.median((t[1] - t[0])[xcd == q])), 2),
                 round(float(np.median((t[2] - t[1])[xcd == q])), 2),
                 round(float(np.median((t[4] - t[3])[xcd == q])), 2),
                 round(float(np.median(t[4][xcd == q])), 2), round(float(np.max(t[4][xcd == q])), 2)]
        for q in range(8)}
    c, kb = main_rows[:, 6], main_rows[:, 7]
    b = (c // 8) * (8 * gy) + kb * 8 + c % 8
    out["by dispatch rank (b // 256): n, median prologue, loop, exit; min, max exit"] = {
        int(q): [int(((b // 256) == q).sum())] + [round(float(np.median(v[(b // 256) == q])), 2)
                                                   for v in (t[1] - t[0], t[2] - t[1], t[4])] +
        [round(float(t[4][(b // 256) == q].min()), 2), round(float(t[4][(b // 256) == q].max()), 2)]
        for q in range(int(b.max()) // 256 + 1)}
    if len(sys.argv) > 2:
        np.save(sys.argv[2], rows - np.array([base, base, base, base, base, 0, 0, 0]))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1:2] == ["build"]:
        build_variant(*sys.argv[2:3])
    else:
        main()
