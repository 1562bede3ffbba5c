"""
Where k_elbo_forward spends its time: per-block phase timestamps (wall clock, 100 MHz) from a
build of the library with -DMI_ELBO_TIMING=1, over eager steps of a bench config.

    python tools/elbo_timing.py build          (on the CPU: tools/_timing/libmininf_amd.so)
    python tools/elbo_timing.py run [c2|c4|c5] (on the GPU)

Stamps per block (thread 0; 16 slots): 0 entry, 1 the block's own work done (reduction or lead terms),
2 tail partials and the block sum, 3 the completion count (the last block known); the last block
only: 4 final loads and the loss sum, 6 the Beta tails (with their Adam updates), 7 the Normal
tail (with its Adam updates), 5 end (flag mirror, generator and optimizer step counts); reducing
blocks also 8 descriptor decoded (segment loads next) and 9 their segments summed.
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# (MI_ELBO_TIMING_LIB: another timing build, e.g. a copy kept for an A/B run)
OUT = os.environ.get("MI_ELBO_TIMING_LIB") or os.path.join(ROOT, "tools", "_timing", "libmininf_amd.so")


def build():
    from mininf_amd import build as b
    b.write_embedded()
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [b.HIPCC, *b.FLAGS, "-DMI_ELBO_TIMING=1", "-o", OUT, *b.SOURCES, *b.LIBS]
    subprocess.run(cmd, check=True)
    print(OUT)


def run(config="c2"):
    import torch
    from mininf_amd import _native as nat
    nat.LIB_PATH = OUT
    lib = nat.lib()
    import bench
    import mininf_amd
    device = torch.device("cuda", 0)
    w = bench.workload(config, device, 1, 0)
    optimizer = mininf_amd.optim.Adam(w["module"].parameters(), lr=w["lr"])
    loss_fn = mininf_amd.nn.EvidenceLowerBoundLoss(num_particles=w["k_local"], seed=1,
                                                 validate=False)   # graph mode: held launch
    import numpy as np
    rows_all = []
    for step in range(12):
        optimizer.zero_grad(set_to_none=True)
        loss = loss_fn(w["conditioned"](), w["guide"]())
        loss.backward()
        optimizer.step()   # (the ELBO forward is held until here: it runs the Adam step)
        torch.cuda.synchronize()
        buf = np.zeros(1 << 20, dtype=np.uint64)
        lib.mi_elbo_timing_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
        if step >= 4:
            rows = buf.reshape(-1, 16)
            rows = rows[rows[:, 0] > 0].astype(np.float64) / 100.0   # microseconds
            rows_all.append(rows)
    torch.cuda.synchronize()
    for rows in rows_all[-3:]:
        base = rows[:, 0].min()
        last = rows[rows[:, 5] > 0]
        print(f"blocks {rows.shape[0]}  entry spread {rows[:, 0].max() - base:.2f} us  "
              f"work {np.mean(rows[:, 1] - rows[:, 0]):.2f} (max {np.max(rows[:, 1] - rows[:, 0]):.2f})  "
              f"sum {np.mean(rows[:, 2] - rows[:, 1]):.2f}  count {np.mean(rows[:, 3] - rows[:, 2]):.2f} "
              f"(max {np.max(rows[:, 3] - rows[:, 2]):.2f})  last block: starts {last[0, 3] - base:.2f}, "
              f"loads+sum {last[0, 4] - last[0, 3]:.2f}, tails {last[0, 6] - last[0, 4]:.2f}, "
              f"normal tail {last[0, 7] - last[0, 6]:.2f}, mirror+step {last[0, 5] - last[0, 7]:.2f}, "
              f"end {last[0, 5] - base:.2f} us", flush=True)
        if last[0, 10] > 0:
            print(f"  last block: count -> acquire fence done {last[0, 10] - last[0, 3]:.2f}, "
                  f"fence -> loads summed {last[0, 4] - last[0, 10]:.2f} us", flush=True)
        if last[0, 11] > 0:
            print(f"  beta tail: sums' barrier -> lanes' start {last[0, 11] - last[0, 4]:.2f}, lanes 0 / 1's "
                  f"tail (grads, Adam) {last[0, 12] - last[0, 11]:.2f}, -> tails done "
                  f"{last[0, 6] - last[0, 12]:.2f} us", flush=True)
        red = rows[rows[:, 8] > 0]   # reducing blocks: descriptor decoded (8), segments summed (9)
        if red.shape[0]:
            print(f"  reducing blocks {red.shape[0]}: entry -> loads issued {np.mean(red[:, 8] - red[:, 0]):.2f} "
                  f"(max {np.max(red[:, 8] - red[:, 0]):.2f}), loads -> summed {np.mean(red[:, 9] - red[:, 8]):.2f} "
                  f"(max {np.max(red[:, 9] - red[:, 8]):.2f}), summed -> work done {np.mean(red[:, 1] - red[:, 9]):.2f} us",
                  flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(*(sys.argv[2:3]))
