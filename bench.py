"""
Benchmark of the ELBO hot path: site-log_prob evals/sec and ELBO step wall time on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c1|c3|c4|c5]

One *step* = ``optimizer.zero_grad()`` + ELBO forward + backward (+ one RCCL all-reduce of the guide
gradients when N > 1) + ``Adam.step()``, as in the reference's training loop (README.md:66-69).
The default workload is C2 (BASELINE.json configs[1]): the README biased-coin model with n = 1e6
observations and 4096 Monte-Carlo particles per GPU (particles are sharded across GPUs: weak
scaling). One site-log_prob eval = one (particle, site, observed element) triple.

Prints ONE JSON line (rank 0) with the metric, the roofline of the dominant kernel (timed by span
stamps -- every workgroup of exactly that kernel folds its start and end device clock into a slot
-- in replays of a capture of the same step, after the timed region; HIP events around the kernel
only for eager runs) and the CPU baseline (the reference's torch-CPU semantics, oracle/cpu_port.py,
on a bounded sample, N = 1 only).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import platform
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import mininf_amd  # noqa: E402
import mininf_amd.optim  # noqa: E402
from mininf_amd import _native as nat, engine, rccl  # noqa: E402
from mininf_amd.distributed import GradientBucket  # noqa: E402
from mininf_amd.graph import StepGraph  # noqa: E402
from torch.distributions import Bernoulli, Beta, Normal  # noqa: E402

METRIC = "site-log_prob evals/sec + ELBO step wall-time, 1/2/4/8 MI355X"
UNIT = "site-log_prob evals/s"
PEAK_FP32_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 vector (FMA = 2 FLOP)
PEAK_HBM_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E spec


class EventTimer:
    """
    Times the main site kernel of each launch (engine.KERNEL_TIMER hook), keyed by the group's
    element count N so the dominant kernel can be picked out.

    * Eager steps: (start, stop) HIP event pairs the library records around the kernel
      (mi_group_forward_deferred / mi_linear_forward_deferred).
    * Captured steps (``captured_only``): span stamps -- each launch gets a slot of a device
      buffer into which every workgroup of the kernel folds its start and end time on the device's
      constant-rate clock (mi_group.stamps, s_memrealtime); slot span = last workgroup end minus
      first workgroup start, read after each replay of the captured step. Unlike event-record
      nodes in the graph (which add a dependency boundary on either side of the kernel), the
      stamps leave the replayed step's structure unchanged.
    """
    def __init__(self):
        self.pairs = []
        self.active = False
        self.captured_only = False
        self.slots = []        # (N, K, slot index) handed out during a capture
        self.buffer = None     # int64 [2 * slots] on the device

    def prepare(self, n, device):
        """A stamp buffer of n slots (allocated outside any capture)."""
        self.buffer = torch.zeros(2 * n, dtype=torch.int64, device=device)
        self.slots = []
        self.reset()

    def reset(self):
        if self.buffer is not None:
            self.buffer.view(-1, 2)[:, 0].fill_(torch.iinfo(torch.int64).max)
            self.buffer.view(-1, 2)[:, 1].zero_()

    def pair(self, launcher):
        if not self.active or self.captured_only:
            return None, None
        start = torch.cuda.Event(enable_timing=True)
        stop = torch.cuda.Event(enable_timing=True)
        start.record()   # materialise the underlying hipEvent_t; re-recorded by the library
        stop.record()
        self.pairs.append((launcher.N, launcher.K, start, stop))
        return start, stop

    def stamps(self, launcher):
        if not (self.active and self.captured_only and torch.cuda.is_current_stream_capturing()):
            return None
        j = len(self.slots)
        if self.buffer is None or 2 * j + 2 > self.buffer.numel():
            return None
        self.slots.append((launcher.N, launcher.K, j))
        return self.buffer.data_ptr() + 16 * j

    def spans_ms(self, khz):
        """(N, K, span in ms) of every slot (after a replay)."""
        raw = self.buffer.view(-1, 2).cpu()
        out = []
        for n, k, j in self.slots:
            t0, t1 = int(raw[j, 0]), int(raw[j, 1])
            if t1 > 0 and t1 >= t0:
                out.append((n, k, (t1 - t0) / khz))
        return out

    def times_ms(self, N):
        return [s.elapsed_time(e) for n, _, s, e in self.pairs if n == N]

    def mean_ms(self, N):
        times = self.times_ms(N)
        return sum(times) / len(times) if times else float("nan"), len(times)


class _GcClock:
    """Host time spent in Python's cyclic garbage collector while active (gc.callbacks): part of
    an eager step's cost, reported beside it."""
    def __init__(self):
        self.seconds, self._t0 = 0.0, None

    def _callback(self, phase, info):
        if phase == "start":
            self._t0 = time.perf_counter()
        elif self._t0 is not None:
            self.seconds += time.perf_counter() - self._t0
            self._t0 = None

    def __enter__(self):
        import gc
        gc.callbacks.append(self._callback)
        return self

    def __exit__(self, *exc):
        import gc
        gc.callbacks.remove(self._callback)


class Watchdog:
    """
    Host deadline for every phase of a run ("Next round" 2): a rank whose phase --
    rendezvous, warm-up, capture, a timed loop of replays -- has not finished within its limit
    prints which config and phase it was in (one JSON line on stdout, also on stderr) and ends with
    exit status 3. A collective that never completes (a peer lost inside a captured RCCL
    all-reduce) then fails the run bounded, naming the config, instead of blocking until the
    driver kills it. The exit is os._exit from this thread: the main thread may be blocked inside a
    HIP or RCCL call that cannot be unwound; nothing is re-executed.
    """
    def __init__(self, rank: int, limit_s: float) -> None:
        import threading
        self.rank, self.limit_s = rank, limit_s
        self._cond = threading.Condition()
        self._phase, self._deadline = None, None
        self._thread = threading.Thread(target=self._run, name="bench-watchdog", daemon=True)
        self._thread.start()

    def arm(self, phase: str, seconds: float | None = None) -> None:
        with self._cond:
            self._phase = phase
            self._deadline = time.monotonic() + (seconds or self.limit_s)
            self._cond.notify()

    def disarm(self) -> None:
        with self._cond:
            self._phase, self._deadline = None, None
            self._cond.notify()

    def _run(self) -> None:
        while True:
            with self._cond:
                if self._deadline is None:
                    self._cond.wait()
                    continue
                left = self._deadline - time.monotonic()
                if left > 0:
                    self._cond.wait(left)
                    continue
                phase = self._phase
            line = json.dumps({"metric": METRIC, "error": "deadline", "rank": self.rank,
                               "phase": phase, "limit_s": self.limit_s})
            print(line, flush=True)
            print(f"bench.py rank {self.rank}: {phase} did not finish within {self.limit_s:.0f} s",
                  file=sys.stderr, flush=True)
            os._exit(3)


WATCHDOG: Watchdog | None = None


def arm(phase: str) -> None:
    if WATCHDOG is not None:
        WATCHDOG.arm(phase)


def wait_device(device) -> None:
    """torch.cuda.synchronize() as an event poll: the host keeps running Python (and the
    watchdog its deadline) while the device drains. The first 20 ms poll without sleeping: a
    sleep of 20 us lasts ~60-80 us on this host (timer slack), which the end of a short timed
    region (the driver's 20-step run: ~1.8 ms) would count as step time."""
    event = torch.cuda.Event()
    event.record(torch.cuda.current_stream(device))
    t0 = time.perf_counter()
    while not event.query():
        if time.perf_counter() - t0 > 0.02:
            time.sleep(20e-6)


# ------------------------------------------------------------------------------------------------
# Workloads (restated from the reference's README / examples).
# ------------------------------------------------------------------------------------------------
def workload(name, device, world, rank):
    gen = torch.Generator().manual_seed(0)
    if name in ("c1", "c2"):
        n = 10 if name == "c1" else 1_000_000
        k_local = 1 if name == "c1" else 4096
        x = (torch.rand(n, generator=gen) < 0.7).float().to(device)

        def model():
            theta = mininf_amd.sample("theta", Beta(2, 2))
            mininf_amd.sample("x", Bernoulli(theta), sample_shape=[n])

        guide = mininf_amd.nn.ParameterizedDistribution(Beta, concentration0=2.0,
                                                        concentration1=2.0).to(device)
        conditioned = mininf_amd.condition(model, x=x)
        return dict(
            desc=f"{name.upper()} Beta-Bernoulli (README model), n={n}, {k_local} particles/GPU",
            k_local=k_local, n=n, module=guide, guide=lambda: {"theta": guide()},
            conditioned=lambda: conditioned, evals=k_local * (n + 1), lr=0.02,
            dominant_N=n, bound="valu", flops_per_eval=2.0, bytes_per_eval=0.0,
            kernel=("k_site_bcast_smem<Bernoulli-probs> (per-particle logits x shared data read by "
                    "the scalar unit, v_pk_fma_f32 on SGPR pairs)"),
            flop_note="2 FLOP/eval (one FMA) x K x n",
            data=f"synthetic: x ~ Bernoulli(0.7)[{n}] fp32 (seed 0); Beta(2,2) guide init")
    if name in ("c3", "c4"):
        p = 32
        if name == "c3":
            n_total, n_obs, k_local = 1_000_000, 1_000_000, 256
        else:
            n_total, n_obs, k_local = 10_000_000, 65536, 32
        X = torch.randn(n_total, p, generator=gen)
        true = torch.randn(p, generator=gen)
        y = X @ true + torch.randn(n_total, generator=gen)
        X, y = X.to(device), y.to(device)

        def model():
            theta = mininf_amd.sample("theta", Normal(0, 1), sample_shape=p)
            with mininf_amd.batch(n_total):
                with mininf_amd.no_log_prob():
                    Xs = mininf_amd.sample("X", Normal(0, 1), sample_shape=(n_total, p))
                mininf_amd.sample("y", Normal(Xs @ theta, 1))

        guide = mininf_amd.nn.ParameterizedDistribution(
            Normal, loc=1e-3 * torch.randn(p, generator=gen),
            scale=(1e-3 * torch.randn(p, generator=gen)).exp()).to(device)
        blocks = n_total // n_obs
        if n_obs == n_total:
            static = mininf_amd.condition(model, X=X, y=y)

            def conditioned():
                return static
        elif device.type == "cuda":
            # Device-resident minibatches (mininf_amd.DeviceDataLoader, replacing the host
            # DataLoader(TensorDataset(X, y), batch_size, shuffle=True) of
            # examples/minibatch.md:78): the rows of each batch are drawn on the device and read
            # by the linear site kernel through the index, so a captured step trains on a new
            # shuffled batch on every replay.
            loader = mininf_amd.DeviceDataLoader(X, y, batch_size=n_obs, shuffle=True,
                                                 drop_last=True, seed=0)

            def conditioned():
                Xb, yb = loader.next()
                return mininf_amd.condition(model, X=Xb, y=yb)
        else:   # the CPU baseline: the reference's host semantics, contiguous windows
            counter = [0]

            def conditioned():
                start = (counter[0] * 7919) % blocks * n_obs
                counter[0] += 1
                return mininf_amd.condition(model, X=X[start:start + n_obs],
                                            y=y[start:start + n_obs])

        return dict(
            desc=(f"{name.upper()} Bayesian linear regression, {n_total}x{p} (minibatch {n_obs}), "
                  f"MF Normal guide, {k_local} particles/GPU"),
            k_local=k_local, n=n_obs, module=guide, guide=lambda: {"theta": guide()},
            conditioned=conditioned, evals=k_local * (n_obs + p), lr=0.01,
            dominant_N=n_obs, bound="mfma", flops_per_eval=4.0 * p, bytes_per_eval=0.0,
            kernel=("k_linear_mfma<Normal> (X @ theta evaluated in the site kernel on "
                    "v_mfma_f32_32x32x2_f32: MU = X theta^T, the residual in the accumulators, "
                    "dtheta = R^T X; 2 FMA per feature per eval)"),
            flop_note=f"{4 * p} FLOP/eval (2 x {p} FMA) x K x n",
            data=f"synthetic: X ~ N(0,1)[{n_total},{p}], y = X theta* + N(0,1) (seed 0)")
    if name == "c5":
        n = 1_000_000
        mu_true = torch.randn((), generator=gen)
        z_true = mu_true + torch.randn(n, generator=gen)
        y = z_true + 0.5 * torch.randn(n, generator=gen)
        b = (torch.rand(n, generator=gen) < torch.sigmoid(z_true)).float()
        mask = torch.rand(n, generator=gen) > 0.2
        shard = data_shard(n, world, rank) if name == "c5" and DATA_SHARD else None
        if shard is None:   # particle sharding: every rank holds every element, K / W particles
            k_local, sl, n_loc, layout = 128, slice(None), n, "particle-sharded"
        else:   # data sharding: the rank's element slice, all particles (DataShard)
            k_local, sl, n_loc = 1024, shard.slice, shard.size
            layout = (f"data-sharded: elements [{shard.start}, {shard.stop}) of {n} "
                      f"(rank {DATA_SHARD_RANK if world == 1 else rank} of {shard.world})")
        y, b, mask = y[sl].to(device), b[sl].to(device), mask[sl].to(device)
        ym = torch.masked.as_masked_tensor(y, mask)
        bm = torch.masked.as_masked_tensor(b, mask)

        def model():
            mu = mininf_amd.sample("mu", Normal(0, 1))
            z = mininf_amd.sample("z", Normal(mu, 1), sample_shape=[n_loc])
            mininf_amd.sample("y", Normal(z, 0.5))
            mininf_amd.sample("b", Bernoulli(logits=z))

        guide = mininf_amd.nn.ParameterizedFactorizedDistribution(
            mu=mininf_amd.nn.ParameterizedDistribution(Normal, loc=0.0, scale=1.0),
            z=mininf_amd.nn.ParameterizedDistribution(Normal, loc=torch.zeros(n_loc),
                                                      scale=torch.ones(n_loc)),
        ).to(device)
        conditioned = mininf_amd.condition(model, y=ym, b=bm)
        observed = int(mask.sum())
        return dict(
            desc=f"C5 masked hierarchical model, n={n}, {k_local} particles/GPU, {layout}",
            k_local=k_local, n=n_loc, module=guide, guide=lambda: guide(),
            conditioned=lambda: conditioned, shard=shard,
            reduce_params=list(guide["mu"].parameters()) if shard is not None else None,
            evals=k_local * (1 + n_loc + 2 * observed), lr=0.01, dominant_N=n_loc, bound="valu",
            flops_per_eval=37.0, bytes_per_eval=None, observed=observed,
            kernel=("mi_site_program (fused z / y / b site group with the z ~ q(z) draw computed "
                    "in registers: Philox + Box-Muller, three log densities, dloc / dscale "
                    "reduced over particles)"),
            flop_note=("37 FLOP per (particle, element): Box-Muller 5, z = loc + eps scale 2, "
                       "Normal(z|mu,1) 7, Normal(y|z,.5) 6, Bernoulli(b|logits z) 11, "
                       "accumulation 6; Philox integer rounds not counted"),
            data=f"synthetic: y ~ N(z, 0.5), b ~ Bernoulli(logits=z), 20% masked (seed 0)")
    raise SystemExit(f"unknown config {name}")


# C5 layout (--shard): "particles" (default: every rank all elements, K / W particles) or "data"
# (DataShard: every rank all K particles on its element slice; --shard-world W with one process
# measures rank --shard-rank's slice of a W-rank run on one GPU, without the all-reduce)
DATA_SHARD = False
DATA_SHARD_WORLD = 0
DATA_SHARD_RANK = 0


def data_shard(n, world, rank):
    from mininf_amd.distributed import element_shard
    if world == 1 and DATA_SHARD_WORLD > 1:
        return element_shard(n, shared=("mu",), world=DATA_SHARD_WORLD, rank=DATA_SHARD_RANK)
    return element_shard(n, shared=("mu",), world=world, rank=rank)


def measured_issue(name):
    """
    The VALU pipe's busy fraction of the dominant kernel by the issue-cost model (profiles/
    summarize.py: SQ instruction counts by type weighted by their measured issue cycles, over the
    kernel's cycles on all SIMDs), from the newest committed profiles/rNN_valu_pmc.json that has
    it for this config; None otherwise.
    """
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_valu_pmc.json")),
                       reverse=True):
        with open(path) as fh:
            entry = json.load(fh).get(name) or {}
        if "valu_busy" in entry:
            return entry["valu_busy"], os.path.relpath(path, ROOT)
    return None, None


def measured_traffic(name):
    """
    HBM bytes per launch of the dominant kernel from the newest committed PMC summary
    (profiles/rNN_pmc.json, written by profiles/summarize.py from separate rocprofv3
    --pmc FETCH_SIZE / WRITE_SIZE passes of this bench, FETCH_SIZE doubled per the gfx950
    correction). None when that config has not been profiled.
    """
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as fh:
        entry = json.load(fh).get(name)
    if entry is None or "traffic_bytes_per_launch" not in entry:
        return None, None
    return entry["traffic_bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def host_cpus():
    """
    The CPUs this process may use: its affinity set, capped by a cgroup CPU quota when one is set
    (os.cpu_count() counts every CPU of the machine, also those a container cannot run on).
    """
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_baseline(name, budget_s=12.0):
    """
    The reference's semantics on the host cores (oracle/cpu_port.py): K_cpu single-draw losses per
    step, timed on a bounded sample; reported as evals/s of the same workload. Every CPU this
    process may use runs torch's intra-op threads.
    """
    from oracle import cpu_port
    torch.set_num_threads(host_cpus())
    cpu = torch.device("cpu")
    w = workload(name, cpu, 1, 0)
    k_cpu = min(w["k_local"], 16)
    optimizer = torch.optim.Adam(w["module"].parameters(), lr=w["lr"])
    steps = 0
    evals_per_particle = w["evals"] / w["k_local"]
    cpu_port.k_particle_step(w["conditioned"](), w["guide"], optimizer, 1)   # warm-up
    start = time.perf_counter()
    while True:
        cpu_port.k_particle_step(w["conditioned"](), w["guide"], optimizer, k_cpu)
        steps += 1
        elapsed = time.perf_counter() - start
        if elapsed > budget_s or steps >= 2000:
            break
    rate = evals_per_particle * k_cpu * steps / elapsed
    model_name = ""
    try:
        with open("/proc/cpuinfo") as fh:
            model_name = next(line.split(":", 1)[1].strip() for line in fh
                              if line.startswith("model name"))
    except (OSError, StopIteration):
        model_name = platform.processor()
    return {"value": rate, "unit": UNIT, "cores": torch.get_num_threads(), "kind": "port",
            "sample": (f"{steps} steps x {k_cpu} single-draw particles of {w['desc']} in "
                       f"{elapsed:.1f} s (reference semantics, torch {torch.__version__} CPU, "
                       f"{torch.get_num_threads()} threads = the CPUs available to this process "
                       f"(affinity and cgroup quota; os.cpu_count()={os.cpu_count()}), "
                       f"{model_name})"),
            "ms_per_step_extrapolated": 1e3 * elapsed / steps * w["k_local"] / k_cpu}


def launch_ranks(n):
    """
    Run this command as ``torch.distributed.run --nproc-per-node n`` in a child process (the
    driver's own launch form) and return its exit status. The parent never touches the GPU.
    """
    import socket
    import subprocess
    with socket.socket() as sock:
        sock.bind(("127.0.0.1", 0))
        port = sock.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd, env=dict(os.environ))


def check_launch(args, world, rank):
    """--check-launch: the ranks meet, sum their ranks with one all-reduce, rank 0 prints."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([float(rank)])
    if world > 1:
        dist.all_reduce(t)
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"metric": METRIC, "n_gpus": world, "check_launch": True,
                          "rank_sum": float(t)}), flush=True)
    return 0


_COMMUNICATOR = None


def communicator(group, device, kind="rccl"):
    """The run's one communicator, shared by every config (graphs of an earlier config may still
    hold its captured collective): RCCL called directly (mininf_amd.rccl), or with
    ``--allreduce peer`` the one-shot peer-write all-reduce (mininf_amd.peer, opt-in)."""
    global _COMMUNICATOR
    if _COMMUNICATOR is None:
        if kind == "peer":
            from mininf_amd.peer import PeerCommunicator
            _COMMUNICATOR = PeerCommunicator(group, device)
        else:
            _COMMUNICATOR = rccl.Communicator(group, device)
    return _COMMUNICATOR


def run_config(config, args, world, rank, device, group, steps, warmup, cpu_budget):
    """Measure one workload (all ranks); rank 0 gets the bench line's dict."""
    arm(f"{config}: set-up")
    w = workload(config, device, world, rank)
    if args.particles_per_gpu:
        w["evals"] = w["evals"] // w["k_local"] * args.particles_per_gpu
        w["k_local"] = args.particles_per_gpu
    module = w["module"]
    if args.optimizer == "torch":
        optimizer = torch.optim.Adam(module.parameters(), lr=w["lr"], capturable=True, fused=True)
    else:   # the same Adam in one HIP launch (mininf_amd.optim, bit-identical to torch's fused)
        optimizer = mininf_amd.optim.Adam(module.parameters(), lr=w["lr"])
    shard = w.get("shard")
    loss_fn = mininf_amd.nn.EvidenceLowerBoundLoss(
        num_particles=w["k_local"] * (world if shard is None else 1), seed=1,
        validate=not args.no_validate, process_group=group, data_shard=shard)
    timer = EventTimer()
    engine.KERNEL_TIMER = timer

    # N > 1: the rank's gradients and its loss share are packed into ONE flat bucket
    # (distributed.GradientBucket), all-reduced once, and Adam runs on gradients bound to the
    # reduced bucket. Over RCCL the whole step -- collective included -- is one captured graph
    # (several steps per replay, like N = 1); gloo cannot be captured, so there the step is split
    # around the host-issued all-reduce (two graphs).
    sharded = group is not None
    collective_in_graph = sharded and (args.dist_backend == "nccl" or args.allreduce == "peer")
    # over RCCL the all-reduce runs on a communicator of our own (mininf_amd.rccl: RCCL called
    # directly, no process-group watchdog polling events of the captured collective); the peer
    # all-reduce is one kernel of ours, captured the same way whatever the process group's backend
    comm = communicator(group, device, args.allreduce) if collective_in_graph else None
    # data sharding reduces only the replicated (shared) parameters' gradients; every rank
    # updates its own slice of the rest
    bucket = GradientBucket(w.get("reduce_params") or module.parameters(), group, with_loss=True,
                            communicator=comm) if sharded else None

    def forward_backward():
        optimizer.zero_grad(set_to_none=True)
        loss = loss_fn(w["conditioned"](), w["guide"]())
        loss.backward()
        if not sharded:
            optimizer.step()
        else:
            bucket.pack(loss)
        return loss

    def apply_update():
        bucket.bind()
        optimizer.step()

    def full_step():
        loss = forward_backward()
        if not sharded:
            return loss
        bucket.all_reduce()
        apply_update()
        return bucket.loss()   # the global loss (sum of the ranks' shares)

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        wait_device(device)

    def timed(run, steps):
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = run()
        barrier()
        seconds = time.perf_counter() - t0
        if world > 1:
            import torch.distributed as dist
            t = torch.tensor([seconds], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            seconds = float(t)
        return seconds, out

    def warm_replays(replay, count):
        """`count` replays, then as many more as fill --warm-ms at the measured replay time: the
        timed replays start with the clocks and caches at their steady state. Every rank runs the
        same number (the slowest rank's replay time): a sharded replay holds a collective."""
        t0 = time.perf_counter()
        for _ in range(count):
            replay()
        barrier()
        per = (time.perf_counter() - t0) / count
        if world > 1:
            import torch.distributed as dist
            t = torch.tensor([per], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            per = float(t)
        extra = 0 if args.warm_ms <= 0 else \
            min(10000, max(0, math.ceil((args.warm_ms / 1e3 - per * count) / per)))
        for i in range(extra):
            replay()
            if i % 8 == 7:
                wait_device(device)
        barrier()

    def eager_step():
        # detached: keep no autograd graph alive across steps (graph capture needs it)
        return full_step().detach()

    # Eager steps: every kernel launched from Python (the kernel timing comes from these).
    arm(f"{config}: eager warm-up")
    for _ in range(warmup):
        eager_step()
    wait_device(device)
    arm(f"{config}: timed eager steps")
    eager_steps = max(3, steps // 3) if args.graph else steps
    gc_clock = _GcClock()
    with gc_clock:
        eager_elapsed, loss = timed(eager_step, eager_steps)
    # a copy: the sharded step's loss is a view into the gradient bucket, which later steps
    # (the kernel-timed ones) overwrite
    loss = loss.detach().clone()
    eager_ms = 1e3 * eager_elapsed / eager_steps
    wait_device(device)

    def kernel_timed_steps():
        """--eager (and split-graph gloo) runs: the kernel durations from further eager steps with
        a HIP event pair around the dominant launch, outside every timed region (the events cost
        host time per launch)."""
        arm(f"{config}: kernel-timed eager steps")
        timer.active = True
        for _ in range(eager_steps):
            eager_step()
        timer.active = False
        wait_device(device)

    kernel_source = "eager steps (HIP events around the kernel)"

    def kernel_timed_replays(repeat, replays=16):
        """The dominant kernel's duration AS REPLAYED: the step captured once more with a span-stamp
        slot per site launch (EventTimer.captured_only: every workgroup folds its start / end
        clock into the slot), then replayed `replays` times after the timed region, the slots
        reset before and read after each replay. The same kernels, grid and step structure as
        the timed graph."""
        arm(f"{config}: kernel-timed graph replays")
        timer.prepare(8 * repeat, device)
        timer.active, timer.captured_only = True, True
        try:
            timing_graph = StepGraph(full_step, warmup=1, repeat=repeat,
                                     capture_error_mode="thread_local" if sharded else "global")
        finally:
            timer.active, timer.captured_only = False, False
        khz = ctypes.c_int(0)
        nat.check(nat.lib().mi_wall_clock_khz(ctypes.byref(khz)), "mi_wall_clock_khz")
        samples = []
        for i in range(replays + 2):
            timer.reset()
            timing_graph()
            wait_device(device)
            if i >= 2:   # (the first replays after a capture are not steady)
                samples += timer.spans_ms(khz.value)
        timing_graph.check()
        return samples

    if not args.graph:
        kernel_timed_steps()
    elapsed, mode = eager_elapsed * steps / eager_steps, "eager"
    if args.graph:
        # The same step captured once into a hipGraph and replayed (mininf_amd.graph.StepGraph).
        # one replay = `repeat` consecutive steps (N = 1): each graph launch leaves the device
        # idle ~13 us, which a launch-bound step amortises (mininf_amd.graph.StepGraph)
        repeat = 1
        if not sharded or collective_in_graph:
            # the largest divisor of --steps up to 24: the driver's 20-step run is one replay
            # (tools/gpurun_r05/t19.sh: 5 steps per replay 94.7-98.1 us per C2 step, 20 per
            # replay 94.5-95.9)
            repeat = args.graph_repeat or next(r for r in range(min(24, steps), 0, -1)
                                               if steps % r == 0)
            if steps % repeat:
                raise SystemExit(f"--graph-repeat {repeat} does not divide --steps {steps}")
        arm(f"{config}: graph capture")
        if not sharded or collective_in_graph:
            # RCCL's watchdog thread polls events during the capture: thread-local capture mode
            graph_step = StepGraph(full_step, warmup=2, repeat=repeat,
                                   capture_error_mode="thread_local" if sharded else "global")
            captured = graph_step
        else:
            # warm-up with whole steps (all-reduce and update included), so the training state
            # advances as in the captured N = 1 / RCCL steps; the update graph needs none
            captured = StepGraph(forward_backward, warmup=2, warmup_step=full_step)
            update = StepGraph(apply_update, warmup=0)

            def graph_step():
                captured()
                bucket.all_reduce()
                update()
                return bucket.loss()

        arm(f"{config}: graph warm-up replays")
        warm_replays(graph_step, max(1, warmup // repeat))
        arm(f"{config}: timed graph replays ({steps // repeat} replays of {repeat} steps)")
        elapsed, loss = timed(graph_step, steps // repeat)
        loss = loss.detach().clone()   # (see above; the graph's own output is static as well)
        captured.check()
        if comm is not None and hasattr(comm, "check"):
            comm.check()   # (the peer all-reduce's timeout word)
        mode = "hipGraph replay" + (f" ({repeat} steps per replay)" if repeat > 1 else "")
        if sharded:
            what = "peer-write" if args.allreduce == "peer" else "RCCL"
            mode += (f" with the {what} all-reduce captured in the graph" if collective_in_graph
                     else f" split around the host-issued {args.dist_backend} all-reduce")
        floor_ms = None
        if config == "c2" and not sharded:
            # C2's per-eval sum over x_i l_k is reducible to l_k sum_i x_i:
            # the same step with the site kernel's closed form, reported beside the per-eval number
            os.environ["MININF_AMD_BCAST_SUFFSTAT"] = "1"
            arm(f"{config}: reducible-floor graph")
            try:
                floor_graph = StepGraph(forward_backward, warmup=2, repeat=repeat)
                warm_replays(floor_graph, max(1, warmup // repeat))
                floor_s, _ = timed(floor_graph, steps // repeat)
                floor_graph.check()
                floor_ms = 1e3 * floor_s / steps
            finally:
                del os.environ["MININF_AMD_BCAST_SUFFSTAT"]
        if not sharded or collective_in_graph:
            replay_samples = kernel_timed_replays(repeat)
            kernel_source = (f"graph replays (span stamps: first workgroup start to last "
                             f"workgroup end on the device clock, in a capture of the same step, "
                             f"{repeat} steps per replay)")
        else:
            kernel_timed_steps()

    if args.profile_host and rank == 0:
        import cProfile
        import pstats
        profiler = cProfile.Profile()
        profiler.enable()
        for i in range(20):
            eager_step()
        torch.cuda.synchronize()
        profiler.disable()
        pstats.Stats(profiler, stream=sys.stderr).sort_stats("tottime").print_stats(30)
        pstats.Stats(profiler, stream=sys.stderr).sort_stats("cumulative").print_stats(45)

    ms = 1e3 * elapsed / steps
    evals_all = w["evals"] * world
    if world > 1:   # data-sharded slices differ by an element or an observation: count them all
        import torch.distributed as dist
        t = torch.tensor([float(w["evals"])], device=device, dtype=torch.float64)
        dist.all_reduce(t)
        evals_all = float(t)
    value = evals_all * steps / elapsed
    if args.graph and (not sharded or collective_in_graph):
        times = [t for n, _, t in replay_samples if n == w["dominant_N"]]
        kernel_ms = sum(times) / len(times) if times else float("nan")
        launches = len(times)
    else:
        kernel_ms, launches = timer.mean_ms(w["dominant_N"])
    kernel_s = kernel_ms * 1e-3
    if w["bound"] in ("valu", "mfma"):
        # FP32 VALU (v_pk_fma_f32) and FP32 MFMA (v_mfma_f32_32x32x2_f32) share the 157.3 TFLOP/s
        # dense peak on MI355X (MI355X_MICROARCH.md)
        flops = w["flops_per_eval"] * w["k_local"] * w["n"]
        achieved = flops / kernel_s / 1e12
        roof = {"bound": w["bound"], "achieved": achieved, "peak": PEAK_FP32_TFLOPS,
                "unit": "TFLOP/s", "frac": achieved / PEAK_FP32_TFLOPS, "traffic": None,
                "kernel": w["kernel"], "kernel_ms": kernel_ms, "launches_timed": launches,
                "kernel_timing": kernel_source,
                "algorithmic_per_launch": f"{flops:.4g} FLOP ({w['flop_note']})"}
    else:
        nbytes = w["bytes_per_launch"]
        achieved = nbytes / kernel_s / 1e9
        roof = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS, "traffic": None, "kernel": w["kernel"],
                "kernel_ms": kernel_ms, "launches_timed": launches,
                "kernel_timing": kernel_source,
                "algorithmic_per_launch": f"{nbytes:.4g} B"}
    if config == "c5":
        # the FLOP count prices transcendentals at 1 and omits the Philox integer work, so it is
        # not the issue-bound resource: the issue model's busy fraction is the bound's fraction
        busy, busy_source = measured_issue(config)
        if busy is not None:
            roof["valu_busy"] = busy
            roof["valu_busy_source"] = (f"{busy_source} (rocprofv3 --pmc SQ_INSTS_VALU by type x "
                                        "measured issue cycles / kernel SIMD cycles)")
    if config == "c4":
        roof["kernel_timing"] += ("; the stamps span first workgroup start to last workgroup end "
                                  "and exclude the dispatch (rocprofv3's trace includes it: "
                                  "~2 us more for this ~24 us launch)")
    traffic, source = measured_traffic(config)
    roof["traffic"] = traffic
    if traffic is not None:
        roof["traffic_source"] = f"{source} (rocprofv3 --pmc, bytes per launch)"
    out = {
        "metric": METRIC, "value": value, "unit": UNIT, "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": w["data"],
        "config": {"workload": w["desc"], "particles_per_gpu": w["k_local"],
                   "global_particles": w["k_local"] * (world if shard is None else 1),
                   "evals_per_step_per_gpu": w["evals"],
                   "parallelism": (f"particle-sharded x{world}" if shard is None else
                                   f"data-sharded x{shard.world} (element slices)") + (
                       (" + peer-write grad all-reduce" if args.allreduce == "peer" else
                        " + RCCL grad all-reduce" if args.dist_backend == "nccl" else
                        f" + {args.dist_backend} grad all-reduce") if sharded else ""),
                   "validate": not args.no_validate, "final_loss": float(loss.detach()),
                   "step_mode": mode, "eager_ms_per_step": eager_ms,
                   "fusions": loss_fn.last_fusions,
                   "eager_gc_ms_per_step": gc_clock.seconds * 1e3 / eager_steps,
                   **({"reducible_floor_ms_per_step": floor_ms,
                       "reducible_floor_note": "the same step with the site kernel evaluating "
                       "sum_i x_i l_k as l_k sum_i x_i (MININF_AMD_BCAST_SUFFSTAT=1); value and "
                       "roofline are the per-eval path"} if args.graph and floor_ms is not None
                      else {}),
                   "optimizer": ("mininf_amd.optim.Adam (one HIP launch)" if args.optimizer == "mi"
                                 else "torch.optim.Adam(fused=True)")},
        "roofline": roof,
    }
    out["config"]["ranks"] = world
    out["scaling"] = "weak" if shard is None else "strong"
    if WATCHDOG is not None:
        WATCHDOG.disarm()
    if rank == 0 and world == 1 and cpu_budget > 0:
        out["cpu_baseline"] = cpu_baseline(config, cpu_budget)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--graph-repeat", type=int, default=0,
                    help="steps captured per graph replay (0: the largest divisor of --steps up to 24)")
    ap.add_argument("--steps", type=int, default=240)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--warm-ms", type=float, default=50.0,
                    help="graph warm-up: replay until the device has run this long (ms)")
    ap.add_argument("--config", default="c2")
    ap.add_argument("--no-validate", action="store_true")
    ap.add_argument("--eager", dest="graph", action="store_false",
                    help="launch every step from Python instead of replaying a captured hipGraph")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="default C2 run: skip measuring C3 / C4 / C5 after it")
    ap.add_argument("--dist-backend", default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo lets "
                         "several ranks share one GPU to exercise the sharded path)")
    ap.add_argument("--allreduce", choices=("rccl", "peer"), default="rccl",
                    help="N > 1: the gradient bucket's all-reduce -- RCCL (nccl backend) or the "
                         "one-shot peer-write kernel (mininf_amd.peer, any backend; opt-in, "
                         "unmeasured on multi-GPU hardware)")
    ap.add_argument("--optimizer", choices=("mi", "torch"), default="mi",
                    help="Adam implementation: mininf_amd.optim.Adam (one HIP launch, default) or "
                         "torch.optim.Adam(fused=True, capturable=True)")
    ap.add_argument("--particles-per-gpu", type=int, default=0,
                    help="override the config's particles per GPU (0: the config's own)")
    ap.add_argument("--shard", choices=("auto", "particles", "data"), default="auto",
                    help="C5 layout over ranks: particles (K / W each) or data (element slices, "
                         "all K particles each: mininf_amd.distributed.DataShard); auto = data "
                         "for C5 at N > 1 (measured faster per GPU, and its all-reduce carries 3 "
                         "values instead of 2e6), particles otherwise")
    ap.add_argument("--shard-world", type=int, default=0,
                    help="with --shard data on ONE process: measure the slice of a run over this "
                         "many ranks (rank --shard-rank), without the all-reduce")
    ap.add_argument("--shard-rank", type=int, default=0)
    ap.add_argument("--process-group", action="store_true",
                    help="run the sharded step (process group, gradient bucket, all-reduce) even "
                         "at N = 1: measures the N > 1 step's own overhead on one GPU")
    ap.add_argument("--profile-host", action="store_true",
                    help="cProfile 20 extra steps and print the hottest host functions to stderr")
    ap.add_argument("--deadline", type=float, default=120.0,
                    help="seconds any phase (rendezvous, warm-up, capture, a timed loop) may take "
                         "before the rank prints the config and phase and exits with status 3")
    ap.add_argument("--check-launch", action="store_true",
                    help="rendezvous and one all-reduce only, no GPU work: prints the line's "
                         "n_gpus (tests the --gpus launch path on a CPU host)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` on its own: start the N ranks as child processes (one per
        # GPU) before this process touches the GPU, and exit with their status.
        raise SystemExit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were started")
    if args.check_launch:
        raise SystemExit(check_launch(args, world, rank))
    global WATCHDOG
    WATCHDOG = Watchdog(rank, args.deadline)
    global DATA_SHARD, DATA_SHARD_WORLD, DATA_SHARD_RANK
    # (the layout applies to C5 only, also when C5 runs after the default C2 line)
    DATA_SHARD = args.shard == "data" or (args.shard == "auto" and
                                          (world > 1 or args.shard_world > 1))
    DATA_SHARD_WORLD, DATA_SHARD_RANK = args.shard_world, args.shard_rank
    device = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(device)
    group = None
    if world > 1 or args.process_group:
        import datetime
        import torch.distributed as dist
        arm("process-group rendezvous")
        init = {"timeout": datetime.timedelta(seconds=args.deadline)}
        if "MASTER_ADDR" not in os.environ:   # --process-group without a launcher: one rank
            import socket
            with socket.socket() as sock:
                sock.bind(("127.0.0.1", 0))
                port = sock.getsockname()[1]
            init.update(init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device, **init)
        else:
            dist.init_process_group(args.dist_backend, **init)
        group = dist.group.WORLD

    out = run_config(args.config, args, world, rank, device, group, args.steps, args.warmup,
                     0.0 if args.no_cpu_baseline else 12.0)
    others = ()
    if args.config == "c2" and not args.no_other_configs:
        # the other configurations of BASELINE.json, measured in the same run (the same number
        # of graph-replayed steps -- with 10 the fixed cost of the timed region's barriers and
        # synchronisations added 5-9 us to C4's 40 us step; CPU baseline only for C3 at
        # N = 1): C3 is a one-GPU config;
        # C4 (particle-sharded, 32 particles per GPU: 256 at N = 8) and C5 (data-sharded, all
        # 1024 particles on each rank's element slice) are the multi-GPU ones
        others = ("c3", "c4", "c5") if world == 1 and group is None else ("c4", "c5")
    if others:
        out["other_configs"] = {}
        for name in others:
            sub = run_config(name, args, world, rank, device, group, args.steps, 3,
                             0.0 if (args.no_cpu_baseline or name != "c3") else 8.0)
            out["other_configs"][name] = {key: sub[key] for key in (
                "value", "unit", "ms_per_step", "scaling", "config", "roofline", "cpu_baseline")
                if key in sub}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if group is not None:
        import torch.distributed as dist
        arm("process-group teardown")
        dist.destroy_process_group()
    WATCHDOG.disarm()


if __name__ == "__main__":
    main()
