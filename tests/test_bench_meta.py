"""
bench.py's host-side bookkeeping (CPU): the committed PMC summary it reads the roofline `traffic`
from exists and covers the configs whose dominant kernel was profiled.
"""
import importlib.util
import os

from tests.conftest import ROOT


def load_bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    module = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(module)
    return module


def test_measured_traffic_reads_the_pmc_summary():
    bench = load_bench()
    for cfg in ("c2", "c3", "c5"):
        traffic, source = bench.measured_traffic(cfg)
        assert traffic is not None and traffic > 0, cfg
        assert source.startswith("profiles/r") and source.endswith("_pmc.json")
    assert bench.measured_traffic("c1") == (None, None)


def _bench(*argv, env_extra=None):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], env=env,
                          capture_output=True, text=True, timeout=300)


def test_bench_gpus_flag_starts_that_many_ranks():
    """`bench.py --gpus 2` on its own starts two ranks (torch.distributed.run child process) and
    the line reports n_gpus 2 (--gpus was ignored)."""
    import json
    out = _bench("--gpus", "2", "--dist-backend", "gloo", "--check-launch")
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["rank_sum"] == 1.0


def test_bench_rejects_a_world_size_mismatch():
    out = _bench("--gpus", "4", "--check-launch", env_extra={"WORLD_SIZE": "2", "RANK": "0"})
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr


def test_bench_watchdog_ends_a_stuck_phase():
    """bench.Watchdog: a phase that overruns its limit prints the phase as JSON and the process
    exits with status 3 (a hung collective fails the run bounded, VERDICT r03 "Next round" 2)."""
    import json
    import subprocess
    import sys
    code = ("import importlib.util, time, sys\n"
            f"spec = importlib.util.spec_from_file_location('bench', {os.path.join(ROOT, 'bench.py')!r})\n"
            "b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)\n"
            "w = b.Watchdog(5, 0.5)\n"
            "w.arm('c4: timed graph replays')\n"
            "time.sleep(30)\n"
            "sys.exit(0)\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert out.returncode == 3, (out.stdout, out.stderr)
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["error"] == "deadline" and line["phase"] == "c4: timed graph replays"
    assert line["rank"] == 5
    assert "did not finish" in out.stderr


def test_bench_watchdog_disarmed_phase_does_not_fire():
    bench = load_bench()
    import time
    w = bench.Watchdog(0, 0.2)
    w.arm("quick phase")
    w.disarm()
    time.sleep(0.5)   # still alive: the disarmed deadline never fires
    w.arm("another", seconds=60)
    w.disarm()
