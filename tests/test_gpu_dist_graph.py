"""
The N > 1 training step on the GPU ("Next round" 1):

* the whole sharded step with the RCCL all-reduce captured inside the hipGraph, several steps per
  replay, against the same steps run eagerly (a one-rank nccl group, tests/rccl_capture_check.py);
* bench.py's sharded path end to end: two gloo ranks sharing the GPU (particles split 32 + 32)
  against one rank with all 64 particles: the same final loss within 1e-5 (the guide generator is
  keyed by the global particle index, the minibatch order by the shared seed).

Each check runs in a child process with its own time limit, so a collective that hangs cannot
take the test session with it.
"""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _last_json(out):
    assert out.returncode == 0, (out.stdout[-3000:], out.stderr[-3000:])
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_rccl_all_reduce_captured_in_step_graph(device):
    out = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "rccl_capture_check.py")],
                         env=_env(), capture_output=True, text=True, timeout=240)
    line = _last_json(out)
    for got, want in zip(line["graph_losses"], line["eager_losses"]):
        assert got == pytest.approx(want, rel=1e-6, abs=1e-6), line
    assert line["param_max_abs_diff"] <= 1e-6, line


def _bench(*argv):
    return subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), *argv],
                          env=_env(), capture_output=True, text=True, timeout=280)


def test_bench_two_gloo_ranks_match_one_rank(device):
    common = ["--config", "c4", "--steps", "4", "--warmup", "2", "--graph-repeat", "1",
              "--no-other-configs", "--no-cpu-baseline"]
    two = _last_json(_bench("--gpus", "2", "--dist-backend", "gloo", "--particles-per-gpu", "32",
                            *common))
    one = _last_json(_bench("--particles-per-gpu", "64", *common))
    assert two["n_gpus"] == 2 and two["config"]["global_particles"] == 64
    assert one["n_gpus"] == 1 and one["config"]["global_particles"] == 64
    assert "gloo all-reduce" in two["config"]["step_mode"]
    assert two["config"]["final_loss"] == pytest.approx(one["config"]["final_loss"], rel=1e-5)
