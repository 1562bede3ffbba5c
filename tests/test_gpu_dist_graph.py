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
              "--warm-ms", "0", "--no-other-configs", "--no-cpu-baseline"]
    two = _last_json(_bench("--gpus", "2", "--dist-backend", "gloo", "--particles-per-gpu", "32",
                            *common))
    one = _last_json(_bench("--particles-per-gpu", "64", *common))
    assert two["n_gpus"] == 2 and two["config"]["global_particles"] == 64
    assert one["n_gpus"] == 1 and one["config"]["global_particles"] == 64
    assert "gloo all-reduce" in two["config"]["step_mode"]
    assert two["config"]["final_loss"] == pytest.approx(one["config"]["final_loss"], rel=1e-5)


def test_bench_two_gloo_ranks_match_one_rank_c5_data_sharded(device):
    """C5 data-sharded (DataShard: each rank all 1024 particles on half the elements, mu's
    gradients and the loss all-reduced) against one rank over all elements: the same final loss
    within 1e-5 after the same steps ("Next round" 2)."""
    common = ["--config", "c5", "--shard", "data", "--steps", "4", "--warmup", "2",
              "--graph-repeat", "1", "--warm-ms", "0", "--no-other-configs", "--no-cpu-baseline"]
    two = _last_json(_bench("--gpus", "2", "--dist-backend", "gloo", *common))
    one = _last_json(_bench(*common))
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["config"]["global_particles"] == one["config"]["global_particles"] == 1024
    assert "data-sharded x2" in two["config"]["parallelism"]
    assert two["scaling"] == "strong"
    assert two["config"]["final_loss"] == pytest.approx(one["config"]["final_loss"], rel=1e-5)


def test_bench_n2_default_run_measures_c4_and_c5(device):
    """`bench.py --gpus 2` (default C2 line) also measures C4 and C5 under other_configs, each
    entry carrying its rank count and layout."""
    line = _last_json(_bench("--gpus", "2", "--dist-backend", "gloo", "--steps", "4", "--warmup",
                             "2", "--graph-repeat", "1", "--warm-ms", "0", "--no-cpu-baseline"))
    assert line["n_gpus"] == 2 and line["config"]["ranks"] == 2
    others = line["other_configs"]
    assert sorted(others) == ["c4", "c5"]
    assert others["c4"]["config"]["ranks"] == 2 and others["c4"]["scaling"] == "weak"
    assert others["c4"]["config"]["global_particles"] == 64
    assert others["c5"]["config"]["ranks"] == 2 and others["c5"]["scaling"] == "strong"
    assert "data-sharded x2" in others["c5"]["config"]["parallelism"]
    for entry in others.values():
        assert entry["value"] > 0 and entry["ms_per_step"] > 0
