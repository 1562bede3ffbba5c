"""
The one-shot peer-write all-reduce (mininf_amd.peer, VERDICT r04 "Next round" 6), run by two
processes sharing the one GPU (the IPC handles exchanged over a gloo group, each rank mapping the
other's region): the kernel's sums equal gloo's all_reduce of the same buckets bit for bit (two
ranks: one addition), eagerly and replayed from a captured graph; and bench.py's sharded C4 step
with the peer all-reduce captured in its graph ends on the same loss as the step split around
gloo's all-reduce. Unmeasured on multi-GPU hardware. Each check runs in child processes with
their own time limits.
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


def test_peer_all_reduce_matches_gloo(device):
    out = subprocess.run([sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                          "--master-port", "29561",
                          os.path.join(ROOT, "tests", "peer_check.py")],
                         env=_env(), capture_output=True, text=True, timeout=240)
    line = _last_json(out)
    assert line["eager_equal"] and line["graph_equal"], line
    assert line["error_word"] == 0, line


def _bench(*argv):
    return subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), *argv],
                          env=_env(), capture_output=True, text=True, timeout=280)


def test_bench_peer_all_reduce_matches_gloo(device):
    common = ["--gpus", "2", "--dist-backend", "gloo", "--config", "c4", "--steps", "4",
              "--warmup", "2", "--graph-repeat", "1", "--warm-ms", "0", "--no-other-configs",
              "--no-cpu-baseline", "--particles-per-gpu", "32"]
    peer = _last_json(_bench("--allreduce", "peer", *common))
    gloo = _last_json(_bench(*common))
    assert "peer-write all-reduce captured" in peer["config"]["step_mode"]
    assert "gloo all-reduce" in gloo["config"]["step_mode"]
    assert peer["config"]["final_loss"] == gloo["config"]["final_loss"]
