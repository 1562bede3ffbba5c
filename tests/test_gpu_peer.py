"""
The one-shot peer-write all-reduce (mininf_amd.peer, VERDICT r04 "Next round" 6), run by two
and three processes sharing the one GPU (the IPC handles exchanged over a gloo group, each rank
mapping the others' regions): the kernel's sums equal gloo's all_reduce of the same buckets (bit for
bit with two ranks: one addition), eagerly and replayed from a captured graph; a rank that never
calls makes every other rank's call fail loudly and bounded (NaN bucket, sticky error word,
PeerTimeout at the next host read, call counter kept); and bench.py's sharded C4 step
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


def _ranks(n, mode, port, timeout=240):
    return subprocess.run([sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1",
                           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
                           "--master-port", str(port),
                           os.path.join(ROOT, "tests", "peer_check.py"), mode],
                          env=_env(), capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("world,port", [(2, 29561), (3, 29563)])
def test_peer_all_reduce_matches_gloo(device, world, port):
    line = _last_json(_ranks(world, "sum", port))
    assert line["world"] == world
    for rank in line["ranks"]:
        assert rank["eager_equal"] and rank["graph_equal"], line
        assert rank["error_word"] == 0, line


@pytest.mark.parametrize("world,port", [(2, 29565), (3, 29567)])
def test_peer_all_reduce_missing_rank_fails_loudly(device, world, port):
    """The last rank never calls: the others time out within the bounded wait (seconds, not the
    test's limit), poison their buckets, raise PeerTimeout at the next host read (the StepGraph's
    check, the next eager call -- which enqueues nothing) and keep their call counters."""
    line = _last_json(_ranks(world, "missing", port, timeout=180))
    callers = line["ranks"][:-1]
    assert len(callers) == world - 1
    for rank in callers:
        assert rank["wait_s"] < 30, line
        assert rank["graph_nan"] and rank["graph_raised"], line
        assert rank["eager_raised"] and rank["eager_untouched"], line
        assert rank["sticky_nan"], line
        assert rank["counter"] == [0, 0], line
        assert rank["error_word"] == 1, line


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
