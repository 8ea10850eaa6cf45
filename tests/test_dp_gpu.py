"""Data-parallel training iteration on the GPU: 2 ranks (gloo, both pinned to
cuda:0 so it runs on a 1-GPU box) through bench.py's DP path -- HIP-graph
segments with the gradient all-reduces between them.  The replicas' weights
must stay bit-identical."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_training_keeps_replicas_in_sync():
    env = dict(os.environ, EXO_BENCH_DEVICE="0", EXO_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "12", "--warmup", "6", "--envs", "256", "--no-cpu-baseline",
           "--kernel-timing-steps", "5"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=REPO)
    assert out.returncode == 0, out.stderr[-4000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2
    assert res["dp_weights_in_sync"] is True
    assert res["value"] > 0


def test_rccl_data_parallel_layout_at_world_one():
    """The RCCL branch the multi-GPU runs take, on a one-GPU box: torchrun with
    one rank and EXO_FORCE_DIST=1 -- bench.py initialises the nccl (RCCL)
    process group, the agent's GradSync is active at world 1, so VecTrainer
    replays the three-graph data-parallel layout with the flat-bucket
    all-reduces, the max_priority MAX reduction and the replica checksum
    all_gather on RCCL between the graphs (RCCL refuses two ranks on one
    device, so world 1 is the most of that path one GPU can run)."""
    env = dict(os.environ, EXO_FORCE_DIST="1")
    env.pop("EXO_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "bench.py"),
           "--steps", "20", "--warmup", "8", "--envs", "512", "--no-cpu-baseline", "--no-td7-variants",
           "--no-reference-schedule", "--kernel-timing-steps", "5"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=REPO)
    assert out.returncode == 0, out.stderr[-4000:]
    res = json.loads([l for l in out.stdout.splitlines() if l.startswith('{"metric')][-1])
    assert res["n_gpus"] == 1
    assert "DP all-reduce" in res["config"]["parallelism"]
    assert res["dp_weights_in_sync"] is True
    assert res["weights_finite"] is True, res["weights_finite"]
    assert res["value"] > 0
