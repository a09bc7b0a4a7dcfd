"""The N>1 path of bench.py executed: 2 ranks as fresh processes on the one GPU of the box.

bench.py's distributed branch (init_process_group, barriers, the per-step StepGather of the packed
[L, obs_dim + 2] block to rank 0, the max-over-ranks timing all_reduce) runs under
torch.distributed.run with --dist-backend gloo --same-device: RCCL refuses two ranks on one
device, so the gather is staged through pinned host memory (dist.StepGather(host_stage=True));
everything else is the code an 8-GPU run executes.  Rank 0 dumps the gathered rows of every timed
step, and one process stepping a single 2L-lane batch with the same seed must produce the same
rows bit for bit (sharding changes nothing about any lane).

The RCCL branch itself (init_process_group("nccl"), dist.gather on device tensors) runs as one
rank under torch.distributed.run with --force-collective: StepGather then calls the collective at
world size 1 instead of short-circuiting, so a one-GPU box executes the code an 8-GPU node runs
over xGMI, and the gathered rows must equal the un-gathered batch bit for bit.

This file sorts before the other GPU test files on purpose: the ranks are started (fork + exec of
a fresh interpreter) before this pytest process has initialised the GPU.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _one_batch_rows(env_id, lanes, W, K):
    """(K, lanes, O + 2) rows [obs | reward | done] of one process stepping one batch (bench.py's seed)."""
    import torch
    assert torch.cuda.is_available()
    from gym_puzzles_amd import Batch
    b = Batch(env_id, lanes, seed=17)   # bench.py's default seed; lane_offset 0
    b.set_auto_reset(True)
    b.reset()
    for _ in range(W):
        b.step()
    rows = []
    for _ in range(K):
        obs, rew, done, _ = b.step()
        rows.append(np.concatenate([obs, rew[:, None], done[:, None].astype(np.float32)], axis=1))
    b.close()
    return np.stack(rows)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_rccl_gather_one_rank(tmp_path):
    """bench.py's distributed branch over RCCL on the box's one GPU: WORLD_SIZE 1 under
    torch.distributed.run, --dist-backend nccl --force-collective (dist.gather of the packed device
    block every step).  The JSON line names the RCCL collective, and the gathered rows equal one
    process's batch bit for bit."""
    W, K, lanes = 2, 6, 256
    dump = tmp_path / "gather.npy"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "1", "--dist-backend", "nccl",
           "--force-collective", "--env", "0", "--lanes", str(lanes), "--steps", str(K), "--warmup", str(W),
           "--no-cpu-baseline", "--dump-gather", str(dump)]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=ROOT, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["config"]["collective"] == "nccl (RCCL) forced at world size 1", line["config"]
    assert line["config"]["dump_gather"] and line["checks"]["ok"]
    got = np.load(dump)
    assert got.shape[:2] == (K, lanes)
    exp = _one_batch_rows(0, lanes, W, K)
    bad = np.argwhere(got != exp)
    assert bad.size == 0, f"gathered rows differ from the one-batch run at {bad[:4].tolist()}"


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("env_id,lanes", [(0, 256), (2, 128)])
def test_bench_two_ranks_gather_equals_one_batch(tmp_path, env_id, lanes):
    W, K = 2, 6
    dump = tmp_path / "gather.npy"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--same-device", "--env", str(env_id), "--lanes", str(lanes), "--steps", str(K), "--warmup", str(W),
           "--no-cpu-baseline", "--dump-gather", str(dump)]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=ROOT, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, "rank 0 (only) prints one JSON line"
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["global_lanes"] == 2 * lanes and line["steps"] == K
    assert line["config"]["collective"].startswith("gloo") and line["checks"]["ok"]
    assert line["value"] == pytest.approx(2 * lanes * K / (line["ms_per_step"] * K * 1e-3), rel=1e-6)
    assert line["config"]["dump_gather"]
    got = np.load(dump)
    assert got.shape[:2] == (K, 2 * lanes)
    exp = _one_batch_rows(env_id, 2 * lanes, W, K)   # lane_offset 0 covers both shards
    for k in range(K):
        bad = np.argwhere(got[k] != exp[k])
        assert bad.size == 0, f"step {k}: gathered rows differ from the one-batch run at {bad[:4].tolist()}"
