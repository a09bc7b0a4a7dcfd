"""The N>1 path of bench.py executed: 2 ranks as fresh processes on the one GPU of the box.

bench.py's distributed branch (init_process_group, barriers, the per-step StepGather of the packed
[L, obs_dim + 2] block to rank 0, the max-over-ranks timing all_reduce) runs under
torch.distributed.run with --dist-backend gloo --same-device: RCCL refuses two ranks on one
device, so the gather is staged through pinned host memory (dist.StepGather(host_stage=True));
everything else is the code an 8-GPU run executes.  Rank 0 dumps the gathered rows of every timed
step, and one process stepping a single 2L-lane batch with the same seed must produce the same
rows bit for bit (sharding changes nothing about any lane).

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
    got = np.load(dump)
    assert got.shape[:2] == (K, 2 * lanes)

    import torch
    assert torch.cuda.is_available()
    from gym_puzzles_amd import Batch
    b = Batch(env_id, 2 * lanes, seed=17)   # bench.py's default seed; lane_offset 0 covers both shards
    b.set_auto_reset(True)
    b.reset()
    for _ in range(W):
        b.step()
    for k in range(K):
        obs, rew, done, _ = b.step()
        exp = np.concatenate([obs, rew[:, None], done[:, None].astype(np.float32)], axis=1)
        bad = np.argwhere(got[k] != exp)
        assert bad.size == 0, f"step {k}: gathered rows differ from the one-batch run at {bad[:4].tolist()}"
    b.close()
