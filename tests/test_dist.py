"""world_size-2 gloo tests of the multi-GPU layout (gym_puzzles_amd/dist.py) on CPU.

Each rank steps its contiguous shard of lanes (the CPU oracle stands in for the GPU step, with
the same counter-RNG inputs the device uses), packs (obs, reward, done), gathers to rank 0,
and rank 0 checks the result against one process stepping all lanes: sharding changes
nothing about any lane.
"""
from __future__ import annotations

import os
import socket
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


def _worker(rank, world, port, lanes_per_rank, steps, to_all, q, force=False):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from gym_puzzles_amd.dist import Shard, StepGather
    from gym_puzzles_amd.spawn import draw_bounds
    from oracle.oracle import batch_run
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = Shard(rank, world, lanes_per_rank)
        _, _, bodies, rsum, eps = batch_run(0, sh.lanes_per_rank, steps, 17, draw_bounds(0), threads=1,
                                            lane_offset=sh.lane_offset, outputs=True)
        g = StepGather(sh, obs_dim=bodies.shape[1], device="cpu", to_all=to_all, force_collective=force)
        if force:   # the collective must run at world size 1: count the calls that reach torch.distributed
            calls = []
            real = dist.all_gather if to_all else dist.gather
            def spy(*a, **k):
                calls.append(1)
                return real(*a, **k)
            setattr(dist, "all_gather" if to_all else "gather", spy)
        out = g(torch.from_numpy(bodies), torch.from_numpy(rsum.astype(np.float32)),
                torch.from_numpy((eps > 1).astype(np.uint8)))
        if force:
            assert calls == [1], "StepGather(force_collective=True) must call the collective at world size 1"
        if out is not None:
            q.put((rank, out[0].numpy().copy(), out[1].numpy().copy(), out[2].numpy().copy()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("to_all", [False, True])
def test_two_rank_gather_equals_single_process(oracle_lib, to_all):
    import torch.multiprocessing as mp

    from gym_puzzles_amd.spawn import draw_bounds
    from oracle.oracle import batch_run
    world, L, steps = 2, 6, 80
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, L, steps, to_all, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world if to_all else 1)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, _, bodies, rsum, eps = batch_run(0, world * L, steps, 17, draw_bounds(0), threads=2, outputs=True)
    for rank, ob, rw, dn in results:
        assert rank == 0 or to_all
        assert np.array_equal(ob, bodies)
        assert np.array_equal(rw, rsum.astype(np.float32))
        assert np.array_equal(dn, eps > 1)


@pytest.mark.parametrize("to_all", [False, True])
def test_forced_collective_world_one(oracle_lib, to_all):
    """bench.py --force-collective at world size 1 (the one-GPU RCCL rehearsal) on gloo: the gather
    runs through torch.distributed and returns the rank's own rows unchanged."""
    import torch.multiprocessing as mp

    from gym_puzzles_amd.spawn import draw_bounds
    from oracle.oracle import batch_run
    L, steps = 6, 40
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), L, steps, to_all, q, True))
    p.start()
    rank, ob, rw, dn = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0 and rank == 0
    _, _, bodies, rsum, eps = batch_run(0, L, steps, 17, draw_bounds(0), threads=1, outputs=True)
    assert np.array_equal(ob, bodies) and np.array_equal(rw, rsum.astype(np.float32)) and np.array_equal(dn, eps > 1)


def test_shard_arithmetic():
    from gym_puzzles_amd.dist import Shard
    s = Shard(3, 8, 1024)
    assert s.lane_offset == 3072 and s.global_lanes == 8192 and list(s.lanes())[:2] == [3072, 3073]
