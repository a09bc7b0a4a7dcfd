"""Multi-GPU layout of the batched step: one process per GPU, lanes sharded contiguously.

Worlds are independent, so the physics never exchanges data between GPUs.
Rank r owns global lanes [r*L, (r+1)*L) and passes ``lane_offset = r*L`` to ``mrp_create``;
the device RNG is keyed by the global lane id, so every lane's trajectory is identical at any
GPU count.  The only collective is the per-step hand-over of (obs, reward, done) to the
policy rank: each rank packs them into ONE contiguous float32 buffer [L, obs_dim + 2] (done as
0.0/1.0) and ``torch.distributed.gather``s it to rank 0 (RCCL turns this into root receives +
peer sends, one message per peer over its own xGMI link).  With a policy replica on every
rank use ``all_gather`` instead (``StepGather(..., to_all=True)``).
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    lanes_per_rank: int

    @property
    def lane_offset(self) -> int:
        return self.rank * self.lanes_per_rank

    @property
    def global_lanes(self) -> int:
        return self.world * self.lanes_per_rank

    def lanes(self) -> range:
        return range(self.lane_offset, self.lane_offset + self.lanes_per_rank)


def shard_from_env(lanes_per_rank: int) -> Shard:
    import os
    return Shard(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), lanes_per_rank)


class StepGather:
    """Packs one step's outputs of this rank and gathers every rank's block to rank 0."""

    def __init__(self, shard: Shard, obs_dim: int, device, group=None, to_all: bool = False, host_stage: bool = False,
                 force_collective: bool = False):
        """``host_stage``: the collective runs on host memory (a CPU backend such as gloo): the packed
        block is copied from the device into a pinned host buffer and gathered there; the receive
        buffer is on the host too.  ``force_collective``: call the collective at world size 1 too
        (a one-GPU box then executes the RCCL gather on device tensors; bench.py --force-collective)."""
        import torch
        self.shard, self.obs_dim, self.group, self.to_all = shard, obs_dim, group, to_all
        self.force_collective = force_collective
        L = shard.lanes_per_rank
        self.packed = torch.zeros((L, obs_dim + 2), dtype=torch.float32, device=device)
        self.host = torch.zeros((L, obs_dim + 2), dtype=torch.float32).pin_memory() if host_stage else None
        root = shard.rank == 0 or to_all
        # the receive blocks are row slices of ONE [G, obs_dim + 2] buffer: the gathered step is
        # contiguous on arrival, no concatenation afterwards
        rdev = "cpu" if host_stage else device
        self.full = torch.zeros((shard.global_lanes, obs_dim + 2), dtype=torch.float32, device=rdev) if root else None
        self.blocks = list(self.full.split(L, dim=0)) if root else None

    def pack(self, obs, reward, done):
        import torch
        # one fused copy into the packed rows [obs | reward | done]
        torch.cat((obs, reward.unsqueeze(1), done.unsqueeze(1).to(torch.float32)), dim=1, out=self.packed)
        return self.packed

    def __call__(self, obs, reward, done):
        """Returns (obs [G, O], reward [G], done [G]) over all G global lanes on rank 0 (every
        rank with to_all), None elsewhere.  Single-process: no collective.  The returned tensors
        are views of this gatherer's receive buffer, valid until its next call."""
        import torch.distributed as dist
        p = self.pack(obs, reward, done)
        if self.host is not None:
            self.host.copy_(p)   # synchronous device -> pinned host copy: the CPU collective reads it next
            p = self.host
        if self.shard.world == 1 and not self.force_collective:
            full = p
        else:
            if self.to_all:
                dist.all_gather(self.blocks, p, group=self.group)
            else:
                dist.gather(p, self.blocks if self.shard.rank == 0 else None, dst=0, group=self.group)
            if self.blocks is None:
                return None
            full = self.full
        O = self.obs_dim
        return full[:, :O], full[:, O], full[:, O + 1] != 0
