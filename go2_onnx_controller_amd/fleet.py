"""Many-robot mode: shard a fleet of robots over the GPUs of one node.

SURVEY §8(e): every robot row is independent (a recurrent robot's hidden row
travels with it), so the batch is partitioned into contiguous row blocks, one
per rank (one process per GPU), weights replicated per GPU. The steady-state
step has NO collective. The only optional exchange is gathering the actions of
all shards to one rank when a consolidated tensor is requested
(torch.distributed all_gather: RCCL over xGMI with the "nccl" backend,
gloo on CPU).
"""
from __future__ import annotations


def shard_range(batch: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [start, stop) rows of `batch` owned by `rank` (sizes differ by <= 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    if batch < 0:
        raise ValueError("negative batch")
    base, rem = divmod(batch, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def shard_sizes(batch: int, world: int) -> list[int]:
    return [b - a for a, b in (shard_range(batch, r, world) for r in range(world))]


def gather_actions(local, batch: int, group=None):
    """All-gather per-rank action shards [rows_r, A] into the full [batch, A] tensor on
    every rank (ragged shards padded to the largest shard for the collective)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    sizes = shard_sizes(batch, world)
    width = local.shape[1]
    mx = max(sizes)
    pad = local.new_zeros((mx, width))
    pad[: local.shape[0]] = local
    bufs = [local.new_empty((mx, width)) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)], dim=0)


class FleetShard:
    """The rank-local slice of a fleet: rows [start, stop) of a global batch."""

    def __init__(self, engine, batch: int, rank: int, world: int):
        self.engine = engine
        self.batch = batch
        self.rank, self.world = rank, world
        self.start, self.stop = shard_range(batch, rank, world)

    @property
    def rows(self) -> int:
        return self.stop - self.start

    def step(self, obs_local, out=None, stream=None):
        """One control tick for this shard's robots (device tensors, no collective)."""
        return self.engine.run_torch(obs_local, out=out, stream=stream)
