"""Goal-sharded distance tables across GPUs.

K1 is independent per goal, so rank r of N builds goals r, r+N, r+2N, ... on its own GPU and
one all-gather (torch.distributed backend "nccl" = RCCL over xGMI) gives every rank every
table. The planning step itself stays on one GPU per replica (sequential agent order).

The table builder is a callback so the same collective code runs in the CPU gloo test
(oracle tables) and on MI355X (Planner.dist_tables_device into a torch tensor).
"""
from __future__ import annotations

from typing import Callable

import numpy as np


def goal_shard(goals: np.ndarray, rank: int, world: int) -> np.ndarray:
    """Round-robin shard: rank r owns goals[r::world]."""
    return np.ascontiguousarray(goals[rank::world])


def shard_rows(n_goals: int, world: int) -> int:
    """Rows per rank in the gathered tensor (ceil; short shards are zero-padded)."""
    return (n_goals + world - 1) // world


def gathered_blocks(goals: np.ndarray, world: int):
    """[(rank, goals of that rank, row offset in the gathered tensor)] for ingesting the gather."""
    per = shard_rows(goals.size, world)
    return [(r, goal_shard(goals, r, world), r * per) for r in range(world)]


def build_and_allgather(goals: np.ndarray, ncell: int, rank: int, world: int,
                        build: Callable[[np.ndarray, "torch.Tensor"], None], dist, device):
    """Build this rank's shard with `build(shard_goals, out_tensor[k, ncell] int16)` and
    all-gather. Returns the gathered int16 tensor [world*per, ncell] (rank-major blocks)."""
    import torch

    per = shard_rows(goals.size, world)
    mine = goal_shard(goals, rank, world)
    local = torch.zeros((per, ncell), dtype=torch.int16, device=device)
    if mine.size:
        build(mine, local[: mine.size])
    full = torch.empty((world * per, ncell), dtype=torch.int16, device=device)
    # u16 tables travel as bytes: neither RCCL/NCCL nor gloo has a 16-bit integer type
    dist.all_gather_into_tensor(full.view(torch.uint8), local.view(torch.uint8))
    return full
