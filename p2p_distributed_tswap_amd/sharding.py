"""Goal-sharded table construction across GPUs.

Both per-goal kernels are independent per goal, so rank r of N takes goals r, r+N, r+2N, ...:
  * K1 (BFS distance tables, u16 per cell) — build_and_allgather;
  * K3 (exact next-hop codes, u8 per cell, every multi-candidate cell resolved by A*) —
    build_and_allgather_codes: the "query batches sharded by goal owner" row of §8e in its batched
    form; the gathered codes let a planner step with no K3 at all for those goals.
One all-gather per table kind (torch.distributed backend "nccl" = RCCL over xGMI) gives every rank
every table; Planner.import_tables_device / import_next_hops_device ingest them. The planning step
itself stays on one GPU per replica (sequential agent order).

The builders are callbacks so the same collective code runs in the CPU gloo tests (oracle tables
and codes) and on MI355X (Planner.dist_tables_device / next_hop_tables_device into torch tensors).
"""
from __future__ import annotations

from typing import Callable

import numpy as np


def goal_shard(goals: np.ndarray, rank: int, world: int) -> np.ndarray:
    """Round-robin shard: rank r owns goals[r::world]."""
    return np.ascontiguousarray(goals[rank::world])


def shard_rows(n_goals: int, world: int) -> int:
    """Rows per rank in the gathered tensor (ceil; short shards are padded)."""
    return (n_goals + world - 1) // world


def gathered_blocks(goals: np.ndarray, world: int):
    """[(rank, goals of that rank, row offset in the gathered tensor)] for ingesting the gather."""
    per = shard_rows(goals.size, world)
    return [(r, goal_shard(goals, r, world), r * per) for r in range(world)]


def _ready(local, device):
    """The zero/fill of `local` was queued on torch's current stream; the library writes it on its
    own stream, so the fill must be complete first (the C API also synchronises the device)."""
    import torch

    if str(device).startswith("cuda"):
        torch.cuda.current_stream(local.device).synchronize()


def build_and_allgather(goals: np.ndarray, ncell: int, rank: int, world: int,
                        build: Callable[[np.ndarray, "torch.Tensor"], None], dist, device):
    """Build this rank's K1 shard with `build(shard_goals, out_tensor[k, ncell] int16)` and
    all-gather. Returns the gathered int16 tensor [world*per, ncell] (rank-major blocks)."""
    import torch

    per = shard_rows(goals.size, world)
    mine = goal_shard(goals, rank, world)
    local = torch.zeros((per, ncell), dtype=torch.int16, device=device)
    _ready(local, device)
    if mine.size:
        build(mine, local[: mine.size])
    full = torch.empty((world * per, ncell), dtype=torch.int16, device=device)
    # u16 tables travel as bytes: neither RCCL/NCCL nor gloo has a 16-bit integer type
    dist.all_gather_into_tensor(full.view(torch.uint8), local.view(torch.uint8))
    return full


def build_and_allgather_codes(goals: np.ndarray, ncell: int, rank: int, world: int,
                              build: Callable[[np.ndarray, "torch.Tensor", "torch.Tensor"], None], dist, device):
    """K1 + K3 shards of this rank — `build(shard_goals, out_codes[k, ncell] uint8, out_tables[k, ncell]
    int16)` resolves every next hop of its goals and writes the K1 tables it used (one K1 build,
    Planner.next_hop_tables_device with dist_ptr) — then one all-gather of each. Returns (tables
    int16, codes uint8), both [world*per, ncell] in rank-major blocks (gathered_blocks gives the
    goal order)."""
    import torch

    per = shard_rows(goals.size, world)
    mine = goal_shard(goals, rank, world)
    local_d = torch.zeros((per, ncell), dtype=torch.int16, device=device)
    local_c = torch.full((per, ncell), 0xFF, dtype=torch.uint8, device=device)
    _ready(local_d, device)
    if mine.size:
        build(mine, local_c[: mine.size], local_d[: mine.size])
    full_d = torch.empty((world * per, ncell), dtype=torch.int16, device=device)
    full_c = torch.empty((world * per, ncell), dtype=torch.uint8, device=device)
    dist.all_gather_into_tensor(full_d.view(torch.uint8), local_d.view(torch.uint8))
    dist.all_gather_into_tensor(full_c, local_c)
    return full_d, full_c
