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


# ---- per-step K3 sharded by goal owner (as specified) -------------------------
# Rank 0 plans (tsw_plan_mapd_resolved: exit mode, the planner stops whenever a step needs next hops it
# does not have). Each stop's batch of (start, goal) pairs is broadcast; rank r answers the pairs whose
# goal it owns (goal % world == r) from its own table store (tsw_next_hop_codes: K1 for its new goals,
# the exact A* for unresolved cells, both kept for later stops), and one all-reduce(MIN) over the u8
# codes (non-owners contribute 0xFF) gathers the answers: <= 4n + 4096 bytes per stop. Every rank holds
# only its goals' tables and A* state. The planner's own step stays sequential on rank 0 (§8e row 3).

def goal_owner(goal: np.ndarray, world: int) -> np.ndarray:
    return (np.asarray(goal, dtype=np.int64) % world).astype(np.int64)


def _codes_for_rank(start: np.ndarray, goal: np.ndarray, rank: int, world: int,
                    codes_fn: Callable[[np.ndarray, np.ndarray], np.ndarray]) -> np.ndarray:
    """u8 codes of the pairs this rank owns, 0xFF elsewhere (the all-reduce MIN fills the rest)."""
    out = np.full(start.size, 0xFF, dtype=np.uint8)
    mine = np.flatnonzero(goal_owner(goal, world) == rank)
    if mine.size:
        out[mine] = codes_fn(np.ascontiguousarray(start[mine]), np.ascontiguousarray(goal[mine]))
    return out


class ShardedK3:
    """The collective half of the protocol. `codes_fn(start, goal) -> u8 codes` answers this rank's
    pairs (Planner.next_hop_codes on MI355X; the oracle in the CPU gloo tests)."""

    # a rank whose codes_fn failed contributes this to the all-reduce: it wins the MIN, so every rank
    # learns of the failure from the same collective and the protocol stays in step
    FAILED = -1

    def __init__(self, rank: int, world: int, dist, device, codes_fn):
        self.rank, self.world, self.dist, self.device, self.codes_fn = rank, world, dist, device, codes_fn
        self.stops = 0
        self.pairs = 0
        self.local_error = None   # this rank's codes_fn exception (first one)
        self.failed_stops = 0     # stops whose all-reduce carried FAILED

    def _bcast(self, arr: np.ndarray, dtype, n: int):
        import torch

        t = torch.zeros(n, dtype=dtype, device=self.device)
        if self.rank == 0:
            t.copy_(torch.from_numpy(arr))
        self.dist.broadcast(t, src=0)
        return t.cpu().numpy()

    def _exchange(self, start: np.ndarray, goal: np.ndarray) -> np.ndarray:
        import torch

        k = int(self._bcast(np.array([start.size if self.rank == 0 else 0], np.int64), torch.int64, 1)[0])
        if k < 0:
            return None
        pairs = np.concatenate([start, goal]).astype(np.int32) if self.rank == 0 else None
        pairs = self._bcast(pairs, torch.int32, 2 * k).astype(np.uint32)
        st, gl = pairs[:k], pairs[k:]
        if self.local_error is not None:
            # this rank already failed once (possibly a broken HIP context): do not re-enter codes_fn for
            # the rest of the plan, contribute FAILED until rank 0 sends finish()
            mine = np.full(k, self.FAILED, dtype=np.int32)
        else:
            try:
                mine = _codes_for_rank(st, gl, self.rank, self.world, self.codes_fn).astype(np.int32)
            except Exception as e:  # noqa: BLE001 — reported after the collective, on every rank
                self.local_error = e
                mine = np.full(k, self.FAILED, dtype=np.int32)
        # u8 codes ride in an int32 tensor (MIN over ranks: the owner's code, others 0xFF; FAILED wins)
        t = torch.from_numpy(mine).to(self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        self.stops += 1
        self.pairs += k
        return t.cpu().numpy()

    def _failure(self) -> RuntimeError:
        if self.local_error is not None:
            return RuntimeError(f"sharded K3: rank {self.rank}'s next-hop codes failed: {self.local_error}")
        return RuntimeError("sharded K3: another rank's next-hop codes failed")

    def resolve(self, start: np.ndarray, goal: np.ndarray) -> np.ndarray:
        """Rank 0's resolver (one planner stop). Raises (after the stop's collectives completed on every
        rank) when any rank failed to answer; the plan then fails and finish() releases the servers."""
        codes = self._exchange(start, goal)
        if np.any(codes == self.FAILED):
            self.failed_stops += 1
            raise self._failure()
        if np.any(codes > 4):
            raise RuntimeError("a next hop was answered by no rank")
        return codes.astype(np.uint8)

    def serve(self) -> None:
        """Ranks > 0: answer stops until rank 0's plan ends (finish()). A stop that failed anywhere does
        not end the loop — rank 0 still sends finish() — and is raised here afterwards."""
        while True:
            codes = self._exchange(np.zeros(0, np.uint32), np.zeros(0, np.uint32))
            if codes is None:
                break
            if np.any(codes == self.FAILED):
                self.failed_stops += 1
        if self.failed_stops:
            raise self._failure()

    def finish(self) -> None:
        """Rank 0: release the serving ranks."""
        import torch

        self._bcast(np.array([-1], np.int64), torch.int64, 1)


def plan_sharded_k3(rank: int, world: int, dist, device, codes_fn, plan_fn=None):
    """All ranks call this. Rank 0 runs plan_fn(resolver) (e.g. lambda r: planner.plan_mapd_resolved(
    starts, tasks, 2000, r, trace_goals=True)) and returns its result; other ranks serve until it ends.
    Returns (result or None, ShardedK3 with per-rank stop / pair counts)."""
    sk = ShardedK3(rank, world, dist, device, codes_fn)
    if rank == 0:
        try:
            res = plan_fn(sk.resolve)
        finally:
            sk.finish()
        return res, sk
    sk.serve()
    return None, sk
