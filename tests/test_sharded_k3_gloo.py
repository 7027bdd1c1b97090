"""CPU, world_size 2 and 3 over gloo: per-step K3 sharded by goal owner.

Rank 0 plans with the reference's own loop (oracle/py_restatement.py: tswap.rs:39-286 restated)
whose every get_path(...)[1] is answered through sharding.ShardedK3 — each batch broadcast, the
pairs answered by the rank owning their goal (goal % world), the codes gathered by one
all-reduce(MIN) — and the plan must equal the C oracle's bit for bit. Ranks > 0 answer from the
oracle A* here (Planner.next_hop_codes on MI355X: tests/test_gpu_sharding.py).
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from p2p_distributed_tswap_amd import maps, sharding

W_STEP = {0: (0, 1), 1: (1, 0), 2: (0, -1), 3: (-1, 0)}  # S, E, N, W (tswap.rs:62)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_codes(og, w):
    def codes(start, goal):
        out = np.empty(start.size, dtype=np.uint8)
        for i, (s, g) in enumerate(zip(start.tolist(), goal.tolist())):
            nxt, _, _ = og.get_path_next(s, g)
            d = nxt - s
            out[i] = 4 if nxt == s else 0 if d == w else 1 if d == 1 else 2 if d == -w else 3
        return out
    return codes


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import py_restatement as pr
    from oracle import OracleGraph

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = maps.random_map(12, 11, 0.2, 4)
    cells = maps.rows_to_array(rows)
    h, w = cells.shape
    og = OracleGraph(cells)
    starts, tasks = maps.make_instance(rows, 6, 14, 4)

    def plan(resolve):
        base = pr.Graph

        class ShardedGraph(base):
            """get_path answered by the goal owners (only path[1] and len >= 2 are read, tswap.rs)."""

            def get_path(self, start, goal):
                if start == goal:
                    return [start]
                sx, sy = self.id2pos[start]
                gx, gy = self.id2pos[goal]
                code = int(resolve(np.array([sy * w + sx], np.uint32), np.array([gy * w + gx], np.uint32))[0])
                dx, dy = W_STEP.get(code, (0, 0))
                return [start, self.pos2id[(sx + dx, sy + dy)]]

        pr.Graph = ShardedGraph
        try:
            return pr.tswap_mapd(rows, [tuple(p) for p in starts.tolist()],
                                 [((a, b), (c, d)) for a, b, c, d in tasks.tolist()], max_t=150)
        finally:
            pr.Graph = base

    paths, sk = sharding.plan_sharded_k3(rank, world, dist, "cpu", _oracle_codes(og, w), plan)
    ok = True
    if rank == 0:
        ref, _ = og.mapd(starts, tasks, 150)
        got = np.array([[x | (y << 16) | (st << 32) for (x, y), st in p] for p in paths], dtype=np.uint64)
        ok = got.shape == ref.shape and bool(np.array_equal(got, ref))
    q.put((rank, ok, sk.stops, sk.pairs))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_k3_plan_matches_oracle(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _, _ in res), res
    stops = {s for _, _, s, _ in res}
    assert len(stops) == 1 and stops.pop() > 0  # every rank took part in every stop


def test_goal_owner_partition():
    g = np.arange(50, dtype=np.uint32)
    own = sharding.goal_owner(g, 4)
    assert set(own.tolist()) == {0, 1, 2, 3} and np.array_equal(own, g % 4)


def _failing_worker(rank, world, port, q, bad_rank):
    """Rank `bad_rank`'s codes_fn raises on the third stop it answers: every rank must leave the protocol
    with an error (no rank left blocked in a collective) — ADVICE r4."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = [0]

    def codes(start, goal):
        calls[0] += 1
        if rank == bad_rank and calls[0] >= 3:
            raise ValueError("injected failure")
        return np.full(start.size, 4, dtype=np.uint8)

    def plan(resolve):
        for _ in range(10):  # ten stops of 8 pairs; goals cover every owner
            resolve(np.arange(8, dtype=np.uint32), np.arange(8, dtype=np.uint32) + 100)
        return "done"

    outcome = "ok"
    try:
        sharding.plan_sharded_k3(rank, world, dist, "cpu", codes, plan)
    except RuntimeError as e:
        outcome = "injected" if "injected failure" in str(e) else "other-rank"
    q.put((rank, outcome))
    dist.destroy_process_group()


@pytest.mark.parametrize("bad_rank", [0, 1])
def test_sharded_k3_failing_rank_does_not_deadlock(bad_rank):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, world, port, q, bad_rank)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[bad_rank] == "injected"
    assert res[1 - bad_rank] == "other-rank"
