"""CPU, world_size 2 over gloo: goal-sharded table build + all-gather reproduces every table.

The GPU builder (Planner.dist_tables_device) is replaced by the oracle BFS here — this test
covers the sharding / collective / ingestion-order logic that bench.py uses at N > 1.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from p2p_distributed_tswap_amd import maps, sharding


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    from oracle import OracleGraph

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = maps.random_map(20, 18, 0.2, 9)
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    free = np.flatnonzero(cells.reshape(-1) != ord("@")).astype(np.uint32)
    goals = free[::7]  # odd count on purpose (padding path)

    def build(g, out):
        out.copy_(torch.from_numpy(np.stack([og.bfs(int(x)) for x in g]).view(np.int16)))

    full = sharding.build_and_allgather(goals, cells.size, rank, world, build, dist, "cpu")
    ok = True
    for r, gl, off in sharding.gathered_blocks(goals, world):
        for j, gg in enumerate(gl):
            got = full[off + j].numpy().view(np.uint16)
            ok &= bool(np.array_equal(got, og.bfs(int(gg))))
    q.put((rank, ok, int(full.shape[0])))
    dist.destroy_process_group()


def _worker_codes(rank, world, port, q):
    """K1 + K3 shards (oracle BFS tables and oracle next-hop codes = get_path(cell, goal)[1] for
    every cell) all-gathered; every rank checks every gathered table and code table."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    from oracle import OracleGraph

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = maps.random_map(14, 11, 0.2, 4)
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    free = np.flatnonzero(cells.reshape(-1) != ord("@")).astype(np.uint32)
    goals = free[::5]

    def build(g, out_codes, out_tables):  # one builder for both (Planner.next_hop_tables_device + dist_ptr)
        out_codes.copy_(torch.from_numpy(np.stack([og.next_codes(int(x)) for x in g])))
        out_tables.copy_(torch.from_numpy(np.stack([og.bfs(int(x)) for x in g]).view(np.int16)))

    full_d, full_c = sharding.build_and_allgather_codes(goals, cells.size, rank, world, build, dist, "cpu")
    ok = True
    for r, gl, off in sharding.gathered_blocks(goals, world):
        for j, gg in enumerate(gl):
            ok &= bool(np.array_equal(full_d[off + j].numpy().view(np.uint16), og.bfs(int(gg))))
            ok &= bool(np.array_equal(full_c[off + j].numpy(), og.next_codes(int(gg))))
    q.put((rank, ok, int(full_c.shape[0])))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_codes_allgather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_codes, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_tables_allgather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res


def test_shard_partition():
    g = np.arange(17, dtype=np.uint32)
    parts = [sharding.goal_shard(g, r, 4) for r in range(4)]
    assert sorted(np.concatenate(parts).tolist()) == g.tolist()
    assert sharding.shard_rows(17, 4) == 5
