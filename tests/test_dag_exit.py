"""CPU check of the exact DAG early exit that the K3 workers' A* uses (tsw_astar.h, astar_wave_par<*, *, DAG>).

The claim (tsw_astar.h, above astar_wave_par): in get_path's A* (tswap.rs:288-390 — consistent Manhattan
heuristic, no closed set, keys (f, then smaller g)), once every node that is relaxed with g + D[n] == d*
(D = the goal's BFS distance, d* = D[start]) but not yet popped carries the same label (direction of its
path[1]), or the goal itself has been relaxed with g == d*, label(goal) is decided. Here the rule is run on
the restated Rust BinaryHeap (oracle/py_restatement.py) for many (start, goal) pairs and its answer is
compared with the oracle's full get_path (oracle/tswap_oracle.c); the fraction of pops saved is reported.
"""
import os
import sys

import numpy as np
import pytest

from p2p_distributed_tswap_amd import maps
from oracle import OracleGraph

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
from py_restatement import RustBinaryHeap, _Node  # noqa: E402

DIRS = ((0, 1), (1, 0), (0, -1), (-1, 0))  # S, E, N, W (tswap.rs:62)
INF = 0xFFFF


def astar_dag_exit(W, H, free, D, v, goal):
    """(direction of path[1], pops until decided, pops of the full search)."""
    gx, gy = goal % W, goal // W
    dstar = int(D[v])

    def h(c):
        return abs(c % W - gx) + abs(c // W - gy)

    heap = RustBinaryHeap()
    gs, lab, dag = {v: 0}, {}, set()
    cnt = [0, 0, 0, 0]
    heap.push(_Node(v, 0, h(v)))
    pops, decided = 0, None
    while True:
        cur = heap.pop()
        pops += 1
        c = cur.node_id
        if c == goal:
            assert decided is None or decided[0] == lab[c]
            return lab[c], (decided[1] if decided else pops), pops
        if c in dag and cur.g_cost == gs[c]:  # a DAG entry is never stale
            cnt[lab[c]] -= 1
            dag.discard(c)
        cx, cy = c % W, c // W
        for d, (dx, dy) in enumerate(DIRS):
            nx, ny = cx + dx, cy + dy
            if not (0 <= nx < W and 0 <= ny < H and free[ny * W + nx]):
                continue
            n = ny * W + nx
            tg = cur.g_cost + 1
            if tg < gs.get(n, 1 << 30):
                assert n not in dag  # an optimal relaxation is never improved
                gs[n] = tg
                lab[n] = d if c == v else lab[c]
                if tg + int(D[n]) == dstar:
                    dag.add(n)
                    cnt[lab[n]] += 1
                heap.push(_Node(n, tg, tg + h(n)))
        if decided is None:
            if goal in gs and gs[goal] == dstar:
                decided = (lab[goal], pops)
            elif sum(1 for k in cnt if k) == 1:
                decided = (next(k for k in range(4) if cnt[k]), pops)


def _pairs(rows, npairs, seed):
    arr = maps.rows_to_array(rows)
    H, W = arr.shape
    free = arr.reshape(-1) != ord("@")
    og = OracleGraph(arr)
    rng = np.random.default_rng(seed)
    cells = np.flatnonzero(free)
    out = []
    for g in rng.choice(cells, max(1, npairs // 20), replace=False):
        D = og.bfs(int(g)).reshape(-1)
        for v in rng.choice(cells, 20, replace=False):
            if v == g or D[v] == INF:
                continue
            out.append((W, H, free, D, og, int(v), int(g)))
    return out


@pytest.mark.parametrize("name,rows", [
    ("open16", maps.open_map(16, 16)),
    ("rand24", maps.random_map(24, 24, 0.2, 7)),
    ("warehouse", maps.warehouse_map(60, 30, 5)),
])
def test_dag_exit_matches_full_astar(name, rows):
    saved = total = 0
    for (W, H, free, D, og, v, g) in _pairs(rows, 200, 0xDA6):
        lab, p_exit, p_full = astar_dag_exit(W, H, free, D, v, g)
        nxt = og.get_path_next(v, g)[0]
        dx, dy = DIRS[lab]
        assert nxt == (v // W + dy) * W + v % W + dx, (name, v, g)
        saved += p_full - p_exit
        total += p_full
    assert total > 0
    print(f"{name}: DAG early exit saves {saved / total:.1%} of {total} pops")


def detour_bytes(D, W, goal, cap=255):
    """The table store's detour bytes (round 6, tsw_internal.h): min((D - |c - goal|_1) / 2, cap), cap for
    unreachable cells. `cap` below 255 makes saturation common on small maps."""
    gx, gy = goal % W, goal // W
    c = np.arange(D.size)
    man = np.abs(c % W - gx) + np.abs(c // W - gy)
    det = (D.astype(np.int64) - man) // 2
    return np.where(D == INF, cap, np.minimum(det, cap)).astype(np.int64)


def astar_dag_exit_bytes(W, H, free, D, v, goal, cap):
    """astar_dag_exit with the workers' byte test: d* = h(v) + 2 b(v) (no early exit when b(v) == cap) and
    a node is a DAG node iff b(n) != cap and g + h(n) + 2 b(n) == d* (tsw_astar.h)."""
    b = detour_bytes(D, W, goal, cap)
    gx, gy = goal % W, goal // W
    h = lambda c: abs(c % W - gx) + abs(c // W - gy)  # noqa: E731
    if b[v] == cap:
        return None
    Dx = np.where(b == cap, INF, np.array([h(c) for c in range(D.size)]) + 2 * b)  # INF never matches
    assert Dx[v] == D[v]
    return astar_dag_exit(W, H, free, Dx, v, goal)


@pytest.mark.parametrize("cap", [2, 6, 255])
def test_dag_exit_with_saturated_detour_bytes(cap):
    """The byte form of the test is exact even when bytes saturate: along a shortest path toward the goal D
    drops by 1 per hop and the Manhattan distance by at most 1, so the detour never grows, and every DAG node
    of a query has detour <= detour(start) < cap — skipping saturated cells skips no DAG node."""
    rows = maps.cave_map(40, 41, 3)
    checked = 0
    for (W, H, free, D, og, v, g) in _pairs(rows, 300, 0xB17E):
        r = astar_dag_exit_bytes(W, H, free, D, v, g, cap)
        if r is None:
            continue
        lab, _, _ = r
        dx, dy = DIRS[lab]
        assert og.get_path_next(v, g)[0] == (v // W + dy) * W + v % W + dx, (cap, v, g)
        checked += 1
    assert checked > 0


def test_detour_never_grows_along_shortest_paths():
    rows = maps.cave_map(40, 41, 3)
    arr = maps.rows_to_array(rows)
    H, W = arr.shape
    free = arr.reshape(-1) != ord("@")
    og = OracleGraph(arr)
    rng = np.random.default_rng(0xDE70)
    for g in rng.choice(np.flatnonzero(free), 12, replace=False):
        D = og.bfs(int(g)).reshape(-1).astype(np.int64)
        det = detour_bytes(D, W, int(g), cap=1 << 30)
        for c in np.flatnonzero((D != INF) & free):
            cx, cy = c % W, c // W
            for dx, dy in DIRS:
                nx, ny = cx + dx, cy + dy
                if 0 <= nx < W and 0 <= ny < H and free[ny * W + nx] and D[ny * W + nx] == D[c] - 1:
                    assert det[ny * W + nx] <= det[c]
