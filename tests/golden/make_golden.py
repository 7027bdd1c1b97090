"""Generate the committed golden fixtures (tests/golden/*.npz, *.json).

Provenance: the reference is Rust and cannot be built or run in this image (no cargo/rustc),
and its own tests pin no planning result. Every vector here is produced
by the C oracle (oracle/tswap_oracle.c) AND independently by the pure-Python restatement
(oracle/py_restatement.py); the script refuses to write a fixture on which they disagree.
Tag: "std-heap-model v1" — Rust std BinaryHeap sift semantics restated by hand (unverified
against rustc here). Parity against these fixtures is therefore "parity unpinned" with
respect to the reference binary itself.

Run:  python tests/golden/make_golden.py   (takes ~1-2 min, CPU only)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from oracle import OracleGraph  # noqa: E402
import py_restatement as pr  # noqa: E402
from p2p_distributed_tswap_amd import maps  # noqa: E402

TAG = "std-heap-model v1"


def py_mapd(rows, starts, tasks, max_t=2000):
    goals = {}
    paths = pr.tswap_mapd(rows, [tuple(p) for p in starts.tolist()],
                          [((t[0], t[1]), (t[2], t[3])) for t in tasks.tolist()], max_t=max_t, trace_goals=goals)
    n = len(paths)
    T = len(paths[0]) if n else 0
    W = len(rows[0])
    rec = np.zeros((n, T), dtype=np.uint64)
    gl = np.zeros((n, T), dtype=np.uint32)
    for i in range(n):
        for t in range(T):
            (x, y), s = paths[i][t]
            rec[i, t] = x | (y << 16) | (int(s) << 32)
            gx, gy = goals[i][t]
            gl[i, t] = gy * W + gx
    return rec, gl


def mapd_case(name, rows, n, m, seed, max_t=2000):
    starts, tasks = maps.make_instance(rows, n, m, seed)
    og = OracleGraph(maps.rows_to_array(rows))
    rec, gl = og.mapd(starts, tasks, max_t, trace_goals=True)
    prec, pgl = py_mapd(rows, starts, tasks, max_t)
    assert rec.shape == prec.shape and np.array_equal(rec, prec) and np.array_equal(gl, pgl), name
    np.savez_compressed(os.path.join(HERE, f"mapd_{name}.npz"), grid=maps.rows_to_array(rows), starts=starts,
                        tasks=tasks, rec=rec, goals=gl, max_t=np.array(max_t), tag=np.array(TAG))
    print(f"mapd_{name}: n={n} m={m} T={rec.shape[1]}")


def astar_allpairs(name, rows):
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    G = pr.Graph(rows)
    W = cells.shape[1]
    free = np.flatnonzero(cells.reshape(-1) != ord("@")).astype(np.uint32)
    S, Gl = np.meshgrid(free, free, indexing="ij")
    S, Gl = S.reshape(-1), Gl.reshape(-1)
    nxt = np.zeros(S.size, dtype=np.uint32)
    ln = np.zeros(S.size, dtype=np.int32)
    for q in range(S.size):
        a, l, _ = og.get_path_next(int(S[q]), int(Gl[q]))
        p = G.get_path(G.pos2id[(int(S[q]) % W, int(S[q]) // W)], G.pos2id[(int(Gl[q]) % W, int(Gl[q]) // W)])
        px, py = G.id2pos[p[1] if len(p) > 1 else p[0]]
        assert (a, l) == (py * W + px, len(p)), (name, q)
        nxt[q], ln[q] = a, l
    np.savez_compressed(os.path.join(HERE, f"astar_{name}.npz"), grid=cells, start=S, goal=Gl, next=nxt, len=ln,
                        tag=np.array(TAG))
    print(f"astar_{name}: {S.size} pairs")


def bfs_case(name, rows, ngoals, seed):
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    G = pr.Graph(rows)
    W = cells.shape[1]
    free = np.flatnonzero(cells.reshape(-1) != ord("@")).astype(np.uint32)
    rng = np.random.default_rng(seed)
    goals = rng.choice(free, size=min(ngoals, free.size), replace=False).astype(np.uint32)
    tabs = np.stack([og.bfs(int(g)) for g in goals])
    # cross-check BFS against A* path lengths of the independent restatement on a sample
    for k, g in enumerate(goals[:8]):
        for c in free[:: max(1, free.size // 40)]:
            p = G.get_path(G.pos2id[(int(c) % W, int(c) // W)], G.pos2id[(int(g) % W, int(g) // W)])
            d = tabs[k, c]
            if d != 0xFFFF:
                assert len(p) - 1 == d, (name, g, c)
    np.savez_compressed(os.path.join(HERE, f"bfs_{name}.npz"), grid=cells, goals=goals, tables=tabs,
                        tag=np.array(TAG))
    print(f"bfs_{name}: {goals.size} goals")


def main():
    astar_allpairs("open8", maps.open_map(8, 8))
    astar_allpairs("rand10", maps.random_map(10, 10, 0.25, 5))
    bfs_case("rand32", maps.random_map(32, 32, 0.20, 0x3232), 64, 1)
    bfs_case("warehouse", maps.warehouse_map(170, 84, 0x170084), 8, 2)
    mapd_case("open8", maps.open_map(8, 8), 6, 12, 3)
    mapd_case("rand12", maps.random_map(12, 12, 0.2, 4), 10, 24, 4)
    mapd_case("rand16_dense", maps.random_map(16, 16, 0.2, 6), 40, 60, 6)
    mapd_case("c1_bundled_10", maps.bundled_map(), 10, 30, 1)  # BASELINE configs[0], library form
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump({"tag": TAG, "generator": "tests/golden/make_golden.py",
                   "oracles": ["oracle/tswap_oracle.c", "oracle/py_restatement.py"],
                   "parity": "unpinned vs the Rust binary (no toolchain); two restatements agree"}, f, indent=1)


if __name__ == "__main__":
    main()
