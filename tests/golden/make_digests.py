"""Per-timestep digests of full-horizon oracle plans too large to commit as raw fixtures.

For each instance: run the CPU oracle (oracle/tswap_oracle.c, the faithful restatement of
tswap.rs:39-394 — "parity unpinned" against the Rust binary) and record, for every
timestep t, the first 16 hex digits of sha1(records[:, t] || goals[:, t]) (records packed
x | y<<16 | state<<32 as u64, goals as u32 cell ids, agent order). The GPU test recomputes the same
digests from its own plan: equal digests at every t <=> bit-exact plans (up to sha1 collisions),
and the first differing t localises a divergence.

Instances (reference loop: tswap.rs:104-170, `timestep > 2000` stop):
  c3_full      BASELINE configs[2], warehouse 170x84, 1,000 agents, full horizon   -> digests.json
  c5_prefix    configs[4] sortation 1024x1024, 10,000 agents, 6 timesteps          -> digests.json
  wh10k_p300   north_star 10k-agent warehouse 510x220, 300 timesteps               -> digests_wh10k_p300.json
  wh10k_full   ... full horizon (2,001 timesteps, hours of oracle time)            -> digests_wh10k_full.json
  c5_p300      configs[4], 300 timesteps                                            -> digests_c5_p300.json
  c5_full      configs[4], full horizon                                             -> digests_c5_full.json
  den520d_10k  K1 tables of the bench's 10,000 den520d goals (configs[3]): per-table sha1[:8] of the
               oracle BFS u16 table (get_path length - 1, tswap.rs:288-390)        -> tables_den520d_10k.npz

The long instances each write their own file so several can be generated in parallel.

Usage: python tests/golden/make_digests.py [name ...]
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

from p2p_distributed_tswap_amd import maps  # noqa: E402


def step_digests(rec: np.ndarray, goals: np.ndarray) -> list:
    rec = np.ascontiguousarray(rec, dtype=np.uint64)
    goals = np.ascontiguousarray(goals, dtype=np.uint32)
    out = []
    for t in range(rec.shape[1]):
        h = hashlib.sha1(np.ascontiguousarray(rec[:, t]).tobytes())
        h.update(np.ascontiguousarray(goals[:, t]).tobytes())
        out.append(h.hexdigest()[:16])
    return out


def table_digests(tables: np.ndarray) -> np.ndarray:
    """First 8 bytes of sha1 of each u16 table (row-major, TSW_DIST_INF for blocked/unreachable), as u64."""
    t = np.ascontiguousarray(tables, dtype=np.uint16)
    return np.array([int.from_bytes(hashlib.sha1(t[k].tobytes()).digest()[:8], "little") for k in range(t.shape[0])],
                    dtype=np.uint64)


def den520d_goals(n: int = 10000) -> tuple:
    """The bench's K1 workload (bench.py `bfs`): den520d-like cave, n distinct sorted goals, seed 0x520D."""
    rows = maps.cave_map(256, 257, 0x520D)
    cells = maps.rows_to_array(rows).reshape(-1)
    free = np.flatnonzero(cells != ord("@")).astype(np.uint32)
    rng = np.random.default_rng(0x520D)
    goals = np.sort(rng.choice(free, size=min(n, free.size), replace=False)).astype(np.uint32)
    return rows, goals


# name -> (instance factory -> (rows, starts, tasks), max_t, output file)
def instances():
    return {
        "c3_full": (lambda: maps.config_instance("c3_warehouse_170x84"), 2000, "digests.json"),
        "c5_prefix": (maps.c5_instance, 6, "digests.json"),
        "wh10k_p300": (maps.wh10k_instance, 299, "digests_wh10k_p300.json"),
        "wh10k_full": (maps.wh10k_instance, 2000, "digests_wh10k_full.json"),
        "c5_p300": (maps.c5_instance, 299, "digests_c5_p300.json"),
        "c5_full": (maps.c5_instance, 2000, "digests_c5_full.json"),
    }


def load(name: str) -> dict:
    """The digest record of a MAPD instance (tests)."""
    _, _, fname = instances()[name]
    with open(os.path.join(HERE, fname)) as f:
        return json.load(f)[name]


def make_tables():
    from oracle import OracleGraph

    rows, goals = den520d_goals()
    og = OracleGraph(maps.rows_to_array(rows))
    t0 = time.time()
    dig = np.zeros(goals.size, dtype=np.uint64)
    for k, g in enumerate(goals):
        dig[k] = table_digests(og.bfs(int(g))[None])[0]
    np.savez_compressed(os.path.join(HERE, "tables_den520d_10k.npz"), goals=goals, sha1_8=dig)
    print(f"den520d_10k: {goals.size} tables in {time.time() - t0:.1f} s", flush=True)


def main(names=None):
    from oracle import OracleGraph

    if names and "den520d_10k" in names:
        make_tables()
        names = [n for n in names if n != "den520d_10k"]
        if not names:
            return
    for name, (fac, max_t, fname) in instances().items():
        if names and name not in names:
            continue
        if not names and name not in ("c3_full", "c5_prefix"):
            continue  # the long ones only on request
        rows, starts, tasks = fac()
        og = OracleGraph(maps.rows_to_array(rows))
        t0 = time.time()
        rec, goals = og.mapd(starts, tasks, max_t, trace_goals=True)
        dt = time.time() - t0
        path = os.path.join(HERE, fname)
        have = json.load(open(path)) if os.path.exists(path) else {}
        have[name] = {"agents": int(starts.shape[0]), "tasks": int(tasks.shape[0]), "max_t": max_t,
                      "T": int(rec.shape[1]), "oracle_s": round(dt, 1), "model": "std-heap-model v1",
                      "digests": step_digests(rec, goals)}
        print(f"{name}: T={rec.shape[1]} in {dt:.1f} s", flush=True)
        with open(path, "w") as f:
            json.dump(have, f, indent=0)


if __name__ == "__main__":
    main(sys.argv[1:] or None)
