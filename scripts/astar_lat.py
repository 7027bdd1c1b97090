"""K3 single-query LATENCY on the C3 warehouse (170x84): the planner's needed queries are
get_path(cell, pickup) one at a time, so one query's A* time is what a step waits for.

Queries: 96 (start, goal) pairs at Manhattan distance 40-120 (assignment-like), plus the 96
hardest detours. Each query runs alone (one k_astar_wave wave) and its device time is the K3
HIP-event time (tsw_get_stats astar_ms); printed: median / p90 per query in us, and the pops per
query from the oracle (so us per pop). Environment TSW_* knobs apply (diagnostic library), e.g.
TSW_ASTAR_OLDPOP=1 for the windowed pop. Answers are checked against the oracle.

usage: python scripts/astar_lat.py [--diag] [--label NAME]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

from p2p_distributed_tswap_amd import Planner, maps  # noqa: E402


def pairs(rows, n=96, seed=5):
    W = len(rows[0])
    comp = np.array([x + y * W for x, y in maps.largest_component(rows)], dtype=np.int64)
    rng = np.random.default_rng(seed)
    s, g = [], []
    while len(s) < n:
        a, b = rng.choice(comp, 2)
        man = abs(a % W - b % W) + abs(a // W - b // W)
        if 40 <= man <= 120:
            s.append(a)
            g.append(b)
    return np.array(s, dtype=np.uint32), np.array(g, dtype=np.uint32)


def main():
    from oracle import OracleGraph

    diag = "--diag" in sys.argv
    label = sys.argv[sys.argv.index("--label") + 1] if "--label" in sys.argv else ("diag" if diag else "default")
    rows = maps.warehouse_map(170, 84, 0x170084)
    og = OracleGraph(maps.rows_to_array(rows))
    s, g = pairs(rows)
    us, pops, bad = [], [], 0
    with Planner(rows, diag=diag) as p:
        p.get_path_next(s[:4], g[:4])  # warm-up
        for q in range(s.size):
            p.reset_stats()
            nxt, ln = p.get_path_next(s[q:q + 1], g[q:q + 1])
            st = p.stats()
            us.append(st["astar_ms"] * 1e3)
            rn, rl, pp = og.get_path_next(int(s[q]), int(g[q]))
            pops.append(pp)
            bad += int((int(nxt[0]), int(ln[0])) != (rn, rl))
        # a batch of all 96 at once: throughput of the worker-like one-query-per-wave kernel
        p.reset_stats()
        p.get_path_next(s, g)
        batch_ms = p.stats()["astar_ms"]
    us, pops = np.array(us), np.array(pops, dtype=np.float64)
    print(json.dumps({"label": label, "queries": int(s.size), "mismatches": bad,
                      "median_us": round(float(np.median(us)), 1), "p90_us": round(float(np.percentile(us, 90)), 1),
                      "median_pops": float(np.median(pops)), "us_per_pop": round(float(np.sum(us) / np.sum(pops)), 4),
                      "batch96_ms": round(batch_ms, 3),
                      "env": {k: v for k, v in os.environ.items() if k.startswith("TSW_")}}), flush=True)


if __name__ == "__main__":
    main()
