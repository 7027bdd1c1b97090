"""K3 latency micro-bench: exact get_path next hops on the 10k-agent warehouse map (510x220).

Runs the same query batches with the wave-cooperative heap (default), the lone-lane core
(TSW_ASTAR_SERIAL=1) and the lone-lane core without the second hand-off tier
(TSW_ASTAR_NO_TIER2=1: detours > 62 go straight to the global-heap k_astar), each in a child
process; checks all give identical answers and prints
per-batch wall times. Long queries (far start/goal pairs in open aisles) dominate the planner's
critical path, so batch 1 is a single far query (pure latency) and batch 2 is
256 far queries (the slowest one sets the time).
usage: python scripts/astar_bench.py [--out gpurun_out/astar_bench.json]
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402


def queries():
    """256 hard pairs: for 256 random goals, the start with the largest detour (BFS distance minus
    Manhattan distance, from the GPU's own K1 tables) — A* with the Manhattan heuristic pops
    every node with f < f*, so detours around shelf rows make the long queries."""
    from p2p_distributed_tswap_amd import Planner, maps
    rows = maps.warehouse_map(510, 220, 0x510220)
    W = len(rows[0])
    comp = np.array([x + y * W for x, y in maps.largest_component(rows)], dtype=np.int64)
    rng = np.random.default_rng(11)
    g = rng.choice(comp, 256)
    with Planner(rows) as p:
        D = p.dist_tables(g.astype(np.uint32)).astype(np.int64)
    s = np.empty_like(g)
    for i in range(g.size):
        d = D[i, comp]
        man = np.abs(comp % W - g[i] % W) + np.abs(comp // W - g[i] // W)
        s[i] = comp[np.argmax(np.where(d < 0xFFFF, d - man + d // 8, -1))]
    order = np.argsort(-(D[np.arange(g.size), s]))
    return rows, s[order].astype(np.uint32), g[order].astype(np.uint32)


def run_mode(out_npz):
    from p2p_distributed_tswap_amd import Planner
    rows, s, g = queries()
    res = {}
    with Planner(rows) as p:
        p.get_path_next(s[:8], g[:8])  # warm-up (scratch allocation, code load)
        for name, sl in (("one_far", slice(0, 1)), ("far256", slice(0, 256))):
            t0 = time.perf_counter()
            nxt, ln = p.get_path_next(s[sl], g[sl])
            res[name] = (time.perf_counter() - t0) * 1e3
            np.save(out_npz + f".{name}.npy", np.stack([nxt.astype(np.int64), ln.astype(np.int64)]))
    print(json.dumps(res))


def main():
    if "--child" in sys.argv:
        run_mode(sys.argv[sys.argv.index("--child") + 1])
        return
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    summary = {}
    for mode, env in (("wave_coop", {}), ("lone_lane", {"TSW_ASTAR_SERIAL": "1"}),
                      ("lone_lane_no_tier2", {"TSW_ASTAR_SERIAL": "1", "TSW_ASTAR_NO_TIER2": "1"})):
        base = os.path.join(ROOT, "gpurun_out", f"astar_{mode}")
        r = subprocess.run([sys.executable, __file__, "--child", base], env={**os.environ, **env},
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            sys.stderr.write(r.stderr)
            raise SystemExit(r.returncode)
        summary[mode] = json.loads(r.stdout.strip().splitlines()[-1])
    for name in ("one_far", "far256"):
        a = np.load(os.path.join(ROOT, "gpurun_out", f"astar_wave_coop.{name}.npy"))
        for other in ("lone_lane", "lone_lane_no_tier2"):
            b = np.load(os.path.join(ROOT, "gpurun_out", f"astar_{other}.{name}.npy"))
            summary[f"{name}_identical_{other}"] = bool(np.array_equal(a, b))
    for other in ("lone_lane", "lone_lane_no_tier2"):
        summary[f"speedup_far256_vs_{other}"] = summary[other]["far256"] / summary["wave_coop"]["far256"]
    line = json.dumps(summary)
    print(line)
    if out:
        with open(out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
