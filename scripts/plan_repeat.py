"""Repeated plans of one instance in ONE context (tables cleared between runs): separates one-time
context costs (table-store allocation, A* scratch) from the plan itself.
usage: python scripts/plan_repeat.py c5|c3|wh10k MAX_T [REPS]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from p2p_distributed_tswap_amd import Planner, maps  # noqa: E402

name, max_t = sys.argv[1], int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
fac = {"c5": maps.c5_instance, "wh10k": maps.wh10k_instance,
       "c3": lambda: maps.config_instance("c3_warehouse_170x84")}[name]
rows, starts, tasks = fac()
with Planner(rows) as p:
    for r in range(reps):
        p.clear_tables()
        p.reset_stats()
        t0 = time.perf_counter()
        rec, _ = p.plan_mapd_arrays(starts, tasks, max_t)
        dt = time.perf_counter() - t0
        st = p.stats()
        print(f"{name} max_t {max_t} rep {r}: {dt:.3f} s  T {rec.shape[1]}  bfs {st['bfs_ms']:.1f} ms  "
              f"sections {sum(st['plan_section_ms']):.1f} ms  waits {st['coop_wait_ms']:.1f} ms  "
              f"queries {st['astar_queries']}", flush=True)
