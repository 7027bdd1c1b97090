"""In-dispatch K3 cost: one full plan per instance, the coop workers' A* time, queries and heap pops by
queue (tsw_stats.coop_worker_*; product library) -> wall us per pop (and clocks at 2.4 GHz), us per query.
VERDICT r5 #2 asks for the pop cost of the workers inside the plan dispatch, beside scripts/astar_lat.py's
lone-query kernel.  usage: python scripts/pop_cost.py [c3 wh10k c5 c2]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from p2p_distributed_tswap_amd import Planner, maps  # noqa: E402

INST = {"c3": lambda: maps.config_instance("c3_warehouse_170x84"), "wh10k": maps.wh10k_instance,
        "c5": maps.c5_instance, "c2": lambda: maps.config_instance("c2_random_32_32_20")}
for name in sys.argv[1:] or ["c3"]:
    rows, starts, tasks = INST[name]()
    with Planner(rows) as p:
        p.plan_mapd_arrays(starts, tasks, 20)
        p.clear_tables()
        p.reset_stats()
        t0 = time.perf_counter()
        p.plan_mapd_arrays(starts, tasks, 2000)
        dt = time.perf_counter() - t0
        st = p.stats()
    out = {"instance": name, "plan_s": round(dt, 3), "workers": st["coop_workers"], "wait_ms": round(st["coop_wait_ms"], 1)}
    for k, q in enumerate(("needed", "speculative", "chains")):
        busy, nq, pops = st["coop_worker_busy_ms"][k], st["coop_worker_queries"][k], st["coop_worker_pops"][k]
        out[q] = {"queries": nq, "pops": pops, "busy_wave_ms": round(busy, 1),
                  "us_per_pop": round(1e3 * busy / pops, 3) if pops else None,
                  "clk_per_pop_2p4ghz": round(2.4e6 * busy / pops) if pops else None,
                  "us_per_query": round(1e3 * busy / nq, 1) if nq else None}
    print(json.dumps(out), flush=True)
