"""Planner-only time of a plan: the same C3 (or other) plan twice in one context, the second time with
every next-hop code the first one resolved still in the table store (no K3 waits), vs cold plans from
an empty store. cold - warm = what the A* latency chain costs the plan.

usage: python scripts/warm_plan.py [--config c3_warehouse_170x84] [--reps 3] [--no-chains]
(--no-chains: the diagnostic library with TSW_TASK_CHAINS=0 — no task-chain jobs, whose walks through
 the resolved store in the warm plan would otherwise count as planner traffic in scripts/warm_split.py)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from p2p_distributed_tswap_amd import Planner, build_id, maps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3_warehouse_170x84")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-chains", action="store_true")
    a = ap.parse_args()
    if a.no_chains:
        os.environ["TSW_TASK_CHAINS"] = "0"  # read at tsw_create by the diagnostic library
    rows, starts, tasks = maps.config_instance(a.config)
    out = {"config": a.config, "build_id": build_id(a.no_chains), "task_chains": not a.no_chains, "cold_ms": [], "warm_ms": [], "warm_waits": [], "cold_waits": [],
           "cold_queries": [], "warm_queries": []}
    with Planner(rows, diag=a.no_chains) as p:
        p.plan_mapd_arrays(starts, tasks, 50)
        for _ in range(a.reps):
            p.clear_tables()
            p.reset_stats()
            t0 = time.perf_counter()
            ref, _ = p.plan_mapd_arrays(starts, tasks, 2000)
            out["cold_ms"].append(round(1e3 * (time.perf_counter() - t0), 2))
            out["cold_waits"].append(p.stats()["coop_waits"])
            out["cold_queries"].append(p.stats()["astar_queries"])
            p.reset_stats()
            t0 = time.perf_counter()
            rec, _ = p.plan_mapd_arrays(starts, tasks, 2000)
            out["warm_ms"].append(round(1e3 * (time.perf_counter() - t0), 2))
            out["warm_waits"].append(p.stats()["coop_waits"])
            out["warm_queries"].append(p.stats()["astar_queries"])
            assert (rec == ref).all()
            out["agent_steps"] = int(rec.shape[0] * rec.shape[1])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
