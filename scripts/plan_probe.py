"""Planner timeline probe: one C3 plan per horizon (max_t) from an empty table store, printing the
plan's wall time and the per-section device times / round counts, so the cost of a window of
timesteps is a difference of two lines. Environment TSW_* knobs apply (diagnostic library).

usage: python scripts/plan_probe.py [--diag] [--config c3_warehouse_170x84] [max_t ...]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from p2p_distributed_tswap_amd import Planner, maps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("horizons", nargs="*", type=int, default=[100, 300, 450, 1000, 2000])
    ap.add_argument("--config", default="c3_warehouse_170x84")
    ap.add_argument("--diag", action="store_true")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    rows, starts, tasks = maps.wh10k_instance() if a.config == "wh10k" else maps.config_instance(a.config)
    with Planner(rows, diag=a.diag) as p:
        p.plan_mapd_arrays(starts, tasks, 50)  # warm-up
        for T in a.horizons:
            best = None
            for _ in range(a.reps):
                p.clear_tables()
                p.reset_stats()
                t0 = time.perf_counter()
                rec, _ = p.plan_mapd_arrays(starts, tasks, T)
                dt = time.perf_counter() - t0
                st = p.stats()
                if best is None or dt < best[0]:
                    best = (dt, st, rec.shape[1])
            dt, st, nt = best
            print(json.dumps({
                "max_t": T, "T": nt, "ms": round(dt * 1e3, 2),
                "section_ms": [round(x, 2) for x in st["plan_section_ms"]],
                "wait_sec_ms": [round(x, 2) for x in st["coop_wait_sec_ms"]],
                "waits": st["coop_waits"], "rule_rounds": st["rule_rounds"], "move_rounds": st["move_rounds"],
                "relabels": [st["relabels_full"], st["relabels_inc"]], "queries": st["astar_queries"],
                "busy_wave_ms": [round(x, 1) for x in st["coop_worker_busy_ms"]],
                "env": {k: v for k, v in os.environ.items() if k.startswith("TSW_")},
            }), flush=True)


if __name__ == "__main__":
    main()
