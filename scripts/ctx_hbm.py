"""Per-context HBM: device memory a planner context holds after one full-horizon plan of each config
(free device memory before the context is created minus free memory after the plan, the context still
open), split into the table store (u8 detour bytes + u8 next-hop codes per goal table since round 6; u16
distances + codes before, from the context's stats)
and everything else (K3 scratch slots, coop queues, records, agent/task state, K1 scratch).

usage: python scripts/ctx_hbm.py [config ...]   (default: the three BASELINE planning configs)
"""
import argparse
import gc
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from p2p_distributed_tswap_amd import Planner, maps  # noqa: E402

GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c3_warehouse_170x84", "wh10k", "c5_sortation_1024_10k"])
    ap.add_argument("--max-t", type=int, default=2000)
    a = ap.parse_args()
    torch.cuda.init()
    for name in a.configs:
        rows, starts, tasks = maps.wh10k_instance() if name == "wh10k" else maps.config_instance(name)
        gc.collect()
        free0, total = torch.cuda.mem_get_info()
        with Planner(rows) as p:
            rec, _ = p.plan_mapd_arrays(starts, tasks, a.max_t)
            free1, _ = torch.cuda.mem_get_info()
            st = p.stats()
            tables = int(st["tables"])
            ncell = len(rows) * len(rows[0])
            store = tables * ncell * 2  # u8 detour bytes + u8 codes per goal table (round 6)
            print(json.dumps({
                "config": name, "agents": len(starts), "tasks": len(tasks), "cells": ncell,
                "timesteps": int(rec.shape[1]), "tables": tables,
                "context_gib": round((free0 - free1) / GIB, 3),
                "table_store_gib": round(store / GIB, 3),
                "other_gib": round((free0 - free1 - store) / GIB, 3),
                "coop_workers": st.get("coop_workers"),
                "device_total_gib": round(total / GIB, 1),
            }), flush=True)
        gc.collect()


if __name__ == "__main__":
    main()
