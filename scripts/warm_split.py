"""Planner / K3-worker split of the coop plan dispatch's HBM traffic.

The coop `k_plan` dispatch runs the planner (workgroup 0) and the K3 workers together, so its PMC
bytes are one number. scripts/warm_plan.py plans the same C3 instance twice in one context: the
cold plan (empty table store: the workers resolve every next hop the plan needs) and the warm plan
(every code already in the store: the workers only idle-poll). Profiled with one PMC pass per
counter, the warm dispatch's bytes are the planner's (plus idle polling), and cold - warm is what the
workers' A* moved. Exit-mode profiles cannot give this split: every exit relaunch re-stages the
planner's state, so the exit-mode planner moves more bytes than the whole fused dispatch.

usage: python scripts/warm_split.py FETCH_DIR WRITE_DIR WARM_JSON OUT_JSON [NC_FETCH_DIR NC_WRITE_DIR NC_JSON]
(the optional NC_* passes are `warm_plan.py --reps 1 --no-chains`: without task chains the warm dispatch
 holds no chain walks through the resolved store, so its bytes are the planner's alone — reported as
 planner_bytes_per_agent_step when given; the default run's warm figure stays as warm_dispatch_bytes)
(FETCH_DIR / WRITE_DIR: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE -d outputs of
 `python3 scripts/warm_plan.py --reps 1`; gfx950 correction as in summarize_profile.py:
 read bytes = 2 x FETCH_SIZE KB, write bytes = WRITE_SIZE KB)
"""
import csv
import glob
import json
import os
import sys


def plan_dispatches(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "k_plan" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                    rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"]),
                                 int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    return rows


def same_sources(product_id, diag_id) -> bool:
    """The no-chains pass runs the diagnostic library, whose build id hashes the flavour too:
    accept the pair when both ids are this tree's product / diagnostic hashes."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from __graft_entry__ import source_hash

    return str(product_id) == source_hash("") and str(diag_id) == source_hash("diag")


def main():
    fdir, wdir, warm_json, out_path = sys.argv[1:5]
    nc = sys.argv[5:8] if len(sys.argv) >= 8 else None
    fe, wr = plan_dispatches(fdir, "FETCH_SIZE"), plan_dispatches(wdir, "WRITE_SIZE")
    # dispatch order of warm_plan.py --reps 1: warm-up plan (50 steps), cold plan, warm plan
    if len(fe) != 3 or len(wr) != 3:
        raise SystemExit(f"expected 3 k_plan dispatches per pass, got {len(fe)} / {len(wr)}")
    with open(warm_json) as fh:
        wj = json.loads([l for l in fh if l.startswith("{")][-1])

    def bytes_of(i):
        return 2.0 * fe[i][1] * 1024.0 + wr[i][1] * 1024.0

    cold, warm = bytes_of(1), bytes_of(2)
    q = wj["cold_queries"][0]
    agent_steps = wj.get("agent_steps", 1000 * 2001)  # agents x recorded timesteps of the plan
    planner = warm
    planner_src = "warm plan dispatch (task chains on: includes the workers' walks through the resolved store)"
    if nc:
        fe2, wr2 = plan_dispatches(nc[0], "FETCH_SIZE"), plan_dispatches(nc[1], "WRITE_SIZE")
        if len(fe2) != 3 or len(wr2) != 3:
            raise SystemExit(f"no-chains: expected 3 k_plan dispatches per pass, got {len(fe2)} / {len(wr2)}")
        with open(nc[2]) as fh:
            wj2 = json.loads([l for l in fh if l.startswith("{")][-1])
        if wj2.get("build_id") != wj.get("build_id") and not same_sources(wj.get("build_id"), wj2.get("build_id")):
            raise SystemExit("no-chains profile of another build")
        planner = 2.0 * fe2[2][1] * 1024.0 + wr2[2][1] * 1024.0
        planner_src = "warm plan dispatch without task chains (diagnostic library, TSW_TASK_CHAINS=0)"
    out = {
        "config": wj["config"],
        "build_id": wj.get("build_id"),
        "method": "PMC FETCH_SIZE / WRITE_SIZE of the cold and the warm coop plan dispatch (scripts/warm_plan.py)",
        "cold_dispatch_bytes": round(cold),
        "warm_dispatch_bytes": round(warm),
        "cold_dispatch_ms": round(fe[1][2] / 1e6, 2),
        "warm_dispatch_ms": round(fe[2][2] / 1e6, 2),
        "planner_bytes_per_agent_step": round(planner / agent_steps, 1),
        "planner_bytes_source": planner_src,
        "warm_dispatch_bytes_per_agent_step": round(warm / agent_steps, 1),
        "planner_algorithmic_bytes_per_agent_step": 46.0,
        "workers_bytes": round(cold - warm),
        "worker_queries": q,
        "workers_bytes_per_query": round((cold - warm) / max(q, 1), 1),
        "warm_plan_json": wj,
    }
    with open(out_path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "warm_plan_json"}))


if __name__ == "__main__":
    main()
