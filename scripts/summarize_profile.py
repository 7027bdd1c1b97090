"""Summarise a scripts/profile_round.sh output directory into profiles/<tag>/.

Per workload (plan = the bench's planning leg, bfs = K1 alone on den520d, 10,000 goals; each
profiled in its own process so launches of different sizes never mix):
  * copies the rocprofv3 --kernel-trace --stats summary  -> profiles/<tag>/<wl>_kernel_stats.csv
  * per kernel CLASS (K1 = k_bfs*/k_classify, K3 = k_astar*/k_enqueue_unknown, k_plan):
      device ns per launch from the kernel trace, HBM bytes per launch from the separate PMC
      passes, and the algorithmic bytes per launch the bench reports for that class.
Launch = what bench.py counts for the class (HIP-event brackets: one K3 pass may dispatch up to
three A* kernels; K1 in the bfs workload = one k_bfs_blk dispatch).
Traffic correction (/opt/skills/guides/MI355X_MICROARCH.md, "HBM"): FETCH_SIZE and WRITE_SIZE are
in KB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so
read bytes = 2 * FETCH_SIZE * 1024 (an upper bound for narrow/scattered reads, which the guide
lists as uncalibrated); write bytes = WRITE_SIZE * 1024.

Writes profiles/<tag>/pmc.json, read by bench.py (profiled_traffic) only when the workload and
its algorithmic bytes per launch match the live run.

A class's PMC traffic is REFUSED (no hbm_bytes_per_launch, a "refused" reason instead) when the
counter pass dispatched that class a different number of times than the kernel-trace pass: the
counter run then executed a different schedule (a plan that fell back to exit mode under
the serialising counter passes ran 212 k_plan dispatches against the trace's 1), and its bytes are
not the timed kernel's. A stderr line from the library's watchdog in a counter pass refuses the
whole workload for the same reason.

Usage: python scripts/summarize_profile.py gpurun_out/prof_r2 profiles/r2
"""
from __future__ import annotations

import collections
import csv
import json
import os
import shutil
import sys

WORKLOADS = {"plan": "plan:c3_warehouse_170x84", "plan_exit": "plan_exit:c3_warehouse_170x84",
             "bfs": "bfs:den520d_10k"}


def short(name: str) -> str:
    base = name.split("(")[0]
    return base.replace("void ", "").replace("tsw::", "").split("<")[0]


def kclass(name: str):
    k = short(name)
    if k.startswith("k_astar") or k.startswith("k_enqueue_unknown"):
        return "K3"
    if k.startswith("k_plan"):
        return "k_plan"
    if k.startswith("k_bfs") or k.startswith("k_classify"):
        return "K1"
    return None


def bench_line(path: str):
    try:
        for ln in open(path):
            if ln.startswith('{"metric"'):
                return json.loads(ln)
    except OSError:
        pass
    return None


def main(src: str, dst: str):
    os.makedirs(dst, exist_ok=True)
    out = {"source": src, "correction": "read = 2*FETCH_SIZE KB, write = WRITE_SIZE KB (gfx950)", "workloads": {},
           "build_id": None}
    builds = set()
    for wl, key in WORKLOADS.items():
        stats = os.path.join(src, f"{wl}_trace", "run_kernel_stats.csv")
        line = bench_line(os.path.join(src, f"{wl}_trace.json"))
        if not os.path.exists(stats) or line is None:
            continue
        shutil.copy(stats, os.path.join(dst, f"{wl}_kernel_stats.csv"))
        builds.add(line.get("build_id"))
        cls = collections.defaultdict(lambda: {"device_ns": 0.0, "dispatches": 0, "kernels": {}})
        for r in csv.DictReader(open(stats)):
            c = kclass(r["Name"])
            if c is None:
                continue
            cls[c]["device_ns"] += float(r["TotalDurationNs"])
            cls[c]["dispatches"] += int(r["Calls"])
            cls[c]["kernels"][short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
        # launches and algorithmic bytes per launch as the bench counts them
        if wl in ("plan", "plan_exit"):
            ref = (line.get("roofline") or {}).get("classes", {})
            launches = {c: d["launches"] for c, d in ref.items()}
            algo = {c: d["algorithmic_bytes_per_launch"] for c, d in ref.items()}
        else:
            b = line["bfs"]["roofline"]
            launches = {"K1": cls["K1"]["kernels"].get("k_bfs_blk", {}).get("calls", cls["K1"]["dispatches"])}
            algo = {"K1": b["algorithmic_bytes_per_launch"]}
        for tag, counter in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
            p = os.path.join(src, f"{wl}_{tag}", "run_counter_collection.csv")
            if not os.path.exists(p):
                continue
            tot = collections.defaultdict(float)
            disp = collections.defaultdict(set)
            for r in csv.DictReader(open(p)):
                if r["Counter_Name"] == counter:
                    c = kclass(r["Kernel_Name"])
                    if c:
                        tot[c] += float(r["Counter_Value"])
                        disp[c].add(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(disp[c]))
            for c, v in tot.items():
                cls[c][counter + "_KB_total"] = v
                cls[c][counter + "_dispatches"] = len(disp[c])
            err = os.path.join(src, f"{wl}_{tag}.err")
            if os.path.exists(err) and "watchdog" in open(err, errors="replace").read():
                for c in cls:
                    cls[c]["refused"] = f"{counter} pass: the library's watchdog fired (another schedule than the trace)"
        res = {}
        for c, d in cls.items():
            L = max(int(launches.get(c, 0)), 1)
            e = {"launches": L, "dispatches": d["dispatches"], "device_us_per_launch": d["device_ns"] / L / 1e3,
                 "kernels": d["kernels"], "algorithmic_bytes_per_launch": algo.get(c)}
            for counter in ("FETCH_SIZE", "WRITE_SIZE"):
                nd = d.get(counter + "_dispatches")
                if nd is not None and nd != d["dispatches"] and "refused" not in d:
                    d["refused"] = (f"{counter} pass ran {nd} dispatches of this class, the kernel trace "
                                    f"{d['dispatches']}: not the traced schedule")
            if "refused" in d:
                e["refused"] = d["refused"]
            elif "FETCH_SIZE_KB_total" in d and "WRITE_SIZE_KB_total" in d:
                e["read_bytes_per_launch"] = 2 * d["FETCH_SIZE_KB_total"] * 1024 / L
                e["write_bytes_per_launch"] = d["WRITE_SIZE_KB_total"] * 1024 / L
                e["hbm_bytes_per_launch"] = e["read_bytes_per_launch"] + e["write_bytes_per_launch"]
                if algo.get(c):
                    e["traffic_over_algorithmic"] = e["hbm_bytes_per_launch"] / algo[c]
            if wl in ("plan", "plan_exit"):  # for the planner / worker traffic split (bench.traffic_split)
                ks = line.get("kernel_stats", {})
                if c == "k_plan":
                    e["agent_steps"] = int(line["config"]["agents"]) * int(ks.get("steps", 0))
                if c == "K3":
                    e["queries"] = int(ks.get("astar_queries", 0))
            res[c] = e
        out["workloads"][key] = res
    # provenance: the library build every profiled run loaded; bench.py pairs this file
    # only with that build. Runs of different builds in one directory: no build_id, nothing is paired.
    if len(builds) == 1:
        out["build_id"] = builds.pop()
    else:
        out["build_ids_seen"] = sorted(str(b) for b in builds)
    bj = os.path.join(src, "bench.json")
    if os.path.exists(bj):
        shutil.copy(bj, os.path.join(dst, "bench.json"))
    with open(os.path.join(dst, "pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1)[:4000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
