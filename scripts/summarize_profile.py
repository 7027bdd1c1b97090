"""Summarise a scripts/profile_round.sh output directory into profiles/<tag>/.

Copies the rocprofv3 --kernel-trace --stats summary and writes summary.json with, per kernel:
average duration (kernel trace), calls, and per-launch HBM traffic from the separate PMC passes.
Traffic correction (/opt/skills/guides/MI355X_MICROARCH.md, "HBM"): FETCH_SIZE and WRITE_SIZE are
in KB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so
read bytes = 2 * FETCH_SIZE * 1024 (an upper bound for narrow/scattered reads, which the guide
lists as uncalibrated); write bytes = WRITE_SIZE * 1024.

Usage: python scripts/summarize_profile.py gpurun_out/prof_r1 profiles/r1
"""
from __future__ import annotations

import collections
import csv
import json
import os
import shutil
import sys


def short(name: str) -> str:
    base = name.split("(")[0]
    return base.replace("void ", "").replace("tsw::", "")


def main(src: str, dst: str):
    os.makedirs(dst, exist_ok=True)
    out = {"source": src, "kernels": {}}
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
        for r in csv.DictReader(open(stats)):
            k = short(r["Name"])
            out["kernels"].setdefault(k, {})
            out["kernels"][k].update(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]),
                                     total_ns=float(r["TotalDurationNs"]), pct=float(r["Percentage"]))
    for tag, counter in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        p = os.path.join(src, tag, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] == counter:
                agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            d = out["kernels"].setdefault(k, {})
            d[counter + "_KB_per_launch"] = sum(v) / len(v)
    for k, d in out["kernels"].items():
        if "FETCH_SIZE_KB_per_launch" in d and "WRITE_SIZE_KB_per_launch" in d:
            d["hbm_bytes_per_launch"] = 2 * d["FETCH_SIZE_KB_per_launch"] * 1024 + d["WRITE_SIZE_KB_per_launch"] * 1024
    bj = os.path.join(src, "bench.json")
    if os.path.exists(bj):
        shutil.copy(bj, os.path.join(dst, "bench.json"))
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
