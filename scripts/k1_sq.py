"""K1 instruction counts per goal and per BFS level ("put SQ_INSTS_* per level into the
K1 model"). Input: a `rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES
SQ_WAVE_CYCLES -d DIR -- python3 bench.py --no-plan --no-cpu --bfs-reps 2` directory. Every k_bfs_blk
dispatch of 10,000 den520d goals is summarised; `levels` is the mean BFS depth per goal (372.5 on this
map, measured with TSW_BFS_PROF in round 2 — the eccentricity of the goals, a property of the map).

usage: python scripts/k1_sq.py DIR [OUT_JSON] [--goals 10000] [--levels 372.5]
"""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out", nargs="?")
    ap.add_argument("--goals", type=int, default=10000)
    ap.add_argument("--levels", type=float, default=372.5)
    a = ap.parse_args()
    per = collections.defaultdict(dict)  # dispatch -> counter -> value
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "k_bfs_blk" not in r["Kernel_Name"]:
                    continue
                d = per[int(r["Dispatch_Id"])]
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    # the bench's timed launches are the 10k-goal ones: keep the dispatches with the most waves
    if not per:
        raise SystemExit("no k_bfs_blk dispatch in " + a.dir)
    wmax = max(d.get("SQ_WAVES", 0.0) for d in per.values())
    big = [d for d in per.values() if d.get("SQ_WAVES", 0.0) >= 0.9 * wmax]
    avg = {k: sum(d.get(k, 0.0) for d in big) / len(big) for k in big[0]}
    gl = a.goals * a.levels
    out = {
        "dispatches": len(big), "goals": a.goals, "levels_per_goal": a.levels,
        "per_launch": {k: round(v) for k, v in avg.items()},
        "per_goal": {k: round(v / a.goals, 1) for k, v in avg.items() if k.startswith("SQ_INSTS")},
        "per_goal_level": {k: round(v / gl, 1) for k, v in avg.items() if k.startswith("SQ_INSTS")},
        "insts_per_goal_level": round(sum(v for k, v in avg.items() if k.startswith("SQ_INSTS")) / gl, 1),
        "wave_cycles_per_goal": round(avg.get("SQ_WAVE_CYCLES", 0.0) * 4.0 / a.goals),  # quad-cycles -> cycles
        "note": "SQ_INSTS_* count wave instructions (decode included: per_goal_level is an upper bound of the level "
                "loop's); SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md), reported here in cycles",
    }
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
