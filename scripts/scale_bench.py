"""End-to-end MAPD planning at scale on one GPU vs the single-thread CPU restatement.

north_star: "a 10k-agent warehouse instance planned end-to-end faster than the host-CPU reference".
For each instance: the GPU plans the full horizon (cap 2000) from an empty table store (K1 BFS
tables + next-hop resolution + every timestep on the device) and is timed end to end; the CPU
oracle (oracle/tswap_oracle.c, -O2, one thread — the checker, used here only as the timed
baseline) plans a bounded PREFIX of timesteps, is timed, and its prefix is compared bit-exactly
with the GPU's. CPU whole-plan time is extrapolated from the prefix rate (labelled as such).

usage: python scripts/scale_bench.py [instance ...] [--cpu-steps N]
instances: c3 (warehouse 170x84, 1,000 agents, well-formed 32,000-task stream — BASELINE configs[2]),
           wh10k (warehouse 510x220, 10,000 agents, well-formed 40,000 tasks — the north_star instance),
           c5 (1024x1024 sortation floor, 10,000 agents packed in a 160x160 window, 24,000 tasks — configs[4]),
           c3_legacy / wh10k_legacy / c5_legacy: the round-1..4 instances (plans freeze before the cap)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from p2p_distributed_tswap_amd import Planner, maps  # noqa: E402

# name: (instance factory -> (rows, starts, tasks), CPU prefix timesteps)
INSTANCES = {
    "c3": (lambda: maps.config_instance("c3_warehouse_170x84"), 20),
    "wh10k": (maps.wh10k_instance, 3),
    "c5": (maps.c5_instance, 2),
    "c3_legacy": (maps.c3_legacy_instance, 20),
    "wh10k_legacy": (maps.wh10k_legacy_instance, 3),
    "c5_legacy": (maps.c5_legacy_instance, 2),
}


def _heartbeat(stop, t0):
    """A long plan is one blocking C call: print progress (stderr) so a batch runner sees it is alive."""
    while not stop.wait(20.0):
        print(f"[scale_bench] still running, {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)


def main():
    import threading

    ap = argparse.ArgumentParser()
    ap.add_argument("instances", nargs="*", default=["c3", "wh10k"])
    ap.add_argument("--cpu-steps", type=int, default=0, help="CPU prefix timesteps (0: per-instance default)")
    ap.add_argument("--max-t", type=int, default=2000)
    ap.add_argument("--diag", action="store_true", help="diagnostic library (TSW_* knobs)")
    ap.add_argument("--cpu-windows", default="",
                    help="comma-separated extra CPU prefixes (e.g. 20): each timed separately, so the rate of "
                         "every window between consecutive prefixes is reported (prefix-rate spread)")
    args = ap.parse_args()
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import OracleGraph  # CPU baseline + prefix check only

    for name in args.instances:
        fac, cpu_steps = INSTANCES[name]
        cpu_steps = args.cpu_steps or cpu_steps
        rows, starts, tasks = fac()
        n, m = starts.shape[0], tasks.shape[0]
        h, w = len(rows), len(rows[0])
        stop = threading.Event()
        hb = threading.Thread(target=_heartbeat, args=(stop, time.perf_counter()), daemon=True)
        hb.start()
        try:
            with Planner(rows, diag=args.diag) as p:
                print(f"[scale_bench] {name}: warm-up", file=sys.stderr, flush=True)
                p.plan_mapd_arrays(starts[:8], tasks[:8], 4)  # context warm-up (not timed)
                p.clear_tables()
                p.reset_stats()
                print(f"[scale_bench] {name}: plan", file=sys.stderr, flush=True)
                t0 = time.perf_counter()
                rec, _ = p.plan_mapd_arrays(starts, tasks, args.max_t)
                gpu_s = time.perf_counter() - t0
                st = p.stats()
        finally:
            stop.set()
        T = rec.shape[1]
        og = OracleGraph(maps.rows_to_array(rows))
        stop = threading.Event()  # the oracle is one long C call: keep printing (batch runners see it alive)
        hb = threading.Thread(target=_heartbeat, args=(stop, time.perf_counter()), daemon=True)
        hb.start()
        windows = []
        prev_T, prev_s = 0, 0.0
        for pre in sorted({int(x) for x in args.cpu_windows.split(",") if x}):
            if pre >= cpu_steps:
                continue
            tw = time.perf_counter()
            wrec, _ = og.mapd(starts, tasks, pre)
            ws = time.perf_counter() - tw
            windows.append({"timesteps": [prev_T, int(wrec.shape[1])], "s": round(ws - prev_s, 3),
                            "agent_steps_per_s": round(n * (wrec.shape[1] - prev_T) / max(ws - prev_s, 1e-9), 1)})
            prev_T, prev_s = int(wrec.shape[1]), ws
        tc = time.perf_counter()
        crec, _ = og.mapd(starts, tasks, cpu_steps)
        cpu_s = time.perf_counter() - tc
        ct = crec.shape[1]
        if windows:
            windows.append({"timesteps": [prev_T, int(ct)], "s": round(cpu_s - prev_s, 3),
                            "agent_steps_per_s": round(n * (ct - prev_T) / max(cpu_s - prev_s, 1e-9), 1)})
        stop.set()
        prefix_ok = bool(np.array_equal(crec, rec[:, :ct]))
        cpu_rate = n * ct / cpu_s
        out = {
            "instance": name, "grid": f"{w}x{h}", "agents": n, "tasks": m, "timesteps": int(T),
            "timesteps_moving": maps.moving_timesteps(rec),
            "gpu_end_to_end_s": round(gpu_s, 3), "gpu_agent_steps_per_s": round(n * T / gpu_s, 1),
            "cpu_prefix_timesteps": int(ct), "cpu_prefix_s": round(cpu_s, 3),
            "cpu_agent_steps_per_s": round(cpu_rate, 1),
            "cpu_end_to_end_s_extrapolated": round(n * T / cpu_rate, 1),
            "speedup_end_to_end": round((n * T / cpu_rate) / gpu_s, 1),
            "prefix_bit_exact": prefix_ok,
            "cpu_prefix_windows": windows,
            "tables": st["tables"], "bfs_ms": round(st["bfs_ms"], 2), "astar_ms": round(st["astar_ms"], 2),
            "plan_ms": round(st["plan_ms"], 2), "astar_queries": st["astar_queries"],
            "astar_launches": st["astar_launches"], "plan_launches": st["walker_launches"],
            "plan_section_ms": [round(x, 2) for x in st["plan_section_ms"]],
            "plan_exits_by_section": st["plan_exits"], "rule_rounds": st["rule_rounds"],
            "coop_waits": st["coop_waits"], "coop_wait_ms": round(st["coop_wait_ms"], 2),
            "coop_wait_sec_ms": [round(x, 2) for x in st["coop_wait_sec_ms"]],
            "coop_waits_sec": st["coop_waits_sec"], "relabels_full": st["relabels_full"],
            "relabels_inc": st["relabels_inc"], "coop_workers": st["coop_workers"],
            "coop_worker_busy_ms": [round(x, 1) for x in st["coop_worker_busy_ms"]],
            "env": {k: v for k, v in os.environ.items() if k.startswith("TSW_")},
        }
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
