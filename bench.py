"""bench.py — TSWAP agent-steps/s (+ BFS cells/s and % HBM peak) on MI355X.

Contract (driver): python bench.py --gpus N --steps K --warmup W ; for N > 1 it is
launched under torch.distributed.run, one rank per GPU. Rank 0 prints ONE JSON line.

Workload (BASELINE.json configs[1]): random-32-32-20 grid (Bernoulli 0.20, seed 0x3232),
200 agents, 600-task MAPD stream, reference step cap (timestep > 2000). One bench "step"
= one complete tsw_plan_mapd over that instance from an empty table store: K1 BFS tables
for every goal cell, next-hop resolution (K3 A*), then every timestep's K4 assign ->
K2 step -> record on the device. value = agent-steps (n x T summed over ranks) / max-over-
ranks wall time of the K timed steps. N > 1: the planning step does not shard (sequential
agent order), so each rank plans its own replica (seed + rank) — weak scaling.

Extra objects on the line:
  roofline      for the kernel with the most device time inside the timed steps, from
                HIP events on the library's stream (tsw_get_stats).
  bfs           K1 alone on a den520d-like 256x257 cave, 10,000 distinct goals (configs[3]),
                cells/s and fraction of the 8 TB/s HBM peak (algorithmic bytes).
  cpu_baseline  the oracle (faithful single-thread C restatement of tswap.rs) on the same
                instance, rank 0 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md:36


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-bfs", action="store_true", help="skip the K1 BFS measurement")
    ap.add_argument("--bfs-goals", type=int, default=10000)
    ap.add_argument("--bfs-reps", type=int, default=3)
    ap.add_argument("--config", default="c2_random_32_32_20")
    ap.add_argument("--nexthop", choices=("auto", "eager", "lazy"), default="auto",
                    help="next-hop resolution policy (TSW_F_EAGER_NEXTHOP / TSW_F_LAZY_NEXTHOP)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI, default) or gloo (rehearsing N ranks on one GPU)")
    return ap.parse_args()


def profiled_traffic(kernel_prefix: str):
    """Per-launch HBM bytes of a kernel from the newest committed PMC summary
    (profiles/<round>/summary.json, made by scripts/profile_round.sh + summarize_profile.py:
    separate FETCH_SIZE / WRITE_SIZE passes, gfx950 FETCH_SIZE x2 correction)."""
    import glob

    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "summary.json")), key=os.path.getmtime)
    for p in reversed(paths):
        try:
            with open(p) as f:
                ks = json.load(f)["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        for name, d in ks.items():
            if name.startswith(kernel_prefix) and "hbm_bytes_per_launch" in d:
                return float(d["hbm_bytes_per_launch"]), os.path.relpath(p, ROOT)
    return None, None


def bfs_bytes_per_goal(w: int, h: int, with_nh: bool) -> int:
    """Algorithmic HBM bytes of one K1 goal: u16 table write (+u8 next-hop codes when fused)
    + the obstacle bitmap read."""
    cells = w * h
    return cells * 2 + (cells if with_nh else 0) + (cells + 7) // 8


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    dev = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(args.dist_backend)

    from p2p_distributed_tswap_amd import Planner, maps

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def allmax(x: float) -> float:
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def allsum(x: float) -> float:
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    fac, n_agents, n_tasks, seed = maps.CONFIGS[args.config]
    rows = fac()
    h, w = len(rows), len(rows[0])
    starts, tasks = maps.make_instance(rows, n_agents, n_tasks, seed + rank)
    from p2p_distributed_tswap_amd import TSW_F_EAGER_NEXTHOP, TSW_F_LAZY_NEXTHOP

    pflags = {"auto": 0, "eager": TSW_F_EAGER_NEXTHOP, "lazy": TSW_F_LAZY_NEXTHOP}[args.nexthop]
    planner = Planner(rows, device=dev, flags=pflags)

    def one_plan():
        planner.clear_tables()
        rec, _ = planner.plan_mapd_arrays(starts, tasks, 2000)
        return rec.shape[1]

    for _ in range(args.warmup):
        one_plan()
    planner.reset_stats()
    barrier()
    t0 = time.perf_counter()
    agent_steps = 0
    Ts = []
    for _ in range(args.steps):
        T = one_plan()
        Ts.append(T)
        agent_steps += n_agents * T
    barrier()
    dt = time.perf_counter() - t0
    st = planner.stats()
    dt_max = allmax(dt)
    total_units = allsum(float(agent_steps))
    value = total_units / dt_max

    # dominant kernel inside the timed region (device time from HIP events)
    cats = {
        "k_astar (K3 exact A* next hop)": (st["astar_ms"], st["astar_launches"]),
        "k_plan (K2 tswap_step + K4 assignment, persistent)": (st["walker_ms"], st["walker_launches"]),
        "k_bfs (K1 BFS tables + next-hop codes)": (st["bfs_ms"], st["bfs_launches"]),
    }
    dom = max(cats, key=lambda k: cats[k][0])
    dom_ms, dom_launches = cats[dom]
    avg_launch_ms = dom_ms / max(dom_launches, 1)
    steps_total = st["steps"]
    if dom.startswith("k_bfs"):
        per_launch_bytes = bfs_bytes_per_goal(w, h, True) * st["bfs_goals"] / max(st["bfs_launches"], 1)
    else:
        # ~46 B per agent-step for the step/assign kernels; per launch =
        # agent-steps covered by one launch of that kernel
        per_launch_bytes = 46.0 * n_agents * steps_total / max(dom_launches, 1)
    achieved = per_launch_bytes / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms > 0 else 0.0
    traffic, traffic_src = profiled_traffic(dom.split()[0])
    roofline = {
        "kernel": dom,
        "bound": "hbm",
        "achieved": round(achieved, 3),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 6),
        "traffic": traffic,
        "traffic_source": traffic_src,
        "avg_launch_us": round(avg_launch_ms * 1e3, 3),
        "launches": int(dom_launches),
        "note": ("k_plan is one persistent workgroup executing tswap_step's sequential agent-order "
                 "semantics (tswap.rs:180-285) as exact parallel rounds; it is latency/barrier-bound, "
                 "so its HBM fraction is tiny by construction. K1 (bfs.roofline) is the HBM-bound kernel."
                 if dom.startswith("k_plan") else None),
        "algorithmic_bytes_per_launch": round(per_launch_bytes, 1),
        "device_ms_by_kernel": {k.split()[0]: round(v[0], 3) for k, v in cats.items()},
    }

    # K1 BFS alone, den520d-like, 10k distinct goals (configs[3]); rank-local shard of the goals
    bfs = None
    if not args.no_bfs:
        crow = maps.cave_map(256, 257, 0x520D)
        ccells = maps.rows_to_array(crow).reshape(-1)
        free = np.flatnonzero(ccells != ord("@")).astype(np.uint32)
        rng = np.random.default_rng(0x520D)
        goals = np.sort(rng.choice(free, size=min(args.bfs_goals, free.size), replace=False)).astype(np.uint32)
        mine = goals[rank::world]
        cp = Planner(crow, device=dev)
        ncell = 256 * 257
        out = torch.empty((mine.size, ncell), dtype=torch.int16, device="cuda")
        cp.dist_tables_device(mine, out.data_ptr())  # warm-up
        cp.reset_stats()
        barrier()
        tb = time.perf_counter()
        for _ in range(args.bfs_reps):
            cp.dist_tables_device(mine, out.data_ptr())
        barrier()
        tbw = allmax(time.perf_counter() - tb)
        cst = cp.stats()
        k_ms = cst["bfs_ms"] / max(cst["bfs_launches"], 1)
        bytes_goal = bfs_bytes_per_goal(256, 257, False)
        gather_ms = None
        if dist is not None:
            # goal-sharded K1 + RCCL all-gather over xGMI (north_star), then every rank ingests
            # every table into its table store (sharding.py)
            from p2p_distributed_tswap_amd import sharding

            build = lambda g, o: cp.dist_tables_device(g, o.data_ptr())  # noqa: E731
            barrier()
            tg = time.perf_counter()
            full = sharding.build_and_allgather(goals, ncell, rank, world, build, dist, "cuda")
            barrier()
            gather_ms = allmax(time.perf_counter() - tg) * 1e3
            torch.cuda.synchronize()
            for _, gl, off in sharding.gathered_blocks(goals, world):
                if gl.size:
                    cp.import_tables_device(gl, full[off:off + gl.size].data_ptr())
            del full
        cells_per_s = allsum(float(mine.size * ncell)) * args.bfs_reps / tbw
        k_gbs = mine.size * bytes_goal / (k_ms * 1e-3) / 1e9 if k_ms > 0 else 0.0
        btraffic, btraffic_src = profiled_traffic("k_bfs_blk")
        bfs = {
            "workload": "den520d-like 256x257 cave (seed 0x520D), distinct goals",
            "goals_total": int(goals.size),
            "goals_per_rank": int(mine.size),
            "cells_per_s": round(cells_per_s, 1),
            "kernel_avg_ms": round(k_ms, 4),
            "kernel_GBps": round(k_gbs, 2),
            "hbm_frac": round(k_gbs / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_goal": bytes_goal,
            # K1 against the HBM roofline: algorithmic bytes per launch (u16 table
            # write + obstacle bitmap read, per goal x goals per launch) / HIP-event launch time
            "roofline": {
                "kernel": "k_bfs_blk (K1 batched BFS tables)",
                "bound": "hbm",
                "achieved": round(k_gbs, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(k_gbs / HBM_PEAK_GBS, 4),
                "traffic": btraffic if world == 1 else None,
                "traffic_source": btraffic_src if world == 1 else None,
                "algorithmic_bytes_per_launch": int(mine.size * bytes_goal),
            },
            # N > 1: wall time of (this rank's K1 shard + RCCL all-gather of all tables), max over ranks
            "sharded_build_allgather_ms": round(gather_ms, 3) if gather_ms is not None else None,
        }
        del out
        cp.close()

    cpu = None
    if rank == 0 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle import OracleGraph  # CPU baseline only

        og = OracleGraph(maps.rows_to_array(rows))
        tc = time.perf_counter()
        rec, _ = og.mapd(starts, tasks, 2000)
        tcd = time.perf_counter() - tc
        cpu = {
            "value": round(n_agents * rec.shape[1] / tcd, 1),
            "unit": "agent-steps/s",
            "cores": 1,
            "kind": "port",
            "sample": f"1 full plan of the same instance ({n_agents} agents x {rec.shape[1]} timesteps, "
                      f"{tcd:.2f} s, single thread, oracle/tswap_oracle.c -O2)",
        }

    if rank == 0:
        line = {
            "metric": "TSWAP agent-steps/sec + BFS cells/sec (% HBM peak) at 1/2/4/8 GPUs",
            "value": round(value, 1),
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded random-32-32-20 map and MAPD task stream; replicas seed+rank)",
            "config": {
                "workload": "random-32-32-20, 200 agents, 600-task MAPD stream, cap 2000 (BASELINE configs[1])",
                "agents": n_agents, "tasks": n_tasks, "grid": f"{w}x{h}",
                "timesteps_per_plan": Ts, "parallelism": f"replicas x{world} (step not shardable)",
            },
            "roofline": roofline,
            "bfs": bfs,
            "cpu_baseline": cpu,
            "kernel_stats": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()},
        }
        print(json.dumps(line), flush=True)
    planner.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
