"""bench.py — TSWAP agent-steps/s (+ BFS cells/s and % HBM peak) on MI355X.

Contract (driver): python bench.py --gpus N --steps K --warmup W ; for N > 1 it is
launched under torch.distributed.run, one rank per GPU. Rank 0 prints ONE JSON line.

Workload: BASELINE.json configs[2], the largest single-GPU planning config — warehouse-like
170x84 grid (shelf blocks, 1-wide aisles, seed 0x170084), 1,000 agents, a well-formed 32,000-task
MAPD stream (task endpoints disjoint from the agents' start cells, maps.make_wf_instance; the
stream outlasts the horizon, so every one of the 2,001 timesteps moves agents — the round-1..4
instance froze from t = 446), reference step cap (timestep > 2000). One bench "step" = one complete tsw_plan_mapd over that
instance from an empty table store: K1 BFS tables for every goal cell, next-hop resolution (K3
exact A*), then every timestep's K4 assign -> K2 step -> record on the device. The instance
(a few KB of host arrays) is handed over through the C ABI like the reference's
`tswap_mapd(grid, starts, tasks)`. value = agent-steps (n x T summed over ranks) / max-over-ranks
wall time of the K timed steps. N > 1: the planning step does not shard (sequential agent order,
SURVEY.md §8e), so each rank plans its own replica (seed + rank) — weak scaling.

Extra objects on the line:
  roofline      the kernel class with the most device time inside the timed steps (HIP events
                on the library's stream, tsw_get_stats), algorithmic bytes per launch, and the
                PMC traffic per launch from profiles/<PROFILE_TAG>/pmc.json — only when that file
                was measured on THIS workload (same algorithmic bytes per launch) with THIS build
                (its build_id equals the loaded library's tsw_build_id), else null. The
                plan dispatch (k_plan) carries the planner AND its exact-A* workers (coop mode): its
                algorithmic bytes are 46 B per agent-step plus 17 B per worker query.
  latency       k_plan against its latency floor (bound "latency"): rules / movement rounds x the
                measured floor per round shape (tsw_probe_round_floors), beside the achieved section
                time; the K3 wait time (the A* critical path) beside it. DESIGN.md "Latency roofline".
  bfs           K1 alone on a den520d-like 256x257 cave, 10,000 distinct goals (configs[3]),
                cells/s and fraction of the 8 TB/s HBM peak (algorithmic bytes).
  cpu_baseline  the oracle (faithful single-thread C restatement of tswap.rs) planning a bounded
                prefix of the same instance on one pinned host core, rank 0 only; its prefix is
                also compared bit-exactly with the GPU plan, and the GPU plans the SAME prefix
                (same max_t, from an empty table store) for a like-for-like rate.
  sharded_plan  N > 1 with --sharded-k3 only: C5 (configs[4]) planned once on rank 0 with its K3
                sharded per step by goal owner across all ranks (tsw_plan_mapd_resolved +
                sharding.ShardedK3, RCCL), timed against rank 0's replica plan of C5 alone. Off by
                default: a plan's K3 time is the latency of single queries, which more GPUs do not
                shorten (Multi-GPU, has the model). The N > 1 data path is the goal-sharded
                K1 + RCCL all-gather in the `bfs` object (den520d, configs[3]).
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

HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md ("HBM: 8 TB/s peak")
PROFILE_TAG = "r6"     # profiles/<tag>/pmc.json: PMC traffic per workload (scripts/profile_round.sh)
BFS_WORKLOAD = "bfs:den520d_10k"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-bfs", action="store_true", help="skip the K1 BFS measurement")
    ap.add_argument("--no-plan", action="store_true", help="skip the planning leg (profiling K1 alone)")
    ap.add_argument("--no-sharded", action="store_true", help=argparse.SUPPRESS)  # round-4 scripts: now the default
    ap.add_argument("--sharded-k3", action="store_true",
                    help="N > 1: also run the sharded-K3 C5 leg (per-step query batches by goal owner); a measured "
                         "null result, off by default (DESIGN.md, Multi-GPU)")
    ap.add_argument("--diag", action="store_true", help="diagnostic library (TSW_* A/B knobs; not the product)")
    ap.add_argument("--exit-mode", action="store_true",
                    help="TSW_F_EXIT_MODE: no K3 workers in the plan dispatch (K3 as host-launched passes) — "
                         "the profile's planner-only traffic (VERDICT r3 #7), not the headline")
    ap.add_argument("--bfs-goals", type=int, default=10000)
    ap.add_argument("--bfs-reps", type=int, default=3)
    ap.add_argument("--cpu-steps", type=int, default=300,
                    help="timesteps of the CPU baseline's prefix (bounded sample of the same plan)")
    ap.add_argument("--config", default="c3_warehouse_170x84")
    ap.add_argument("--nexthop", choices=("auto", "eager", "lazy"), default="auto",
                    help="next-hop resolution policy (TSW_F_EAGER_NEXTHOP / TSW_F_LAZY_NEXTHOP)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI, default) or gloo (rehearsing N ranks on one GPU)")
    return ap.parse_args()


def running_build_id(diag: bool = False):
    try:
        from p2p_distributed_tswap_amd import build_id
        return build_id(diag)
    except Exception:  # noqa: BLE001 — no library: nothing can be paired with a profile
        return None


def profiled_traffic(workload: str, kclass: str, algo_bytes_per_launch: float, build: str = None):
    """HBM bytes per launch of kernel class `kclass` measured by PMC on `workload`
    (profiles/<PROFILE_TAG>/pmc.json, written by scripts/summarize_profile.py from separate
    FETCH_SIZE / WRITE_SIZE passes with the gfx950 FETCH_SIZE x2 correction). Returned only if the
    profiled run had the same algorithmic bytes per launch (within 2 %) AND was recorded with the
    library build that is running now (pmc.json `build_id` == tsw_build_id): a profile
    of another workload or of other code never feeds this line."""
    p = os.path.join(ROOT, "profiles", PROFILE_TAG, "pmc.json")
    try:
        with open(p) as f:
            pj = json.load(f)
        d = pj["workloads"][workload][kclass]
    except (OSError, ValueError, KeyError):
        return None, None
    if build is None or pj.get("build_id") != build:
        return None, None
    a = float(d.get("algorithmic_bytes_per_launch", 0.0))
    if a <= 0 or abs(a - algo_bytes_per_launch) > 0.02 * algo_bytes_per_launch or "hbm_bytes_per_launch" not in d:
        return None, None
    return float(d["hbm_bytes_per_launch"]), os.path.relpath(p, ROOT)


def traffic_split(config: str, coop_traffic, steps: int, queries: int, build: str = None):
    """the coop plan dispatch carries the planner AND its K3 workers, so its PMC bytes
    are split with profiles/<tag>/warm_split.json (scripts/warm_split.py): the same plan run warm in
    one context (every next-hop code already stored: the workers only idle-poll) gives the planner's
    bytes per agent-step; the workers' part is the cold dispatch's bytes minus that. The exit-mode
    profile (workload plan_exit) is kept as a cross-check of K3's bytes per query; it cannot give the
    planner's share (every exit relaunch re-stages the planner's state)."""
    base = os.path.join(ROOT, "profiles", PROFILE_TAG)
    out = {}
    try:
        with open(os.path.join(base, "warm_split.json")) as f:
            ws = json.load(f)
        if ws.get("config") == config and build is not None and ws.get("build_id") == build:
            out = {"source": os.path.relpath(os.path.join(base, "warm_split.json"), ROOT),
                   "method": "warm vs cold plan dispatch (PMC), same instance",
                   "planner_bytes_per_agent_step": ws["planner_bytes_per_agent_step"],
                   "planner_algorithmic_bytes_per_agent_step": ws["planner_algorithmic_bytes_per_agent_step"],
                   "profiled_workers_bytes_per_query": ws["workers_bytes_per_query"]}
    except (OSError, ValueError, KeyError, TypeError):
        out = {}
    try:
        with open(os.path.join(base, "pmc.json")) as f:
            k3 = json.load(f)["workloads"][f"plan_exit:{config}"].get("K3", {})
        if "hbm_bytes_per_launch" in k3 and k3.get("queries"):
            out["exit_mode_k3_bytes_per_query"] = round(k3["hbm_bytes_per_launch"] * k3["launches"] / k3["queries"], 1)
    except (OSError, ValueError, KeyError, TypeError):
        pass
    if not out:
        return None
    if coop_traffic is not None and steps and queries and "planner_bytes_per_agent_step" in out:
        planner_part = out["planner_bytes_per_agent_step"] * steps  # steps: agent-steps of one launch
        out["coop_dispatch_bytes"] = round(coop_traffic, 1)
        out["planner_part_bytes"] = round(planner_part, 1)
        out["workers_part_bytes"] = round(coop_traffic - planner_part, 1)
        out["workers_bytes_per_query"] = round((coop_traffic - planner_part) / queries, 1)
    return out


def bfs_bytes_per_goal(w: int, h: int, with_nh: bool) -> int:
    """Algorithmic HBM bytes of one K1 goal: u16 table write (+u8 next-hop codes when fused)
    + the obstacle bitmap read."""
    cells = w * h
    return cells * 2 + (cells if with_nh else 0) + (cells + 7) // 8


# block-wide passes every timestep makes outside the rounds (ASSIGN compaction, PRE1 and PRE2 refresh,
# movement init, RECORD): the per-step part of k_plan's floor
STEP_PASSES = 5


def latency_roofline(st: dict, us_wave: float, us_pass: float) -> dict:
    """k_plan against its latency floor (DESIGN.md "Latency roofline"). k_plan runs tswap_step's two
    sequential scans as rounds of one workgroup; a round's floor is the dependent chain its shape
    cannot avoid, measured live by tsw_probe_round_floors: a wave-0 rules firing (LDS load, ballot,
    first lane, readlane, store) and a block-wide pass (LDS exchange + barrier; a movement round is
    three). floor = rule_rounds * wave + (3 * move_rounds + STEP_PASSES * steps) * pass. achieved =
    section device time minus the time the planner waited for K3 (exact A* on the concurrent workers:
    the other critical path, reported beside it)."""
    sec, wsec = st["plan_section_ms"], st["coop_wait_sec_ms"]
    rr, mr, steps = st["rule_rounds"], st["move_rounds"], st["steps"]

    def part(rounds, us_round, achieved_ms):
        floor_ms = rounds * us_round / 1e3
        return {"rounds": int(rounds), "rounds_per_step": round(rounds / max(steps, 1), 2),
                "floor_us_per_round": round(us_round, 4),
                "achieved_us_per_round": round(achieved_ms * 1e3 / max(rounds, 1), 4),
                "floor_ms": round(floor_ms, 3), "achieved_ms": round(achieved_ms, 3),
                "frac": round(floor_ms / achieved_ms, 4) if achieved_ms > 0 else None}

    rules = part(rr, us_wave, sec[2] - wsec[2])
    move = part(mr, 3.0 * us_pass, sec[4] - wsec[4])
    achieved = st["walker_ms"] - st["coop_wait_ms"]
    floor = rules["floor_ms"] + move["floor_ms"] + STEP_PASSES * steps * us_pass / 1e3
    return {
        "k_plan": {"bound": "latency", "unit": "ms", "floor_ms": round(floor, 3), "achieved_ms": round(achieved, 3),
                   "frac": round(floor / achieved, 4) if achieved > 0 else None,
                   "steps": int(steps), "step_passes": STEP_PASSES},
        "rules": rules,
        "movement": move,
        "probe": {"us_wave_round": round(us_wave, 4), "us_block_pass": round(us_pass, 4),
                  "block": int(st.get("plan_block", 0))},
        "k3_wait_ms": round(st["coop_wait_ms"], 3),
        "k3_waits": int(st["coop_waits"]),
    }


def host_cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(rows, starts, tasks, n_agents, steps, gpu_rec, gpu_prefix=None):
    """The C oracle (single thread, -O2) planning the first `steps` timesteps of the same instance,
    pinned to one host core (sched_setaffinity = taskset -c <core>), compared with the GPU plan."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import OracleGraph  # CPU baseline (and prefix check) only

    og = OracleGraph(np.frombuffer("".join(rows).encode("latin-1"), dtype=np.uint8).reshape(len(rows), -1))
    old = os.sched_getaffinity(0)
    core = min(old)
    os.sched_setaffinity(0, {core})
    try:
        tc = time.perf_counter()
        rec, _ = og.mapd(starts, tasks, steps)
        tcd = time.perf_counter() - tc
    finally:
        os.sched_setaffinity(0, old)
    T = rec.shape[1]
    return {
        "value": round(n_agents * T / tcd, 1),
        "unit": "agent-steps/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"first {T} timesteps of the same plan ({n_agents} agents x {T} = {n_agents * T} agent-steps, "
                   f"{tcd:.2f} s), oracle/tswap_oracle.c -O2, one thread pinned to core {core} "
                   f"(sched_setaffinity, = taskset -c {core})"),
        "host_cpu": host_cpu_model(),
        "host_cores_total": os.cpu_count(),
        "host_cores_allowed": len(old),
        "prefix_bit_exact_vs_gpu": bool(gpu_rec is not None and np.array_equal(rec, gpu_rec[:, :T])),
        # the GPU timed on the same sample (same instance, same max_t, empty table store),
        # so the CPU/GPU ratio compares the same work; the headline value covers the full horizon
        "gpu_same_sample": gpu_prefix,
        "gpu_over_cpu_same_sample": (round(gpu_prefix["agent_steps_per_s"] / (n_agents * T / tcd), 1)
                                     if gpu_prefix else None),
        "note": ("a C port with dense stamped arrays (no HashMap) and the Rust std BinaryHeap restated: "
                 "likely faster than the Rust original, so the GPU/CPU ratio is conservative"),
    }


def goal_set(rows, starts, tasks) -> np.ndarray:
    """The closed goal set of a MAPD instance (start cells, pickups, deliveries: goals only move
    between agents by rule 3/4, tswap.rs:198-249), as sorted cell ids."""
    w = len(rows[0])
    c = np.concatenate([starts[:, 1] * w + starts[:, 0], tasks[:, 1] * w + tasks[:, 0], tasks[:, 3] * w + tasks[:, 2]])
    return np.unique(c.astype(np.uint32))


def sharded_plan_leg(args, rank, world, dev, dist, barrier, allmax):
    """N > 1: the multi-GPU pipeline on the instance where the planner's time is K3 — C5 (BASELINE
    configs[4]: 1024x1024 sortation floor, 10,000 agents, dense rotations; ~1M exact-A* queries per
    plan) — planned ONCE on rank 0 with its K3 sharded per step by goal owner:
    tsw_plan_mapd_resolved runs the planner in exit mode and hands every stop's batch of (start, goal)
    pairs to sharding.ShardedK3, which broadcasts it, lets the rank owning each goal (goal % N) answer
    from its own table store (tsw_next_hop_codes: K1 + exact A* for its goals only) and gathers the
    u8 codes with one all-reduce(MIN) over RCCL. Timed against the replica plan of the same instance
    on rank 0 alone (coop mode: K3 workers inside the plan dispatch), bit-exact against it. K1 tables
    are NOT all-gathered here: C5's 17,885 tables are 36 GB of u16, more than the 279 ms they take to
    build (the `bfs` object carries the goal-sharded K1 + all-gather on den520d)."""
    from p2p_distributed_tswap_amd import Planner, maps, sharding

    rows, starts, tasks = maps.c5_instance()
    n = starts.shape[0]
    owner = Planner(rows, device=dev)
    planner = Planner(rows, device=dev) if rank == 0 else None
    ref_rec, replica_s = None, None
    if rank == 0:
        planner.plan_mapd_arrays(starts[:8], tasks[:8], 4)  # context warm-up
        planner.clear_tables()
        t0 = time.perf_counter()
        ref_rec, _ = planner.plan_mapd_arrays(starts, tasks, 2000)
        replica_s = time.perf_counter() - t0
    times, rec, stops, pairs = [], None, 0, 0
    for rep in range(2):  # warm-up + one timed plan (a C5 plan is seconds)
        owner.clear_tables()
        if planner is not None:
            planner.clear_tables()
            planner.reset_stats()
        barrier()
        t0 = time.perf_counter()
        res, sk = sharding.plan_sharded_k3(
            rank, world, dist, "cuda" if args.dist_backend == "nccl" else "cpu", owner.next_hop_codes,
            (lambda r: planner.plan_mapd_resolved(starts, tasks, 2000, r)) if rank == 0 else None)
        barrier()
        dt = allmax(time.perf_counter() - t0)
        if rep == 1:
            times.append(dt)
            stops, pairs = sk.stops, sk.pairs
            if rank == 0:
                rec = res[0]
    st = planner.stats() if planner is not None else None
    owner.close()
    if planner is not None:
        planner.close()
    if rank != 0:
        return None
    return {
        "instance": "c5_sortation_1024_10k (BASELINE configs[4]): 1024x1024, 10,000 agents, well-formed 24,000-task stream, cap 2000",
        "k3": f"per-step batches sharded by goal owner (goal % {world}) over {args.dist_backend}, all-reduce(MIN) of u8 codes",
        "sharded_plan_s": round(times[0], 3),
        "replica_plan_s_rank0_alone": round(replica_s, 3),
        "speedup_vs_replica": round(replica_s / times[0], 3),
        "agent_steps_per_s": round(n * rec.shape[1] / times[0], 1),
        "planner_stops": int(stops), "k3_pairs_resolved_by_owners": int(pairs),
        "planner_k1_goals": int(st["bfs_goals"]), "planner_section_ms": [round(x, 1) for x in st["plan_section_ms"]],
        "bit_exact_vs_replica_plan": bool(ref_rec is not None and np.array_equal(rec, ref_rec)),
        "backend": args.dist_backend,
    }


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

    from p2p_distributed_tswap_amd import TSW_F_EAGER_NEXTHOP, TSW_F_EXIT_MODE, TSW_F_LAZY_NEXTHOP, Planner, maps

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

    _, n_agents, n_tasks, _ = maps.CONFIGS[args.config]
    rows, starts, tasks = maps.config_instance(args.config, rank)  # replicas: seed + rank
    h, w = len(rows), len(rows[0])
    build = running_build_id(args.diag)
    workload = f"{'plan_exit' if args.exit_mode else 'plan'}:{args.config}"

    value = dt_max = None
    Ts, st, roofline, latency, last_rec = [], {}, None, None, None
    if not args.no_plan:
        pflags = {"auto": 0, "eager": TSW_F_EAGER_NEXTHOP, "lazy": TSW_F_LAZY_NEXTHOP}[args.nexthop]
        if args.exit_mode:
            pflags |= TSW_F_EXIT_MODE
        planner = Planner(rows, device=dev, flags=pflags, diag=args.diag)

        def one_plan():
            planner.clear_tables()
            rec, _ = planner.plan_mapd_arrays(starts, tasks, 2000)
            return rec

        for _ in range(args.warmup):
            one_plan()
        planner.reset_stats()
        barrier()
        t0 = time.perf_counter()
        agent_steps = 0
        for _ in range(args.steps):
            last_rec = one_plan()
            Ts.append(int(last_rec.shape[1]))
            agent_steps += n_agents * last_rec.shape[1]
        barrier()
        dt = time.perf_counter() - t0
        st = planner.stats()
        dt_max = allmax(dt)
        value = allsum(float(agent_steps)) / dt_max
        # latency floors of k_plan's round shapes on its own workgroup size (tsw_probe.hip), measured
        # after the timed region
        us_wave, us_pass = planner.probe_round_floors(0)
        gpu_prefix = None
        if rank == 0 and not args.no_cpu:
            # the CPU baseline's sample on the GPU (outside the timed region)
            planner.clear_tables()
            torch.cuda.synchronize()
            tp = time.perf_counter()
            prec, _ = planner.plan_mapd_arrays(starts, tasks, args.cpu_steps)
            tpd = time.perf_counter() - tp
            gpu_prefix = {"timesteps": int(prec.shape[1]), "s": round(tpd, 4),
                          "agent_steps_per_s": round(n_agents * prec.shape[1] / tpd, 1),
                          "bit_exact_vs_full_plan": bool(np.array_equal(prec, last_rec[:, :prec.shape[1]]))}
        planner.close()

        # kernel classes inside the timed region (device time from HIP events on the library stream)
        steps_total = st["steps"]
        # K3 in coop mode runs INSIDE the plan dispatch (workgroups 1.. of k_plan): its time is the
        # workers' A* busy time summed over worker waves (wave-ms, overlapping the dispatch), plus any
        # host-launched K3 passes (exit mode / eager tables: HIP events)
        worker_wave_ms = float(sum(st["coop_worker_busy_ms"]))
        cats = {
            "K3": ("exact A* next hop (get_path tswap.rs:288-390): coop workers inside the plan dispatch "
                   "+ host-launched k_astar_wave / k_astar_lds / k_astar passes",
                   st["astar_ms"] + worker_wave_ms, st["astar_launches"],
                   # every query read (16 B) + its next-hop code written (1 B)
                   17.0 * st["astar_queries"] / max(st["astar_launches"], 1)),
            "k_plan": ("k_plan dispatch (K2 tswap_step + K4 assignment, persistent planner, tswap.rs:104-286; "
                       "with its coop K3 workers)",
                       st["walker_ms"], st["walker_launches"],
                       # ~46 B per agent-step, + 17 B per query the in-dispatch workers ran
                       (46.0 * n_agents * steps_total + 17.0 * st["astar_queries"]) / max(st["walker_launches"], 1)),
            "K1": ("k_bfs_blk + k_classify (BFS tables + next-hop codes)", st["bfs_ms"], st["bfs_launches"],
                   bfs_bytes_per_goal(w, h, True) * st["bfs_goals"] / max(st["bfs_launches"], 1)),
        }
        # the dominant kernel: the most DEVICE time (dispatch-level; K3's wave-ms overlap k_plan)
        dom = max(("k_plan", "K1") + (("K3",) if worker_wave_ms == 0.0 else ()), key=lambda k: cats[k][1])
        name, dom_ms, dom_launches, per_launch_bytes = cats[dom]
        avg_launch_ms = dom_ms / max(dom_launches, 1)
        achieved = per_launch_bytes / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms > 0 else 0.0
        traffic, traffic_src = profiled_traffic(workload, dom, per_launch_bytes, build)
        roofline = {
            "kernel": name,
            "bound": "hbm",
            "achieved": round(achieved, 4),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 8),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "avg_launch_us": round(avg_launch_ms * 1e3, 3),
            "launches": int(dom_launches),
            "algorithmic_bytes_per_launch": round(per_launch_bytes, 1),
            # every kernel class of the timed plans (scripts/summarize_profile.py pairs these with PMC)
            "classes": {k: {"device_ms": round(v[1], 3), "launches": int(v[2]),
                            "algorithmic_bytes_per_launch": round(v[3], 1)} for k, v in cats.items()},
            "k3_workers": {"waves": int(st["coop_workers"]), "busy_wave_ms": round(worker_wave_ms, 3),
                           "busy_wave_ms_by_queue": {q: round(x, 3) for q, x in
                                                     zip(("needed", "speculative", "task_chains"),
                                                         st["coop_worker_busy_ms"])},
                           "note": "K3 device_ms = these busy wave-ms (workers run inside the k_plan dispatch) "
                                   "+ host-launched K3 passes"},
            "note": ("K3 and k_plan move a few bytes per serial heap / commit step: their HBM fraction is tiny by "
                     "construction and their binding limit is latency (see `latency`). K1 (bfs.roofline) is the "
                     "HBM-bound kernel." if dom != "K1" else None),
        }
        plans = max(int(st["walker_launches"]), 1) if dom == "k_plan" else max(args.steps, 1)
        roofline["traffic_split"] = (traffic_split(args.config, traffic, n_agents * steps_total / plans,
                                                   st["astar_queries"] / plans, build)
                                     if dom == "k_plan" and not args.exit_mode else None)
        latency = latency_roofline(st, us_wave, us_pass)

    sharded = None
    if world > 1 and not args.no_plan and args.sharded_k3:
        sharded = sharded_plan_leg(args, rank, world, dev, dist, barrier, allmax)

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
        gather_ms = local_ms = None
        if dist is not None:
            # the alternative the sharded build competes with: every rank builds all the
            # goals' tables itself, no collective (wall time, max over ranks)
            allout = torch.empty((goals.size, ncell), dtype=torch.int16, device="cuda")
            barrier()
            tl = time.perf_counter()
            cp.dist_tables_device(goals, allout.data_ptr())
            barrier()
            local_ms = allmax(time.perf_counter() - tl) * 1e3
            del allout
            # goal-sharded K1 + RCCL all-gather over xGMI (north_star), then every rank ingests
            # every table into its table store (sharding.py)
            from p2p_distributed_tswap_amd import sharding

            build_fn = lambda g, o: cp.dist_tables_device(g, o.data_ptr())  # noqa: E731
            barrier()
            tg = time.perf_counter()
            full = sharding.build_and_allgather(goals, ncell, rank, world, build_fn, dist, "cuda")
            barrier()
            gather_ms = allmax(time.perf_counter() - tg) * 1e3
            torch.cuda.synchronize()
            for _, gl, off in sharding.gathered_blocks(goals, world):
                if gl.size:
                    cp.import_tables_device(gl, full[off:off + gl.size].data_ptr())
            del full
        cells_per_s = allsum(float(mine.size * ncell)) * args.bfs_reps / tbw
        k_gbs = mine.size * bytes_goal / (k_ms * 1e-3) / 1e9 if k_ms > 0 else 0.0
        algo_launch = float(mine.size * bytes_goal)
        btraffic, btraffic_src = (profiled_traffic(BFS_WORKLOAD, "K1", algo_launch, build) if world == 1
                                  else (None, None))
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
                "traffic": btraffic,
                "traffic_source": btraffic_src,
                "algorithmic_bytes_per_launch": int(algo_launch),
            },
            # N > 1: wall time of (this rank's K1 shard + RCCL all-gather of all tables), max over ranks
            "sharded_build_allgather_ms": round(gather_ms, 3) if gather_ms is not None else None,
            # ... and the same N ranks each building all goals locally (the sharded form pays iff smaller)
            "local_build_all_goals_ms": round(local_ms, 3) if local_ms is not None else None,
        }
        del out
        cp.close()

    cpu = None
    if rank == 0 and not args.no_cpu and not args.no_plan:
        cpu = cpu_baseline(rows, starts, tasks, n_agents, args.cpu_steps, last_rec, gpu_prefix)

    if rank == 0:
        line = {
            "metric": "TSWAP agent-steps/sec + BFS cells/sec (% HBM peak) at 1/2/4/8 GPUs",
            "value": round(value, 1) if value is not None else None,
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 3) if dt_max is not None else None,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded warehouse-like map and MAPD task stream; replicas seed+rank)",
            "config": {
                "workload": (f"{args.config}: {w}x{h} grid, {n_agents} agents, "
                             f"{'well-formed ' if args.config in maps.WELL_FORMED else ''}{n_tasks}-task MAPD "
                             "stream, cap 2000, full plan from an empty table store per step "
                             f"(BASELINE configs[{list(maps.CONFIGS).index(args.config)}])"),
                "agents": n_agents, "tasks": n_tasks, "grid": f"{w}x{h}",
                "well_formed": args.config in maps.WELL_FORMED,
                "timesteps_per_plan": Ts,
                # timesteps t >= 1 of the last timed plan in which any agent moved
                "timesteps_moving": maps.moving_timesteps(last_rec) if last_rec is not None else None,
                "parallelism": f"replicas x{world} (step not shardable)",
            },
            "build_id": build,
            "roofline": roofline,
            "latency": latency,
            "bfs": bfs,
            "cpu_baseline": cpu,
            "sharded_plan": sharded,
            "kernel_stats": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()},
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
