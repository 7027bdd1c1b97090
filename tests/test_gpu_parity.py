"""GPU parity: HIP path (through the C ABI) vs the CPU oracle, bit-exact."""
import numpy as np
import pytest

from p2p_distributed_tswap_amd import Planner, TSW_F_EAGER_NEXTHOP, TSW_F_EXIT_MODE, TSW_F_LAZY_NEXTHOP, maps
from oracle import OracleGraph

pytestmark = pytest.mark.gpu


def _grid(name):
    if name == "open8":
        return maps.open_map(8, 8)
    if name == "rand16":
        return maps.random_map(16, 16, 0.25, 3)
    if name == "rand32":
        return maps.random_map(32, 32, 0.20, 0x3232)
    if name == "bundled":
        return maps.bundled_map()
    if name == "warehouse":
        return maps.warehouse_map(170, 84, 0x170084)
    if name == "cave":
        return maps.cave_map(256, 257, 0x520D)
    if name == "serpentine":
        # 200x130 (> 24k cells: byte g-score A*): walls every 4th column with alternating end
        # gaps, so paths detour far beyond the Manhattan distance (exercises the h > 31 hand-off)
        a = np.zeros((130, 200), dtype=bool)
        for i, x in enumerate(range(3, 200, 4)):
            a[:, x] = True
            a[(1 if i % 2 else 128), x] = False
        return maps.to_rows(a)
    raise KeyError(name)


@pytest.mark.parametrize("name,ngoals", [("open8", 64), ("rand32", 300), ("bundled", 64), ("warehouse", 48),
                                         ("cave", 16)])
def test_bfs_tables_bit_exact(name, ngoals):
    rows = _grid(name)
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    free = np.flatnonzero(cells.reshape(-1) != ord("@"))
    rng = np.random.default_rng(1)
    goals = rng.choice(free, size=min(ngoals, free.size), replace=False).astype(np.uint32)
    with Planner(rows) as p:
        got = p.dist_tables(goals)
    for k, g in enumerate(goals):
        ref = og.bfs(int(g))
        assert np.array_equal(got[k], ref), f"{name} goal {g}: {np.count_nonzero(got[k] != ref)} cells differ"


def test_astar_all_pairs_open8():
    rows = _grid("open8")
    og = OracleGraph(maps.rows_to_array(rows))
    s, g = np.meshgrid(np.arange(64), np.arange(64), indexing="ij")
    s, g = s.reshape(-1).astype(np.uint32), g.reshape(-1).astype(np.uint32)
    with Planner(rows) as p:
        nxt, ln = p.get_path_next(s, g)
    for q in range(s.size):
        rn, rl, _ = og.get_path_next(int(s[q]), int(g[q]))
        assert (nxt[q], ln[q]) == (rn, rl), f"query {s[q]}->{g[q]}"


@pytest.mark.parametrize("name,nq", [("rand16", 2000), ("rand32", 4000), ("bundled", 1500), ("warehouse", 800),
                                     ("cave", 300), ("serpentine", 200)])
def test_astar_random_pairs(name, nq):
    rows = _grid(name)
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    free = np.flatnonzero(cells.reshape(-1) != ord("@"))
    rng = np.random.default_rng(2)
    s = rng.choice(free, nq).astype(np.uint32)
    g = rng.choice(free, nq).astype(np.uint32)
    with Planner(rows) as p:
        nxt, ln = p.get_path_next(s, g)
    bad = []
    for q in range(nq):
        rn, rl, _ = og.get_path_next(int(s[q]), int(g[q]))
        if (nxt[q], ln[q]) != (rn, rl):
            bad.append((int(s[q]), int(g[q]), int(nxt[q]), int(ln[q]), rn, rl))
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"


@pytest.mark.parametrize("name", ["warehouse", "cave", "serpentine"])
def test_astar_wave_heap_overflow_handoff(monkeypatch, name):
    """k_astar_wave (grids > 1024 cells) with a tiny LDS heap (read at context creation): queries
    that outgrow it are handed to the global-heap kernel; results stay bit-exact."""
    rows = _grid(name)
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    free = np.flatnonzero(cells.reshape(-1) != ord("@"))
    rng = np.random.default_rng(5)
    s = rng.choice(free, 200).astype(np.uint32)
    g = rng.choice(free, 200).astype(np.uint32)
    monkeypatch.setenv("TSW_ASTAR_WAVE_HCAP", "16")
    with Planner(rows, diag=True) as p:
        nxt, ln = p.get_path_next(s, g)
    for q in range(s.size):
        rn, rl, _ = og.get_path_next(int(s[q]), int(g[q]))
        assert (nxt[q], ln[q]) == (rn, rl), f"query {s[q]}->{g[q]}"


@pytest.mark.parametrize("name,n,seed", [("rand16", 40, 1), ("rand32", 200, 2), ("bundled", 60, 3),
                                          ("warehouse", 300, 4)])
def test_step_matches_oracle(name, n, seed):
    rows = _grid(name)
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    comp = maps.largest_component(rows)
    rng = np.random.default_rng(seed)
    idx = rng.choice(len(comp), size=2 * n, replace=True)
    cellid = np.array([y * cells.shape[1] + x for (x, y) in comp], dtype=np.uint32)
    v = cellid[idx[:n]]
    g = cellid[idx[n:]]
    g[: n // 5] = v[: n // 5]  # some agents at goal (rule 3 partners)
    with Planner(rows) as p:
        for _ in range(6):
            rv, rg = og.step(v, g)
            hv, hg = p.step(v, g)
            assert np.array_equal(hv, rv) and np.array_equal(hg, rg)
            v, g = rv, rg


@pytest.mark.parametrize("name,n,m,seed,flags", [
    ("rand16", 10, 20, 7, 0),
    ("rand16", 30, 90, 8, TSW_F_LAZY_NEXTHOP),
    ("rand32", 200, 600, 0x3232, 0),
    ("rand32", 120, 300, 5, TSW_F_LAZY_NEXTHOP),
    ("bundled", 10, 30, 1, 0),
    ("warehouse", 100, 300, 9, 0),
])
def test_mapd_matches_oracle(name, n, m, seed, flags):
    rows = _grid(name)
    starts, tasks = maps.make_instance(rows, n, m, seed)
    og = OracleGraph(maps.rows_to_array(rows))
    ref, rgoal = og.mapd(starts, tasks, 2000, trace_goals=True)
    with Planner(rows, flags=flags) as p:
        rec, goal = p.plan_mapd_arrays(starts, tasks, 2000, trace_goals=True)
    assert rec.shape == ref.shape
    if not np.array_equal(goal, rgoal):
        t = int(np.argmax((goal != rgoal).any(axis=0)))
        pytest.fail(f"goal divergence first at t={t}")
    assert np.array_equal(rec, ref)


@pytest.mark.parametrize("name,n,seed", [("rand16", 30, 11), ("open8", 20, 12)])
def test_step_duplicate_cells(name, n, seed):
    """Duplicate agent cells: position() picks the lowest index (tswap.rs:192/269)."""
    rows = _grid(name)
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    comp = maps.largest_component(rows)
    cellid = np.array([y * cells.shape[1] + x for (x, y) in comp], dtype=np.uint32)
    rng = np.random.default_rng(seed)
    v = cellid[rng.choice(len(comp), size=n // 2, replace=True)]
    v = np.concatenate([v, v[: n - v.size]])  # every cell doubled
    g = cellid[rng.choice(len(comp), size=n, replace=True)]
    with Planner(rows) as p:
        for _ in range(5):
            rv, rg = og.step(v, g)
            hv, hg = p.step(v, g)
            assert np.array_equal(hv, rv) and np.array_equal(hg, rg)
            v, g = rv, rg


@pytest.mark.parametrize("name,n,m,seed,flags", [
    ("rand32", 200, 600, 0x3232, TSW_F_LAZY_NEXTHOP),
    ("warehouse", 150, 400, 9, 0),
    ("bundled", 40, 120, 10, TSW_F_LAZY_NEXTHOP),
])
def test_mapd_more(name, n, m, seed, flags):
    rows = _grid(name)
    starts, tasks = maps.make_instance(rows, n, m, seed)
    og = OracleGraph(maps.rows_to_array(rows))
    ref, rgoal = og.mapd(starts, tasks, 2000, trace_goals=True)
    with Planner(rows, flags=flags) as p:
        rec, goal = p.plan_mapd_arrays(starts, tasks, 2000, trace_goals=True)
    assert rec.shape == ref.shape
    if not np.array_equal(goal, rgoal):
        t = int(np.argmax((goal != rgoal).any(axis=0)))
        pytest.fail(f"goal divergence first at t={t}")
    assert np.array_equal(rec, ref)


@pytest.mark.parametrize("n,max_t", [(600, 60), (1100, 40)])
def test_mapd_block_paths(n, max_t):
    """k_plan's block-wide paths: n > 512 runs the rules scan across the whole workgroup (not
    wave 0 alone), n > 1024 (block < n) never enters the movement wave tail. A capped horizon
    keeps the oracle fast; records and goals bit-exact."""
    rows = _grid("warehouse")
    starts, tasks = maps.make_instance(rows, n, 3 * n, 0x5EED + n)
    og = OracleGraph(maps.rows_to_array(rows))
    ref, rgoal = og.mapd(starts, tasks, max_t, trace_goals=True)
    with Planner(rows) as p:
        rec, goal = p.plan_mapd_arrays(starts, tasks, max_t, trace_goals=True)
    assert rec.shape == ref.shape
    if not np.array_equal(goal, rgoal):
        t = int(np.argmax((goal != rgoal).any(axis=0)))
        pytest.fail(f"goal divergence first at t={t}")
    assert np.array_equal(rec, ref)


def test_mapd_global_agent_arrays():
    """6,000 agents: the agent arrays no longer fit LDS (global-memory k_plan variant, pointer-
    doubling buffers carved in LDS on their own) — lazy next hops with the wide prefetch on the
    510x220 warehouse, a few timesteps, bit-exact."""
    rows = maps.warehouse_map(510, 220, 0x510220)
    starts, tasks = maps.make_instance(rows, 6000, 18000, 0x6000)
    og = OracleGraph(maps.rows_to_array(rows))
    ref, rgoal = og.mapd(starts, tasks, 4, trace_goals=True)
    with Planner(rows) as p:
        rec, goal = p.plan_mapd_arrays(starts, tasks, 4, trace_goals=True)
    assert rec.shape == ref.shape
    assert np.array_equal(goal, rgoal)
    assert np.array_equal(rec, ref)


@pytest.mark.parametrize("split", ["1", "0"])
def test_mapd_occ_placement(split, monkeypatch):
    """170x84 warehouse: the occupancy grid in LDS without the movement rounds' MU words (default,
    k_plan<.., OC, !MUL>) and both in global memory (TSW_OCC_SPLIT=0), 400 agents, bit-exact."""
    monkeypatch.setenv("TSW_OCC_SPLIT", split)
    rows = maps.warehouse_map(170, 84, 0x170084)
    starts, tasks = maps.make_instance(rows, 400, 1200, 0x400)
    og = OracleGraph(maps.rows_to_array(rows))
    ref, rgoal = og.mapd(starts, tasks, 150, trace_goals=True)
    with Planner(rows, diag=True) as p:
        rec, goal = p.plan_mapd_arrays(starts, tasks, 150, trace_goals=True)
    assert np.array_equal(goal, rgoal)
    assert np.array_equal(rec, ref)


@pytest.mark.parametrize("name,flags,ngoals", [("rand32", TSW_F_EAGER_NEXTHOP, 0), ("rand16", TSW_F_EAGER_NEXTHOP, 0),
                                               ("open8", TSW_F_EAGER_NEXTHOP, 0)])
def test_next_hop_tables_all_pairs(name, flags, ngoals):
    """Every (cell, goal) next hop of the eager tables == get_path(cell, goal)[1] (exhaustive)."""
    rows = _grid(name)
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    free = np.flatnonzero(cells.reshape(-1) != ord("@")).astype(np.uint32)
    goals = free if ngoals == 0 else free[:ngoals]
    with Planner(rows, flags=flags) as p:
        tabs = p.next_hop_tables(goals)
    bad = []
    for k, g in enumerate(goals):
        ref = og.next_codes(int(g))
        got = tabs[k]
        mism = np.flatnonzero((got != ref) & (ref != 0xFF))
        if mism.size:
            bad.append((int(g), int(mism[0]), int(got[mism[0]]), int(ref[mism[0]]), int(mism.size)))
    assert not bad, f"{len(bad)} goals with mismatching next hops, first {bad[:4]}"


@pytest.mark.parametrize("name,n,seed", [("rand32", 200, 2), ("rand32", 300, 5), ("bundled", 400, 6)])
def test_step_deterministic_and_exact(name, n, seed):
    """Repeated identical tsw_step calls (fresh contexts) give identical results == oracle."""
    rows = _grid(name)
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    comp = maps.largest_component(rows)
    rng = np.random.default_rng(seed)
    cellid = np.array([y * cells.shape[1] + x for (x, y) in comp], dtype=np.uint32)
    v = cellid[rng.choice(len(comp), size=n, replace=False)]
    g = cellid[rng.choice(len(comp), size=n, replace=True)]
    g[: n // 4] = v[: n // 4]
    outs = []
    for rep in range(3):
        with Planner(rows) as p:
            vv, gg = v.copy(), g.copy()
            for _ in range(4):
                vv, gg = p.step(vv, gg)
            outs.append((vv, gg))
    rv, rg = v.copy(), g.copy()
    for _ in range(4):
        rv, rg = og.step(rv, rg)
    for rep, (vv, gg) in enumerate(outs):
        dv = np.flatnonzero(vv != rv)
        dg = np.flatnonzero(gg != rg)
        assert dv.size == 0 and dg.size == 0, f"rep {rep}: v differs at {dv[:8]}, g differs at {dg[:8]}"


@pytest.mark.parametrize("mode", ["coop", "serial", "no_tier2"])
def test_astar_wave_cores_and_tiers(monkeypatch, mode):
    """k_astar_wave's wave-cooperative heap (default), the lone-lane core (TSW_ASTAR_SERIAL) and
    the hand-off chain byte-g LDS -> u32-g global slots (tier 2) -> k_astar, or straight to
    k_astar (TSW_ASTAR_NO_TIER2): all bit-exact on long detour queries of the serpentine map."""
    if mode == "serial":
        monkeypatch.setenv("TSW_ASTAR_SERIAL", "1")
    if mode == "no_tier2":
        monkeypatch.setenv("TSW_ASTAR_NO_TIER2", "1")
    rows = _grid("serpentine")
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    W = cells.shape[1]
    free = np.flatnonzero(cells.reshape(-1) != ord("@"))
    rng = np.random.default_rng(9)
    # far-apart columns: the path snakes through many wall gaps (detour >> 62)
    left = free[(free % W) < 20]
    right = free[(free % W) > W - 20]
    s = np.concatenate([rng.choice(left, 48), rng.choice(free, 16)]).astype(np.uint32)
    g = np.concatenate([rng.choice(right, 48), rng.choice(free, 16)]).astype(np.uint32)
    with Planner(rows, diag=mode != "coop") as p:
        nxt, ln = p.get_path_next(s, g)
    for q in range(s.size):
        rn, rl, _ = og.get_path_next(int(s[q]), int(g[q]))
        assert (nxt[q], ln[q]) == (rn, rl), f"query {s[q]}->{g[q]} ({mode})"


@pytest.mark.parametrize("gs", ["auto", "lds", "global"])
def test_astar_wave_batch_gscore_placement(monkeypatch, gs):
    """A k_astar_wave batch with several queries per wave (dynamic dequeue) and the g-scores in
    LDS (small batches), in the global slots (batches larger than the LDS-resident waves, the
    default then) or forced either way: bit-exact on the 170x84 warehouse."""
    if gs != "auto":
        monkeypatch.setenv("TSW_ASTAR_GLOBAL_GS", "1" if gs == "global" else "0")
    rows = _grid("warehouse")
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    free = np.flatnonzero(cells.reshape(-1) != ord("@"))
    rng = np.random.default_rng(13)
    nq = 3000
    s = rng.choice(free, nq).astype(np.uint32)
    g = rng.choice(free, nq).astype(np.uint32)
    with Planner(rows, diag=gs != "auto") as p:
        nxt, ln = p.get_path_next(s, g)
    bad = [q for q in range(nq) if (nxt[q], ln[q]) != og.get_path_next(int(s[q]), int(g[q]))[:2]]
    assert not bad, f"{len(bad)} mismatches ({gs}), first {bad[:5]}"


def test_astar_lds_more_queries_than_slots():
    """k_astar_lds (<= 1024 cells) with more queries than its 65,536 lane slots: the dynamic
    dequeue hands the surplus to lanes that finished early; every answer bit-exact."""
    rows = _grid("rand32")
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    free = np.flatnonzero(cells.reshape(-1) != ord("@"))
    rng = np.random.default_rng(17)
    nq = 70000
    s = rng.choice(free, nq).astype(np.uint32)
    g = rng.choice(free, nq).astype(np.uint32)
    with Planner(rows) as p:
        nxt, ln = p.get_path_next(s, g)
    idx = np.concatenate([np.arange(0, nq, 7), np.arange(65536, nq)])  # surplus checked in full
    bad = [int(q) for q in idx if (nxt[q], ln[q]) != og.get_path_next(int(s[q]), int(g[q]))[:2]]
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"


def _plan_vs_oracle(rows, starts, tasks, max_t, **kw):
    og = OracleGraph(maps.rows_to_array(rows))
    ref, rgoal = og.mapd(starts, tasks, max_t, trace_goals=True)
    with Planner(rows, **kw) as p:
        rec, goal = p.plan_mapd_arrays(starts, tasks, max_t, trace_goals=True)
        st = p.stats()
    assert rec.shape == ref.shape
    if not np.array_equal(goal, rgoal):
        t = int(np.argmax((goal != rgoal).any(axis=0)))
        pytest.fail(f"goal divergence first at t={t}")
    assert np.array_equal(rec, ref)
    return st


@pytest.mark.parametrize("name,n,m,seed,max_t", [("rand32", 200, 600, 0x3232, 2000), ("warehouse", 1000, 3000, 0x170084, 120)])
def test_mapd_exit_mode(name, n, m, seed, max_t):
    """the exit mode (TSW_F_EXIT_MODE: lazy next hops resolved by host-launched K3 passes
    at planner exits, no concurrent workers) on lazy configs, bit-exact; the C3 warehouse prefix
    exercises the speculative queue leftovers resolved at the end of the call."""
    rows = _grid(name)
    starts, tasks = maps.make_instance(rows, n, m, seed)
    st = _plan_vs_oracle(rows, starts, tasks, max_t, flags=TSW_F_LAZY_NEXTHOP | TSW_F_EXIT_MODE)
    assert st["coop_workers"] == 0 and sum(st["plan_exits"]) > 0


def test_mapd_watchdog_fallback_mid_plan():
    """the watchdog fallback. A 1 ms watchdog fires during the C3 plan (one step of 1,000
    agents' assignment already takes longer): the coop plan gives up its waits, the workers leave, the
    call resumes in exit mode from the returned PlanCtl, and the plan stays bit-exact."""
    rows, starts, tasks = maps.config_instance("c3_warehouse_170x84")
    st = _plan_vs_oracle(rows, starts, tasks, 150, watchdog_ms=1)
    assert st["watchdog_fires"] >= 1


def test_mapd_coop_workers_in_plan_dispatch():
    """The C3 prefix in coop mode: the plan dispatch carries its K3 workers (coop_workers > 0), the
    planner never leaves the kernel for K3 (no exits), the workers report busy time; bit-exact."""
    rows, starts, tasks = maps.config_instance("c3_warehouse_170x84")
    st = _plan_vs_oracle(rows, starts, tasks, 150)
    assert st["coop_workers"] > 0 and st["walker_launches"] == 1 and sum(st["plan_exits"]) == 0
    assert st["coop_worker_busy_ms"][0] + st["coop_worker_busy_ms"][1] > 0 and st["watchdog_fires"] == 0


@pytest.mark.parametrize("env", [{"TSW_DAG_EXIT": "0"}, {"TSW_TASK_CHAINS": "0"}, {"TSW_DAG_MASK": "1"}])
def test_mapd_coop_knobs(monkeypatch, env):
    """Coop-mode A/B knobs (diagnostic build) on the C3 prefix, bit-exact: the workers' A* without the
    DAG early exit, with the exit tested after every pop, and without task-chain jobs."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rows, starts, tasks = maps.config_instance("c3_warehouse_170x84")
    st = _plan_vs_oracle(rows, starts, tasks, 150, diag=True)
    assert st["coop_workers"] > 0 and st["watchdog_fires"] == 0


@pytest.mark.parametrize("mask", [0, 0x3, 0x3F, 0x7F])
def test_mapd_partial_lds_agent_arrays(monkeypatch, mask):
    """6,000 agents: the agent arrays do not fit LDS as a set, so k_plan admits them one by one
    (PlanArgs::part_lds, TSW_PART_LDS mask): none, SUCC + ONC, all that fit — bit-exact each way."""
    monkeypatch.setenv("TSW_PART_LDS", str(mask))
    rows = maps.random_map(128, 128, 0.1, 0x6000)
    starts, tasks = maps.make_instance(rows, 6000, 600, 0x6001)
    _plan_vs_oracle(rows, starts, tasks, 30, diag=True)


def test_mapd_workers_leave_when_idle(monkeypatch):
    """coop workers that all leave (idle timeout cut to 20 us, TSW_WORKER_IDLE_US) while the
    planner still needs pairs: the planner sees `alive == 0`, stops waiting within ~1 ms, the call
    relaunches with fresh workers, and the C3 prefix stays bit-exact."""
    monkeypatch.setenv("TSW_WORKER_IDLE_US", "20")
    monkeypatch.setenv("TSW_TASK_CHAINS", "0")  # no long chain jobs keeping workers busy
    rows, starts, tasks = maps.config_instance("c3_warehouse_170x84")
    st = _plan_vs_oracle(rows, starts, tasks, 150, diag=True)
    assert st["coop_workers"] > 0 and st["watchdog_fires"] == 0
    assert st["walker_launches"] >= 2, st["walker_launches"]  # the planner did give up on absent workers


@pytest.mark.parametrize("case", range(4))
@pytest.mark.parametrize("flags", [0, TSW_F_EXIT_MODE])
def test_mapd_task_cells_checked_when_used(case, flags):
    """Off-grid/blocked task cells fail the call only where the reference panics (pickup assigned,
    tswap.rs:136; delivery looked up on reaching the pickup, :112); otherwise the plan is bit-exact."""
    from test_oracle import _lazy_task_cases
    from p2p_distributed_tswap_amd import TSW_EINVAL, TswapError

    rows, starts, tasks, max_t, fails = _lazy_task_cases()[case]
    og = OracleGraph(maps.rows_to_array(rows))
    with Planner(rows, flags=flags) as p:
        if fails:
            with pytest.raises(TswapError) as ei:
                p.plan_mapd_arrays(starts, tasks, max_t)
            assert ei.value.code == TSW_EINVAL
            # the context stays usable: a valid plan afterwards is still exact
            ok = tasks[:2] if case == 1 else tasks[:0]
            ref, _ = og.mapd(starts, ok, 50)
            rec, _ = p.plan_mapd_arrays(starts, ok, 50)
            assert np.array_equal(rec, ref)
            return
        ref, rgoal = og.mapd(starts, tasks, max_t, trace_goals=True)
        rec, goal = p.plan_mapd_arrays(starts, tasks, max_t, trace_goals=True)
    assert np.array_equal(goal, rgoal) and np.array_equal(rec, ref)
