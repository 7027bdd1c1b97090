"""GPU: the multi-GPU ingest paths on one device ("the multi-GPU ingest path has never
run on a GPU").

* K1 shards built with tsw_dist_tables_device by two contexts ("ranks"), laid out rank-major as
  sharding.build_and_allgather gathers them, then tsw_import_tables_device into a fresh context:
  its plan equals the oracle's and the self-built plan, and the importing context ran no K1.
* K3 shards (tsw_next_hop_tables_device: every multi-candidate cell resolved) + tables, imported
  with tsw_import_next_hops_device: the plan needs neither K1 nor K3 for those goals and is exact.
Device buffers come from the HIP runtime the library links (test_gpu_bfs._DevBuf)."""
import numpy as np
import pytest

from p2p_distributed_tswap_amd import Planner, maps, sharding
from oracle import OracleGraph
from test_gpu_bfs import _DevBuf

pytestmark = pytest.mark.gpu


def _goalset(rows, starts, tasks):
    w = len(rows[0])
    cells = [y * w + x for x, y in starts.tolist()]
    cells += [y * w + x for x, y in tasks[:, :2].tolist()] + [y * w + x for x, y in tasks[:, 2:].tolist()]
    return np.array(sorted(set(cells)), dtype=np.uint32)


def _gathered(rows, goals, world, codes):
    """Build every rank's shard in its own context and lay the shards out as the all-gather does."""
    ncell = len(rows) * len(rows[0])
    per = sharding.shard_rows(goals.size, world)
    dbuf = _DevBuf(world * per * ncell * 2)
    cbuf = _DevBuf(world * per * ncell) if codes else None
    for r, gl, off in sharding.gathered_blocks(goals, world):
        with Planner(rows) as p:
            if codes:  # codes + the K1 tables they came from, one K1 build
                p.next_hop_tables_device(gl, cbuf.ptr.value + off * ncell, dbuf.ptr.value + off * ncell * 2)
                assert p.stats()["bfs_goals"] == gl.size
            else:
                p.dist_tables_device(gl, dbuf.ptr.value + off * ncell * 2)
    return dbuf, cbuf, per


@pytest.mark.parametrize("name,n,m,seed", [("warehouse", 150, 400, 9), ("rand32", 120, 300, 5)])
def test_import_tables_then_plan(name, n, m, seed):
    rows = maps.warehouse_map(170, 84, 0x170084) if name == "warehouse" else maps.random_map(32, 32, 0.2, 0x3232)
    starts, tasks = maps.make_instance(rows, n, m, seed)
    goals = _goalset(rows, starts, tasks)
    ncell = len(rows) * len(rows[0])
    dbuf, _, _ = _gathered(rows, goals, 2, codes=False)
    ref, rgoal = OracleGraph(maps.rows_to_array(rows)).mapd(starts, tasks, 2000, trace_goals=True)
    with Planner(rows) as p:
        for _, gl, off in sharding.gathered_blocks(goals, 2):
            p.import_tables_device(gl, dbuf.ptr.value + off * ncell * 2)
        rec, goal = p.plan_mapd_arrays(starts, tasks, 2000, trace_goals=True)
        assert p.stats()["bfs_goals"] == 0  # every table came from the import
    with Planner(rows) as p:
        rec2, _ = p.plan_mapd_arrays(starts, tasks, 2000)
    assert np.array_equal(goal, rgoal) and np.array_equal(rec, ref)
    assert np.array_equal(rec2, rec)


@pytest.mark.parametrize("name,n,m,seed", [("rand32", 200, 600, 0x3232), ("rand16", 30, 90, 8)])
def test_sharded_next_hops_then_plan(name, n, m, seed):
    rows = maps.random_map(32, 32, 0.2, 0x3232) if name == "rand32" else maps.random_map(16, 16, 0.25, 3)
    starts, tasks = maps.make_instance(rows, n, m, seed)
    goals = _goalset(rows, starts, tasks)
    ncell = len(rows) * len(rows[0])
    og = OracleGraph(maps.rows_to_array(rows))
    dbuf, cbuf, _ = _gathered(rows, goals, 2, codes=True)
    codes = cbuf.to_host(np.empty((2 * sharding.shard_rows(goals.size, 2), ncell), dtype=np.uint8))
    for _, gl, off in sharding.gathered_blocks(goals, 2):  # every gathered code == get_path()[1]
        for j, g in enumerate(gl[:5]):
            assert np.array_equal(codes[off + j], og.next_codes(int(g)))
    ref, rgoal = og.mapd(starts, tasks, 2000, trace_goals=True)
    with Planner(rows) as p:
        for _, gl, off in sharding.gathered_blocks(goals, 2):
            p.import_next_hops_device(gl, dbuf.ptr.value + off * ncell * 2, cbuf.ptr.value + off * ncell)
        p.reset_stats()
        rec, goal = p.plan_mapd_arrays(starts, tasks, 2000, trace_goals=True)
        st = p.stats()
    assert st["bfs_goals"] == 0 and st["astar_queries"] == 0  # no K1, no K3 on the planning GPU
    assert np.array_equal(goal, rgoal) and np.array_equal(rec, ref)


@pytest.mark.parametrize("name,n,m,seed,world,max_t", [
    ("warehouse", 300, 900, 5, 2, 2000),
    ("warehouse", 1000, 3000, 0x170084, 3, 400),
    ("rand32", 200, 600, 0x3232, 2, 2000),
])
def test_plan_with_k3_sharded_by_goal_owner(name, n, m, seed, world, max_t):
    """SURVEY §8e row 2 as specified, on one device: the planner's every K3 batch goes to the
    "rank" (its own context) owning each pair's goal (goal % world), answered by
    tsw_next_hop_codes from that rank's table store, and gathered (sharding._codes_for_rank + MIN,
    exactly what ShardedK3 does over RCCL). The plan equals the oracle's and the replica plan."""
    from test_gpu_parity import _grid

    rows = _grid(name)
    starts, tasks = maps.make_instance(rows, n, m, seed)
    og = OracleGraph(maps.rows_to_array(rows))
    ref, rgoal = og.mapd(starts, tasks, max_t, trace_goals=True)
    owners = [Planner(rows) for _ in range(world)]
    calls = []

    def resolve(st, gl):
        calls.append(st.size)
        parts = [sharding._codes_for_rank(st, gl, r, world, owners[r].next_hop_codes) for r in range(world)]
        return np.minimum.reduce(parts)

    try:
        with Planner(rows) as p:
            rec, goal = p.plan_mapd_resolved(starts, tasks, max_t, resolve, trace_goals=True)
            st = p.stats()
        assert st["bfs_goals"] > 0 and st["astar_launches"] == 0  # the planner ran no K3 itself
        owned = [o.stats()["bfs_goals"] for o in owners]
    finally:
        for o in owners:
            o.close()
    assert calls and sum(owned) > 0 and min(owned) > 0  # every owner built its own goals' tables
    if not np.array_equal(goal, rgoal):
        t = int(np.argmax((goal != rgoal).any(axis=0)))
        pytest.fail(f"goal divergence first at t={t}")
    assert np.array_equal(rec, ref)


def test_next_hop_codes_match_oracle():
    """tsw_next_hop_codes (a goal owner's answers) == get_path(start, goal)[1] of the oracle, on
    random pairs, twice (the second call is served from the store)."""
    from test_gpu_parity import _grid

    rows = _grid("warehouse")
    cells = maps.rows_to_array(rows)
    w = cells.shape[1]
    og = OracleGraph(cells)
    free = np.flatnonzero(cells.reshape(-1) != ord("@")).astype(np.uint32)
    rng = np.random.default_rng(7)
    st = rng.choice(free, 600).astype(np.uint32)
    gl = rng.choice(free[:200], 600).astype(np.uint32)
    st[:5] = gl[:5]  # start == goal: code 4
    want = np.empty(st.size, np.uint8)
    for i, (s, g) in enumerate(zip(st.tolist(), gl.tolist())):
        nxt, _, _ = og.get_path_next(s, g)
        d = nxt - s
        want[i] = 4 if nxt == s else 0 if d == w else 1 if d == 1 else 2 if d == -w else 3
    with Planner(rows) as p:
        assert np.array_equal(p.next_hop_codes(st, gl), want)
        assert np.array_equal(p.next_hop_codes(st, gl), want)
