"""GPU parity on the BASELINE configs at their real sizes (VERDICT r1 "close the untested configs").

* C3 (configs[2]): warehouse 170x84, 1,000 agents, well-formed 32,000-task stream, full horizon (cap
  2000) — every timestep's records and goals against the oracle's per-timestep digests
  (tests/golden/digests_c3_busy.json, made by tests/golden/make_digests.py). Every one of its 2,001
  timesteps moves agents (round 5; the round-1..4 instance, which froze from t = 446, stays as
  `c3_full`).
* C5 (configs[4]): 1024x1024 sortation floor, 10,000 agents packed in a 160x160 window (dense
  traffic, rule-3 swaps and rule-4 rotations every step):
    - K1 tables of a seeded goal sample vs the oracle BFS,
    - next hops (get_path(...)[1] and len) on random pairs vs the oracle A*,
    - a 6-timestep MAPD prefix and the full horizon vs the oracle digests.
Reference: tswap.rs:39-172 (tswap_mapd), :174-286 (tswap_step), :288-390 (get_path)."""
import json
import os

import numpy as np
import pytest

from p2p_distributed_tswap_amd import Planner, maps
from oracle import OracleGraph

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _digests(name):
    import sys

    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_digests import load, step_digests

    # every digest file is committed: a missing one is a failure, not a skip
    return load(name), step_digests


def _check_digests(name, rec, goals):
    ref, step_digests = _digests(name)
    got = step_digests(rec, goals)
    assert rec.shape == (ref["agents"], ref["T"]), (rec.shape, ref["agents"], ref["T"])
    bad = [t for t, (a, b) in enumerate(zip(got, ref["digests"])) if a != b]
    assert not bad, f"{name}: first divergent timestep {bad[0]} ({len(bad)} of {ref['T']})"


def _plan_against_digests(name):
    import sys

    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_digests import instances

    ref, _ = _digests(name)
    fac, max_t, _ = instances()[name]
    assert max_t == ref["max_t"]
    rows, starts, tasks = fac()
    with Planner(rows) as p:
        rec, goals = p.plan_mapd_arrays(starts, tasks, max_t, trace_goals=True)
    _check_digests(name, rec, goals)


@pytest.mark.parametrize("name", ["c3_busy_full", "c3_full"])
def test_c3_full_horizon_matches_oracle(name):
    """C3 over the full horizon: the busy well-formed instance (the bench's) and the legacy one."""
    _plan_against_digests(name)


@pytest.mark.parametrize("name", ["c2_busy_full", "c2_legacy_full"])
def test_c2_full_horizon_matches_oracle(name):
    """C2 (configs[1], random-32-32-20, 200 agents) over the full horizon: the well-formed 16,000-task
    stream (every transition moves agents; round 6) and the round-1..5 600-task instance."""
    _plan_against_digests(name)


def test_c3_busy_movement_round_tag_wrap():
    """The movement rounds' MU words sit in LDS as u32 with a 16-bit round tag, cleared when the tag
    wraps (tsw_plan.hip, MU32). Starting the round counter at 65,000 (TSW_MOVE_ROUND0, diagnostic
    build) puts the wrap ~535 rounds into the busy C3 plan; every timestep must still match the oracle."""
    import sys

    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_digests import instances

    name = "c3_busy_full"
    ref, _ = _digests(name)
    fac, max_t, _ = instances()[name]
    rows, starts, tasks = fac()
    old = os.environ.get("TSW_MOVE_ROUND0")
    os.environ["TSW_MOVE_ROUND0"] = "65000"
    try:
        with Planner(rows, diag=True) as p:
            rec, goals = p.plan_mapd_arrays(starts, tasks, max_t, trace_goals=True)
            assert p.stats()["move_rounds"] > 65535
    finally:
        if old is None:
            os.environ.pop("TSW_MOVE_ROUND0", None)
        else:
            os.environ["TSW_MOVE_ROUND0"] = old
    _check_digests(name, rec, goals)


@pytest.fixture(scope="module")
def c5():
    rows, starts, tasks = maps.c5_instance()
    return rows, starts, tasks, OracleGraph(maps.rows_to_array(rows))


def test_c5_bfs_tables(c5):
    rows, starts, tasks, og = c5
    cells = maps.rows_to_array(rows).reshape(-1)
    free = np.flatnonzero(cells != ord("@"))
    rng = np.random.default_rng(0xC5)
    # window cells (where C5's goals live) and cells anywhere on the floor
    win = np.array([y * 1024 + x for (x, y) in starts[:2000].tolist()], dtype=np.uint32)
    goals = np.concatenate([rng.choice(win, 24, replace=False), rng.choice(free, 8, replace=False)]).astype(np.uint32)
    with Planner(rows) as p:
        got = p.dist_tables(goals)
    for k, g in enumerate(goals):
        ref = og.bfs(int(g))
        assert np.array_equal(got[k], ref), f"goal {g}: {np.count_nonzero(got[k] != ref)} cells differ"


def test_c5_next_hops(c5):
    rows, starts, tasks, og = c5
    rng = np.random.default_rng(0xC55)
    cid = np.array([y * 1024 + x for (x, y) in starts.tolist()], dtype=np.uint32)
    tc = np.array([y * 1024 + x for (x, y) in tasks[:, :2].tolist()], dtype=np.uint32)
    s = rng.choice(cid, 300).astype(np.uint32)
    g = rng.choice(tc, 300).astype(np.uint32)
    with Planner(rows) as p:
        nxt, ln = p.get_path_next(s, g)
    bad = [q for q in range(s.size) if (nxt[q], ln[q]) != og.get_path_next(int(s[q]), int(g[q]))[:2]]
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"


def test_c5_mapd_prefix(c5):
    rows, starts, tasks, og = c5
    with Planner(rows) as p:
        rec, goals = p.plan_mapd_arrays(starts, tasks, 6, trace_goals=True)
    ref, step_digests = _digests("c5_busy_p50")  # a 6-step plan = the first 7 digests of the prefix
    assert step_digests(rec, goals) == ref["digests"][:7]


@pytest.mark.parametrize("name", ["wh10k_busy_p100", "wh10k_busy_full", "wh10k_p300", "wh10k_full"])
def test_wh10k_long_horizon_matches_oracle(name):
    """the north_star's 10k-agent warehouse (510x220, 10,000 agents) over the
    full horizon (2,001 timesteps), every timestep's records and goals against the oracle's digests —
    the busy well-formed 40,000-task instance (every timestep moves agents, so the incremental
    relabels, batched rule-3 firings and the coop PENDING protocol run all the way), its plain-oracle
    100-step prefix, and the legacy 30,000-task instance (frozen from t = 1,282)."""
    _plan_against_digests(name)


@pytest.mark.parametrize("name", ["c5_busy_p50", "c5_busy_full", "c5_p300", "c5_full"])
def test_c5_long_horizon_matches_oracle(name):
    """C5 (1024x1024 sortation floor, 10,000 agents in dense rotation traffic)
    over the full horizon against the oracle's per-timestep digests: the busy well-formed 24,000-task
    instance, its plain-oracle prefix, and the legacy instance (frozen from t = 152)."""
    _plan_against_digests(name)
