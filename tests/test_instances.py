"""The benchmark instances are well-formed and keep planning (round 5).

The reference loop (tswap.rs:104-170) has no notion of parking: an Idle agent keeps g = v
(:92-101, :119-121), so a task endpoint on a cell where an agent rests makes rule 3 swap two equal
goals (:198-202) and the plan spins to the cap with nothing moving. The round-1..4 instances did
exactly that (C3 frozen from t = 446, C5 from t = 152, wh10k from t = 1,282). These CPU tests pin
that the instances the bench and the full-horizon GPU parity tests now use are well-formed (task
endpoints disjoint from the start cells) and that their committed oracle digests change at >= 95 %
of timesteps.
"""
import os
import sys

import numpy as np
import pytest

from p2p_distributed_tswap_amd import maps

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from make_digests import instances, load  # noqa: E402


def _cells(a):
    return {(int(x), int(y)) for x, y in np.asarray(a).reshape(-1, 2)}


def test_wf_instance_endpoints_disjoint_from_starts():
    rows = maps.warehouse_map(60, 30, 7)
    starts, tasks = maps.make_wf_instance(rows, 80, 500, 7)
    s = _cells(starts)
    assert len(s) == 80
    ep = _cells(tasks[:, :2]) | _cells(tasks[:, 2:])
    assert not (s & ep)
    assert np.all((tasks[:, 0] != tasks[:, 2]) | (tasks[:, 1] != tasks[:, 3]))
    comp = set(maps.largest_component(rows))
    assert s <= comp and ep <= comp
    # seeded: same seed, same instance
    s2, t2 = maps.make_wf_instance(rows, 80, 500, 7)
    assert np.array_equal(starts, s2) and np.array_equal(tasks, t2)


def test_wf_instance_window():
    rows = maps.sortation_map(64, 64)
    starts, tasks = maps.make_wf_instance(rows, 50, 100, 3, window=(8, 8, 20, 20))
    for x, y in list(_cells(starts)) + list(_cells(tasks[:, :2])) + list(_cells(tasks[:, 2:])):
        assert 8 <= x < 28 and 8 <= y < 28
    assert not (_cells(starts) & (_cells(tasks[:, :2]) | _cells(tasks[:, 2:])))


@pytest.mark.parametrize("name", ["c2_random_32_32_20", "c3_warehouse_170x84", "c5_sortation_1024_10k"])
def test_bench_configs_are_well_formed(name):
    rows, starts, tasks = maps.config_instance(name)
    _, n, m, _ = maps.CONFIGS[name]
    assert starts.shape == (n, 2) and tasks.shape == (m, 4)
    assert not (_cells(starts) & (_cells(tasks[:, :2]) | _cells(tasks[:, 2:])))


@pytest.mark.parametrize("name", ["c2_busy_full", "c3_busy_full", "wh10k_busy_full", "c5_busy_full"])
def test_busy_digests_change_at_every_timestep(name):
    """Done-criterion of VERDICT r4 #1: the committed full-horizon digests of the busy instances change
    at >= 95 % of timesteps (the plan runs to the cap with agents moving)."""
    d = load(name)
    dig = d["digests"]
    assert d["T"] == 2001 and len(dig) == 2001
    changed = sum(1 for t in range(1, len(dig)) if dig[t] != dig[t - 1])
    assert changed >= 0.95 * (len(dig) - 1), f"{name}: only {changed} of {len(dig) - 1} timesteps change"
    assert instances()[name][1] == d["max_t"]


@pytest.mark.parametrize("name,frozen_from", [("c3_full", 446), ("c5_full", 152), ("wh10k_full", 1282)])
def test_legacy_digests_freeze(name, frozen_from):
    """The legacy instances' digests are one repeated state from the verdict's timesteps on (kept as
    extra parity tests, not as the benchmark)."""
    dig = load(name)["digests"]
    assert len(set(dig[frozen_from:])) == 1
    assert dig[frozen_from - 1] != dig[frozen_from] or dig[frozen_from - 2] != dig[frozen_from - 1]


def test_c2_busy_moves_at_every_transition():
    """C2 (configs[1]) planned by the oracle moves agents at all 2,000 transitions with the
    well-formed 16,000-task stream, where the legacy 600-task instance moved at 180 of them."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
    from oracle import OracleGraph

    rows, starts, tasks = maps.config_instance("c2_random_32_32_20")
    rec, _ = OracleGraph(maps.rows_to_array(rows)).mapd(starts, tasks, 300, trace_goals=True)
    assert rec.shape == (200, 301) and maps.moving_timesteps(rec) == 300
