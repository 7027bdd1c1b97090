"""GPU: the committed golden fixtures and single-step KATs through the C ABI (bit-exact)."""
import json
import os

import numpy as np
import pytest

from p2p_distributed_tswap_amd import Planner, TSW_F_EAGER_NEXTHOP, TSW_F_LAZY_NEXTHOP

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _files(prefix):
    return sorted(f for f in os.listdir(GOLD) if f.startswith(prefix))


@pytest.mark.parametrize("fname", _files("mapd_"))
@pytest.mark.parametrize("flags", [TSW_F_EAGER_NEXTHOP, TSW_F_LAZY_NEXTHOP])
def test_golden_mapd_gpu(fname, flags):
    z = np.load(os.path.join(GOLD, fname))
    with Planner(z["grid"], flags=flags) as p:
        rec, goals = p.plan_mapd_arrays(z["starts"], z["tasks"], int(z["max_t"]), trace_goals=True)
    assert rec.shape == z["rec"].shape
    assert np.array_equal(goals, z["goals"]) and np.array_equal(rec, z["rec"])


@pytest.mark.parametrize("fname", _files("astar_"))
def test_golden_astar_gpu(fname):
    z = np.load(os.path.join(GOLD, fname))
    with Planner(z["grid"]) as p:
        nxt, ln = p.get_path_next(z["start"], z["goal"])
    assert np.array_equal(nxt, z["next"]) and np.array_equal(ln, z["len"])


@pytest.mark.parametrize("fname", _files("bfs_"))
def test_golden_bfs_gpu(fname):
    z = np.load(os.path.join(GOLD, fname))
    with Planner(z["grid"]) as p:
        assert np.array_equal(p.dist_tables(z["goals"]), z["tables"])


def _kats():
    with open(os.path.join(GOLD, "kats.json")) as f:
        return json.load(f)["kats"]


@pytest.mark.parametrize("kat", _kats(), ids=lambda k: k["name"])
@pytest.mark.parametrize("flags", [TSW_F_EAGER_NEXTHOP, TSW_F_LAZY_NEXTHOP])
def test_kats_gpu(kat, flags):
    with Planner(kat["grid"], flags=flags) as p:
        v, g = p.step(np.array(kat["v"], dtype=np.uint32), np.array(kat["g"], dtype=np.uint32))
    assert list(v) == kat["v_after"] and list(g) == kat["g_after"]
