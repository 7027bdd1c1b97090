"""GPU parity for the batched decentralized decision (tsw_decide, k_decide) against the CPU
oracle's restatement of compute_next_move_with_tswap (src/bin/decentralized/agent.rs:329-462),
bit-exact on every output: action, destination, goal-swap partner, rotation participants."""
import random

import numpy as np
import pytest

from p2p_distributed_tswap_amd import Planner, maps
from oracle import OracleGraph
from test_oracle import _decide_cases, _to_cell

pytestmark = pytest.mark.gpu


def _ring_cases(rows, seed, count):
    """Position cycles that Rule 4 can close: agents on a 2 x k loop of an open region, each
    heading to the next loop cell (so its next hop is the next agent), with a stale entry at
    the deciding agent's own cell (the only way the reference's position-keyed check closes a
    cycle, agent.rs:403-411)."""
    rng = random.Random(seed)
    H, W = len(rows), len(rows[0])
    cases = []
    for _ in range(200 * count):
        if len(cases) >= count:
            break
        k = rng.randrange(2, 5)
        x0, y0 = rng.randrange(0, W - k), rng.randrange(0, H - 2)
        loop = [(x0 + i, y0) for i in range(k)] + [(x0 + i, y0 + 1) for i in reversed(range(k))]
        if any(rows[y][x] == "@" for x, y in loop):
            continue
        me = loop[0]
        nb = [(loop[i], loop[(i + 1) % len(loop)]) for i in range(1, len(loop))]
        rng.shuffle(nb)
        nb.insert(rng.randrange(len(nb) + 1), (me, loop[rng.randrange(len(loop))]))  # stale self
        cases.append((me, loop[1], nb))
    return cases


@pytest.mark.parametrize("name,n,seed", [("dense12", 60, 1), ("rand20", 90, 3), ("open6", 20, 4),
                                          ("warehouse", 400, 5), ("cave", 200, 6)])
def test_decide_matches_oracle(name, n, seed):
    rows = {"dense12": lambda: maps.random_map(12, 12, 0.15, 9), "rand20": lambda: maps.random_map(20, 16, 0.2, 5),
            "open6": lambda: maps.open_map(6, 6), "warehouse": lambda: maps.warehouse_map(170, 84, 0x170084),
            "cave": lambda: maps.cave_map(96, 97, 7)}[name]()
    H, W = len(rows), len(rows[0])
    cases = _decide_cases(rows, n, seed) + _ring_cases(rows, seed, 40)
    og = OracleGraph(maps.rows_to_array(rows))
    my_v = np.array([_to_cell(p, W, H) for p, _, _ in cases], dtype=np.uint32)
    my_g = np.array([_to_cell(g, W, H) for _, g, _ in cases], dtype=np.uint32)
    nearby = [[(_to_cell(p, W, H), _to_cell(g, W, H)) for p, g in nb] for _, _, nb in cases]
    with Planner(rows) as p:
        got = p.decide(my_v, my_g, nearby)
    kinds = set()
    for i, (v, g, nb) in enumerate(zip(my_v, my_g, nearby)):
        ref = og.decide(int(v), int(g), [a for a, _ in nb], [b for _, b in nb])
        assert got[i] == ref, f"agent {i}: gpu {got[i]} oracle {ref}"
        kinds.add(ref[0])
    assert {0, 2, 3} <= kinds, kinds
    if name in ("dense12", "rand20", "open6"):
        assert 1 in kinds, kinds


def test_decide_rejects_blocked_agent_cell():
    rows = maps.random_map(12, 12, 0.3, 2)
    cells = maps.rows_to_array(rows).reshape(-1)
    blocked = int(np.flatnonzero(cells == ord("@"))[0])
    free = int(np.flatnonzero(cells != ord("@"))[0])
    from p2p_distributed_tswap_amd import TswapError
    with Planner(rows) as p, pytest.raises(TswapError):
        p.decide([blocked], [free], [[]])
