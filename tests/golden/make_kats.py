"""Known-answer tests for single tswap_step calls (tests/golden/kats.json).

Each KAT is one (grid, v, g) -> (v', g') step that exercises one rule of tswap_step
(src/algorithm/tswap.rs:174-286): rule 3 goal swap, rule 4 rotation (2- and >=3-cycles),
the chase "clear" when the chain revisits a non-i agent (:224-227), the mutual swap in
the movement phase (:273-278), an agent moving twice in one step, the unreachable-goal
fallback (:378-389) and duplicate start cells (position() = lowest index).
A few are written by hand; the rest are found by searching seeded random configurations
with an instrumented copy of the step. Expected outputs come from the pure-Python
restatement and are re-checked against the C oracle before being written.
"""
from __future__ import annotations

import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from oracle import OracleGraph  # noqa: E402
import py_restatement as pr  # noqa: E402
from p2p_distributed_tswap_amd import maps  # noqa: E402


def instrumented_step(agents, G, ev):
    """py_restatement.tswap_step with event counters (same semantics)."""
    n = len(agents)

    def position(u):
        for k, a in enumerate(agents):
            if a[0] == u:
                return k
        return None

    for i in range(n):
        if agents[i][0] == agents[i][1]:
            continue
        path = G.get_path(agents[i][0], agents[i][1])
        u = path[1]
        j = position(u)
        if j is None or j == i:
            continue
        if agents[j][0] == agents[j][1]:
            ev.add("rule3")
            agents[i][1], agents[j][1] = agents[j][1], agents[i][1]
        else:
            a_p = [i]
            cur = j
            found = False
            while True:
                bv, bg = agents[cur]
                if bv == bg:
                    break
                bpath = G.get_path(bv, bg)
                c = position(bpath[1])
                if c is None:
                    break
                if cur in a_p:
                    a_p.clear()
                    ev.add("clear")
                    break
                a_p.append(cur)
                cur = c
                if cur == i:
                    found = True
                    break
            if found and len(a_p) > 1:
                ev.add("rule4_cycle2" if len(a_p) == 2 else "rule4_cycle3plus")
                first = a_p[0]
                last_goal = agents[a_p[-1]][1]
                for k in range(len(a_p) - 1, 0, -1):
                    agents[a_p[k]][1] = agents[a_p[k - 1]][1]
                agents[first][1] = last_goal
    moved = [0] * n
    for i in range(n):
        if agents[i][0] == agents[i][1]:
            continue
        path = G.get_path(agents[i][0], agents[i][1])
        u = path[1]
        j = position(u)
        if j is not None:
            if i != j:
                pj = G.get_path(agents[j][0], agents[j][1])
                if len(pj) >= 2 and pj[1] == agents[i][0]:
                    ev.add("mutual_swap")
                    agents[i][0], agents[j][0] = agents[j][0], agents[i][0]
                    moved[i] += 1
                    moved[j] += 1
        else:
            agents[i][0] = u
            moved[i] += 1
    if max(moved, default=0) >= 2:
        ev.add("double_move")


def to_cells(G, W, ids):
    return [G.id2pos[a][1] * W + G.id2pos[a][0] for a in ids]


def kat_from(name, rows, v_xy, g_xy):
    G = pr.Graph(rows)
    W = len(rows[0])
    agents = [[G.pos2id[tuple(a)], G.pos2id[tuple(b)]] for a, b in zip(v_xy, g_xy)]
    v0 = to_cells(G, W, [a[0] for a in agents])
    g0 = to_cells(G, W, [a[1] for a in agents])
    pr.tswap_step(agents, G)
    v1 = to_cells(G, W, [a[0] for a in agents])
    g1 = to_cells(G, W, [a[1] for a in agents])
    og = OracleGraph(maps.rows_to_array(rows))
    cv, cg = og.step(np.array(v0, dtype=np.uint32), np.array(g0, dtype=np.uint32))
    assert list(cv) == v1 and list(cg) == g1, name
    return {"name": name, "grid": rows, "v": v0, "g": g0, "v_after": v1, "g_after": g1}


def search(event, rows_fn, n_agents, seeds=4000):
    for seed in range(seeds):
        rng = random.Random(seed * 7919 + sum(map(ord, event)))
        rows = rows_fn(seed)
        G = pr.Graph(rows)
        ids = list(range(len(G.id2pos)))
        if len(ids) <= n_agents:
            continue
        rng.shuffle(ids)
        v = ids[:n_agents]
        g = [rng.choice(ids) if rng.random() < 0.8 else v[k] for k in range(n_agents)]
        ev = set()
        instrumented_step([[a, b] for a, b in zip(v, g)], G, ev)
        if event in ev:
            return kat_from(f"{event}_seed{seed}", rows, [G.id2pos[a] for a in v], [G.id2pos[b] for b in g])
    raise RuntimeError(f"no configuration found for {event}")


def main():
    kats = []
    corridor = ["....."]
    # rule 3 by hand: agent 0 -> x=4 blocked by agent 1 sitting on its goal
    kats.append(kat_from("hand_rule3_corridor", corridor, [(0, 0), (1, 0)], [(4, 0), (1, 0)]))
    # rule 4, 2-cycle by hand: agents want each other's cells
    kats.append(kat_from("hand_rule4_pair", corridor, [(1, 0), (2, 0)], [(3, 0), (0, 0)]))
    # rule 4, 4-cycle around a 2x2 block: every goal is the next cell
    kats.append(kat_from("hand_rule4_ring4", ["..", ".."], [(0, 0), (1, 0), (1, 1), (0, 1)],
                         [(1, 0), (1, 1), (0, 1), (0, 0)]))
    # unreachable goal (other component): fallback to the first Manhattan-closer neighbour
    kats.append(kat_from("hand_unreachable_fallback", ["..@..", "..@..", "..@.."], [(1, 1)], [(4, 1)]))
    kats.append(kat_from("hand_unreachable_stay", [".@.", "@@.", "..."], [(0, 0)], [(2, 0)]))
    # duplicate start cells: lowest index occupies the cell
    kats.append(kat_from("hand_duplicates", ["....", "...."], [(0, 0), (0, 0), (1, 0)],
                         [(3, 0), (0, 1), (1, 0)]))
    rnd = lambda s: maps.random_map(7, 7, 0.15, 1000 + s)  # noqa: E731
    openm = lambda s: maps.open_map(5, 5)  # noqa: E731
    for ev, fn, n in [("rule3", rnd, 8), ("rule4_cycle2", openm, 10), ("rule4_cycle3plus", openm, 14),
                      ("clear", openm, 14), ("mutual_swap", rnd, 12), ("double_move", openm, 14),
                      ("mutual_swap", openm, 16)]:
        kats.append(search(ev, fn, n))
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump({"tag": "std-heap-model v1", "kats": kats}, f, indent=0)
    print("\n".join(k["name"] for k in kats))


if __name__ == "__main__":
    main()
