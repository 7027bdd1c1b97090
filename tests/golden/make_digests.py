"""Per-timestep digests of full-horizon oracle plans too large to commit as raw fixtures.

For each instance: run the CPU oracle (oracle/tswap_oracle.c, the faithful restatement of
tswap.rs:39-394 — "parity unpinned" against the Rust binary) and record, for every
timestep t, the first 16 hex digits of sha1(records[:, t] || goals[:, t]) (records packed
x | y<<16 | state<<32 as u64, goals as u32 cell ids, agent order). The GPU test recomputes the same
digests from its own plan: equal digests at every t <=> bit-exact plans (up to sha1 collisions),
and the first differing t localises a divergence.

Usage: python tests/golden/make_digests.py            (writes tests/golden/digests.json)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

from p2p_distributed_tswap_amd import maps  # noqa: E402


def step_digests(rec: np.ndarray, goals: np.ndarray) -> list:
    rec = np.ascontiguousarray(rec, dtype=np.uint64)
    goals = np.ascontiguousarray(goals, dtype=np.uint32)
    out = []
    for t in range(rec.shape[1]):
        h = hashlib.sha1(np.ascontiguousarray(rec[:, t]).tobytes())
        h.update(np.ascontiguousarray(goals[:, t]).tobytes())
        out.append(h.hexdigest()[:16])
    return out


# name -> (rows, starts, tasks, max_t)
def instances():
    return {
        "c3_full": lambda: (*maps.config_instance("c3_warehouse_170x84"), 2000),
        "c5_prefix": lambda: (*maps.c5_instance(), 6),
    }


def main(names=None):
    from oracle import OracleGraph

    path = os.path.join(HERE, "digests.json")
    have = json.load(open(path)) if os.path.exists(path) else {}
    for name, fac in instances().items():
        if names and name not in names:
            continue
        rows, starts, tasks, max_t = fac()
        og = OracleGraph(maps.rows_to_array(rows))
        t0 = time.time()
        rec, goals = og.mapd(starts, tasks, max_t, trace_goals=True)
        dt = time.time() - t0
        have[name] = {"agents": int(starts.shape[0]), "tasks": int(tasks.shape[0]), "max_t": max_t,
                      "T": int(rec.shape[1]), "oracle_s": round(dt, 1), "model": "std-heap-model v1",
                      "digests": step_digests(rec, goals)}
        print(f"{name}: T={rec.shape[1]} in {dt:.1f} s", flush=True)
        with open(path, "w") as f:
            json.dump(have, f, indent=0)


if __name__ == "__main__":
    main(sys.argv[1:] or None)
