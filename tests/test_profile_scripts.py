"""CPU tests of the profile summarisers whose numbers the round's documents quote: scripts/k1_sq.py (K1
instructions per goal-level) and scripts/warm_split.py (planner / worker split of the coop dispatch's
PMC bytes, with the no-chain planner pass). Synthetic rocprofv3 counter CSVs with known values."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]


def _csv(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=FIELDS)
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _row(did, kernel, counter, value, t0=0, t1=1_000_000):
    return {"Dispatch_Id": did, "Kernel_Name": kernel, "Counter_Name": counter, "Counter_Value": value,
            "Start_Timestamp": t0, "End_Timestamp": t1}


def test_k1_sq_per_goal_level(tmp_path):
    k = "void tsw::k_bfs_blk<false, false>(tsw::BlkBfsArgs)"
    rows = []
    for did in (1, 2):  # two 10k-goal launches with identical counts
        rows += [_row(did, k, "SQ_INSTS_VALU", 10000 * 372.5 * 300), _row(did, k, "SQ_INSTS_SALU", 10000 * 372.5 * 100),
                 _row(did, k, "SQ_INSTS_LDS", 10000 * 372.5 * 25), _row(did, k, "SQ_INSTS_SMEM", 0),
                 _row(did, k, "SQ_WAVES", 3072), _row(did, k, "SQ_WAVE_CYCLES", 10000 * 400000)]
    rows.append(_row(3, k, "SQ_WAVES", 12))  # a small launch (another workload) is ignored
    _csv(str(tmp_path / "sq"), rows)
    out = tmp_path / "k1.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "k1_sq.py"), str(tmp_path / "sq"), str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    d = json.loads(out.read_text())
    assert d["dispatches"] == 2
    assert d["per_goal_level"]["SQ_INSTS_VALU"] == 300.0
    assert d["insts_per_goal_level"] == 425.0
    assert d["wave_cycles_per_goal"] == 1600000  # quad-cycles x 4


def test_warm_split_planner_from_no_chain_pass(tmp_path):
    k = "void tsw::k_plan<true, true, true, false>(tsw::PlanArgs, tsw::WorkerArgs)"
    KB = 1024.0

    def passes(name, fetch_kb, write_kb):  # dispatches: warm-up, cold, warm
        _csv(str(tmp_path / f"{name}_fetch"), [_row(i, k, "FETCH_SIZE", v) for i, v in enumerate(fetch_kb)])
        _csv(str(tmp_path / f"{name}_write"), [_row(i, k, "WRITE_SIZE", v) for i, v in enumerate(write_kb)])

    steps = 2001000
    passes("warm", [1, 500000, 200000], [1, 300000, 100000])
    passes("nc", [1, 900000, 50000], [1, 700000, 60000])
    for name, chains in (("warm", True), ("nc", False)):
        (tmp_path / f"{name}.json").write_text(json.dumps({
            "config": "c3_warehouse_170x84", "build_id": "abc", "task_chains": chains, "cold_queries": [1000],
            "agent_steps": steps}) + "\n")
    out = tmp_path / "ws.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "warm_split.py"),
                        str(tmp_path / "warm_fetch"), str(tmp_path / "warm_write"), str(tmp_path / "warm.json"), str(out),
                        str(tmp_path / "nc_fetch"), str(tmp_path / "nc_write"), str(tmp_path / "nc.json")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    d = json.loads(out.read_text())
    cold = (2 * 500000 + 300000) * KB
    warm = (2 * 200000 + 100000) * KB
    planner = (2 * 50000 + 60000) * KB
    assert abs(d["workers_bytes_per_query"] - (cold - warm) / 1000) < 1.0
    assert abs(d["planner_bytes_per_agent_step"] - planner / steps) < 0.1
    assert abs(d["warm_dispatch_bytes_per_agent_step"] - warm / steps) < 0.1
    assert "without task chains" in d["planner_bytes_source"]
