"""bench.py's N > 1 path end to end: two ranks launched the way the driver launches its scaling runs
(`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`), here over gloo with both
ranks on the one visible GPU (the builder has no multi-GPU box; the driver's node runs use RCCL). The
replica plans, the goal-sharded K1 build + all-gather and the rank-0 JSON line must all go through:
round 5 found the line failing to serialise at N > 1 (a local shadowed the build id)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo_one_gpu():
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "0", "--dist-backend", "gloo", "--no-cpu"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["value"] > 0
    assert isinstance(d["build_id"], str)
    assert d["config"]["timesteps_moving"] >= 1990
    assert d["bfs"]["sharded_build_allgather_ms"] is not None
    # the same-N local build the sharded form is compared against
    assert d["bfs"]["local_build_all_goals_ms"] is not None
