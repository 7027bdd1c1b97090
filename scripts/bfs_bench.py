"""K1 micro-bench: den520d-like 256x257 cave (BASELINE configs[3]), G distinct goals, tables into a
device buffer (the bench's `bfs` leg without the rest). Prints ms/launch, GB/s and HBM fraction
(algorithmic bytes: 2*W*H + ceil(W*H/8) per goal). TSW_BFS_PROF=1 adds the in-kernel cycle split."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from p2p_distributed_tswap_amd import Planner, maps  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
mapname = sys.argv[3] if len(sys.argv) > 3 else "cave"
torch.cuda.init()
if mapname == "cave":
    rows = maps.cave_map(256, 257, 0x520D)
elif mapname == "sort":
    rows = maps.sortation_map(1024, 1024)
else:
    rows = maps.warehouse_map(170, 84, 0x170084)
h, w = len(rows), len(rows[0])
cells = maps.rows_to_array(rows).reshape(-1)
free = np.flatnonzero(cells != ord("@")).astype(np.uint32)
rng = np.random.default_rng(0x520D)
goals = np.sort(rng.choice(free, size=min(G, free.size), replace=False)).astype(np.uint32)
p = Planner(rows)
out = torch.empty((goals.size, w * h), dtype=torch.int16, device="cuda")
p.dist_tables_device(goals, out.data_ptr())
p.reset_stats()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(reps):
    p.dist_tables_device(goals, out.data_ptr())
torch.cuda.synchronize()
wall = (time.perf_counter() - t) / reps
st = p.stats()
ms = st["bfs_ms"] / max(st["bfs_launches"], 1)
bpg = 2 * w * h + (w * h + 7) // 8
gbs = goals.size * bpg / (ms * 1e-3) / 1e9
print(f"{mapname} {w}x{h} goals {goals.size}: kernel {ms:.3f} ms  wall {wall*1e3:.3f} ms  "
      f"{gbs:.1f} GB/s  frac {gbs/8000:.4f}  cells/s {goals.size*w*h/(ms*1e-3):.3e}", flush=True)
