"""K1 A/B probe (diagnostic build): den520d 10k goals with TSW_BFS_KERNEL=<kernel> TSW_BFS_PROF=1 —
ms per launch and the in-kernel cycle split (bfs / decode cycles per goal, levels)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from p2p_distributed_tswap_amd import Planner, maps  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from test_gpu_bfs import _DevBuf  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
mapname = sys.argv[2] if len(sys.argv) > 2 else "cave"
rows = maps.cave_map(256, 257, 0x520D) if mapname == "cave" else maps.warehouse_map(170, 84, 0x170084)
h, w = len(rows), len(rows[0])
cells = maps.rows_to_array(rows).reshape(-1)
free = np.flatnonzero(cells != ord("@")).astype(np.uint32)
goals = np.sort(np.random.default_rng(0x520D).choice(free, size=min(G, free.size), replace=False)).astype(np.uint32)
buf = _DevBuf(goals.size * w * h * 2)
with Planner(rows, diag=True) as p:
    for rep in range(3):
        p.reset_stats()
        t = time.perf_counter()
        p.dist_tables_device(goals, buf.ptr.value)
        wall = time.perf_counter() - t
        st = p.stats()
        ms = st["bfs_ms"]
        print(f"{os.environ.get('TSW_BFS_KERNEL', 'auto')} {mapname} goals {goals.size}: {ms:.3f} ms "
              f"({goals.size * (2 * w * h + (w * h + 7) // 8) / ms / 1e6:.0f} GB/s) wall {wall*1e3:.1f} ms", flush=True)
